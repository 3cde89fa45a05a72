"""The bench.py contract the driver relies on (task spec): under torch.distributed.run
with N ranks, rank 0 prints one JSON line with the whole-job value, n_gpus = N, the
timed step count and the metric named in BASELINE.json.  Exercised here on the CPU with
gloo and 2 ranks (the same code path as RCCL ranks, the device aside)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(nproc, port):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--cpu", "--shape", "32,16,16", "--steps", "3", "--warmup", "1", "--gpus", str(nproc)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_two_ranks_json_line():
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    out = _run(2, 29611)
    assert out["n_gpus"] == 2 and out["steps"] == 3 and out["warmup"] == 1
    assert out["iterations_timed"] == 3            # the window holds exactly `steps` iterations
    assert out["value"] > 0 and out["higher_is_better"] is True
    assert out["config"]["parallelism"] == "zslab2"
    assert out["globals_finite"] is True
    assert out["loop"] == "native-dist/callback" and out["checks"]["z_invariant"]
    metric = base.get("metric") or base.get("headline", {}).get("metric")
    if metric:
        assert out["metric"] == metric


def test_bench_eight_ranks_like_the_scaling_run():
    """the driver's 8-GPU command line (torch.distributed.run, 8 ranks, --gpus 8) on gloo
    ranks: 32 z planes over 8 slabs of 4, every physics check on, one JSON line"""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=8",
           "--master-addr", "127.0.0.1", "--master-port", "29617", os.path.join(ROOT, "bench.py"),
           "--cpu", "--size", "32", "--steps", "3", "--warmup", "1", "--gpus", "8"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "zslab8"
    assert out["config"]["lattice"] == [32, 32, 32] and out["scaling"] == "strong"
    assert all(out["checks"][k] for k in ("mass_ok", "z_invariant", "x_invariant", "collides"))


def test_bench_spawns_its_own_ranks():
    """--gpus N without a launcher starts N ranks itself (torch.distributed.run as a child
    process): the line reports n_gpus = N, never a silent 1-rank run; the ranks step
    through the native multi-rank loop"""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--shape", "32,16,16",
           "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "zslab2"
    assert out["loop"] == "native-dist/callback"
    assert all(out["checks"][k] for k in ("globals_finite", "mass_ok", "z_invariant", "x_invariant"))


def test_bench_rejects_rank_count_mismatch():
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "3", "--shape", "32,16,16",
           "--steps", "1", "--warmup", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_bench_window_holds_exactly_steps_iterations():
    """one rank: the timed window runs exactly --steps iterations (steps - 1 plain, the last
    with globals), so MLUPS = nodes * steps / window is not under-reported (round-4 bug:
    steps + 1 iterations over a steps divisor)"""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    for steps in (1, 4):
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--shape", "32,16,16",
               "--steps", str(steps), "--warmup", "1"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        assert out["iterations_timed"] == steps and out["steps"] == steps
        window = 32 * 16 * 16 * steps / (out["value"] * 1e6)          # seconds, from the MLUPS
        assert abs(out["ms_per_step"] * steps / 1e3 - window) <= 0.01 * window + 1e-7


def test_bench_rank_failure_ends_the_job():
    """one rank of `bench.py --gpus 2` dies (TCLB_BENCH_FAIL_RANK=1) while rank 0 waits in
    a collective: the launcher tears the job down and exits non-zero in bounded time, with
    no JSON line (a failed run reports nothing rather than a number)"""
    import time
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", TCLB_BENCH_FAIL_RANK="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--gpus", "2", "--shape", "32,16,16",
           "--steps", "3", "--warmup", "1"]
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert time.time() - t0 < 240
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "failing on purpose" in r.stderr
