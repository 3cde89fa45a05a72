"""Multi-process runs on ONE MI355X: 2 and 4 processes share device 0 and exchange halos
(and the particle forces) through the native loop's IPC transport — each rank pulls its
neighbours' packed send buffers from their memory, ordered by counters in uncached
shared memory (csrc/device/dist.hip xstart_ipc).  RCCL refuses two ranks on one device,
so this is the one way a single-GPU box runs the cross-process path: communicator-free
set-up (handles through gloo), issue order, the pulls, the all-reduce and the waits.
N processes must reproduce one rank bit for bit (d3q27, slab and Y x Z grid); the particle
case to rounding (its force sums are atomic).  Reference: every MPI rank exchanging its
margins with real peers, src/Lattice.cu.Rt:327-389,466-533."""
import json
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(world, args, limit=240):
    """world worker processes (spawned interpreters, nothing inherited from this one's GPU
    state), joined with a deadline: a hang kills them and fails the test"""
    import torch.multiprocessing as mp
    import ipc_worker
    ctx = mp.start_processes(ipc_worker.worker, args=(world, _port(), *args), nprocs=world, start_method="spawn",
                             join=False)
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > limit:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail(f"IPC ranks did not finish within {limit} s")


def _ref(case, shape, steps):
    import ipc_worker
    from tclb_amd.parallel.comm import LoopbackComm
    lat = ipc_worker.run_case(case, shape, steps, LoopbackComm())
    torch.cuda.synchronize()
    return lat


@pytest.mark.parametrize("shape,world,grid", [
    ((32, 16, 24), 2, None),        # prev == next: both directions to one peer
    ((32, 16, 24), 4, None),
    ((32, 16, 16), 4, (2, 2)),      # Y x Z grid: z pulls, then staged y rows (edges)
])
def test_ipc_ranks_match_single(tmp_path, shape, world, grid):
    steps = 6
    ref = _ref("d3q27", shape, steps)
    out = str(tmp_path / "full.npy")
    _spawn(world, ("d3q27", shape, steps, out, grid))
    meta = json.load(open(out + ".json"))
    assert meta["transport"] == ["ipc"] * world
    assert meta["axis"] == (3 if grid else 2)
    full = np.load(out)
    r = ref.fields_interior().cpu().numpy()
    assert np.array_equal(full, r), float(np.abs(full - r).max())
    for k, v in ref.globals.items():
        assert abs(meta["globals"][k] - v) <= 1e-11 * (1 + abs(v)), k


def test_ipc_particle_allreduce(tmp_path):
    """the part256 case at 64^3 on 2 processes: particle forces summed over the ranks by
    the IPC all-reduce inside the native loop, the rigid step on every rank"""
    shape, steps = (64, 64, 64), 10
    ref = _ref("part", shape, steps)
    out = str(tmp_path / "full.npy")
    _spawn(2, ("part", shape, steps, out))
    meta = json.load(open(out + ".json"))
    assert meta["transport"] == ["ipc", "ipc"]
    full = np.load(out)
    r = ref.fields_interior().cpu().numpy()
    assert np.abs(full - r).max() <= 1e-12 * np.abs(r).max()
    ps = ref.particles
    for key, val in (("x", ps.x), ("v", ps.v), ("force", ps.force)):
        a, b = np.asarray(meta["part"][key]), np.asarray(val, dtype=float)
        assert np.allclose(a, b, rtol=1e-9, atol=1e-14), (key, a, b)
    assert float(np.abs(np.asarray(ps.force)).max()) > 0.0      # the coupling acts


def test_ipc_particles_cross_ranks(tmp_path):
    """4 processes on one GPU: three spheres straddle, wrap and cross the z-slab cuts
    (tests/dist_worker.py particle_case); halos and the force all-reduce through IPC
    inside the native loop equal one rank to rounding (atomic force sums)"""
    shape, steps = (32, 32, 48), 8
    ref = _ref("part3", shape, steps)
    out = str(tmp_path / "full.npy")
    _spawn(4, ("part3", shape, steps, out))
    meta = json.load(open(out + ".json"))
    assert meta["transport"] == ["ipc"] * 4
    full = np.load(out)
    r = ref.fields_interior().cpu().numpy()
    assert np.abs(full - r).max() <= 1e-12 * np.abs(r).max()
    ps = ref.particles
    for key, val in (("x", ps.x), ("v", ps.v), ("force", ps.force)):
        a, b = np.asarray(meta["part"][key]), np.asarray(val, dtype=float)
        assert np.allclose(a, b, rtol=1e-9, atol=1e-13), (key, a, b)
    assert float(np.abs(np.asarray(ps.force)).max()) > 0.0


def test_ipc_loopback_one_rank(monkeypatch):
    """one process pulling from itself through the same IPC code (no peer to map) equals
    the plain one-rank lattice bit for bit"""
    import ipc_worker
    from tclb_amd.parallel.comm import LoopbackComm
    shape, steps = (32, 16, 24), 6
    ref = _ref("d3q27", shape, steps)
    monkeypatch.setenv("TCLB_DIST_TRANSPORT", "ipc")
    lat = ipc_worker.run_case("d3q27", shape, steps, LoopbackComm(exercise_dist_path=True))
    torch.cuda.synchronize()
    assert lat._dist is not None and lat._dist.transport == "ipc"
    lat._dist.wait()
    assert torch.equal(lat.fields_interior(), ref.fields_interior())


def test_ipc_dead_peer_times_out(tmp_path):
    """a peer that stops stepping: the survivor's bounded waits time out (3 s, later waits
    return at once), the wait after the steps raises NativeDistError, and the GPU queue
    drains — no hang (a dead peer must raise, not hang the rank)"""
    import torch.multiprocessing as mp
    import ipc_worker
    out = str(tmp_path / "dead.json")
    ctx = mp.start_processes(ipc_worker.worker_dead_peer, args=(2, _port(), out), nprocs=2, start_method="spawn",
                             join=False)
    t0 = time.time()
    while not ctx.join(timeout=5):
        if time.time() - t0 > 180:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("the surviving rank hung")
    res = json.load(open(out))
    assert "timed out" in res["error"], res
    assert res["seconds"] < 60, res
