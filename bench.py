#!/usr/bin/env python3
"""Headline benchmark: MLUPS of the d3q27 MRT channel flow at 512^3 (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One process per GPU.  The global lattice is 512^3 (strong scaling) unless --weak,
decomposed in z-slabs with RCCL halo exchange overlapped with the interior kernel.
Geometry: channel (bounce-back walls at y=0 and y=ny-1, reference zone "Channel"),
MRT collision everywhere, body force ForceX; uniform initial state (synthetic case,
as BASELINE.json prescribes).  Each timed step is the full reference iteration
(collide-stream of every node + boundary + halo exchange; globals on the last step
of the window, as Lattice::Iterate does).  Compute and storage precision: fp64
(the reference default, src/configure.ac:208-211) unless --precision names one of the
reduced-storage modes (mixed[-shift]: fp64 compute / fp32 storage, half[-shift]: fp32
compute / fp16 storage; *-shift stores f - w_i, reference --with-storage=...-shift).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from tclb_amd.lattice import Lattice  # noqa: E402
from tclb_amd.ops.abi import PRECISIONS  # noqa: E402
from tclb_amd.parallel.comm import init_distributed_from_env  # noqa: E402
from tclb_amd.utils.guard import collision_check  # noqa: E402

METRIC = "MLUPS (million lattice updates/sec) whole-node, d3q27 512^3, at 1/2/4/8 MI355X"


def channel_flags(lat: Lattice) -> np.ndarray:
    m = lat.model
    mrt = m.node_type("MRT").value
    wall = m.node_type("Wall").value
    nx = lat.shape[0]
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    # global y of local rows (y is never split in 3-D)
    fl[:, lat.gy + 0, :] = wall
    fl[:, lat.gy + lat.shape[1] - 1, :] = wall
    return fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int, argv) -> int:
    """--gpus N without a launcher: start N ranks of this script under
    torch.distributed.run as a child process (nothing here has touched the GPU yet, and
    this process never execs); rank 0's JSON line reaches our stdout through the
    inherited descriptor.  Returns the launcher's exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def total_mass(lat: Lattice, comm) -> float:
    """sum of every population over the lattice, in fp64 (one field at a time; the
    *-shift storage modes keep f - w: the shift is added back per node)"""
    nx, ny, nz = lat.shape
    s = lat.snaps[lat.cur]
    tot = 0.0
    for i in range(lat.nf):
        v = s[i, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx]
        tot += float(v.double().sum().item())
        if lat._shift_t is not None:
            tot += float(lat._shift_t[i, 0, 0, 0].item()) * nx * ny * nz
    return comm.allreduce_scalar(tot, "sum")


def physics_checks(lat: Lattice, comm, mass0: float, precision: str) -> dict:
    """the run is physics, not noise: finite globals; total mass conserved (bounce-back
    walls, periodic x/z, body force); and the channel's x- and z-invariance (uniform init,
    walls only in y) holds bit for bit between the first and last x column and z plane of
    every rank — a high-address fault or a wrong halo would break it"""
    ok_glob = all(np.isfinite(v) for v in lat.globals.values())
    mass1 = total_mass(lat, comm)
    drift = abs(mass1 - mass0) / abs(mass0)
    tol = 1e-10 if precision == "double" else 1e-5
    nx, ny, nz = lat.shape
    s = lat.snaps[lat.cur]
    zinv = bool(torch.equal(s[:, lat.gz, lat.gy:lat.gy + ny, :nx], s[:, lat.gz + nz - 1, lat.gy:lat.gy + ny, :nx]))
    xinv = bool(torch.equal(s[:, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, 0],
                            s[:, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, nx - 1]))
    # the MRT nodes collide (tclb_amd/utils/guard.py: a stream-only run passes the rest)
    g = collision_check(lat)
    coll = comm.allreduce_scalar(0.0 if g["collides"] else 1.0, "max") == 0.0
    zinv = comm.allreduce_scalar(0.0 if zinv else 1.0, "max") == 0.0
    xinv = comm.allreduce_scalar(0.0 if xinv else 1.0, "max") == 0.0
    ok_glob = comm.allreduce_scalar(0.0 if ok_glob else 1.0, "max") == 0.0
    return {"globals_finite": ok_glob, "mass_rel_drift": drift, "mass_ok": bool(np.isfinite(drift) and drift <= tol),
            "z_invariant": zinv, "x_invariant": xinv, "collides": coll, "collision_rel_diff": g["rel_diff"]}


def main():
    argv = sys.argv[1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--model", default="d3q27")
    ap.add_argument("--precision", default="double", choices=list(PRECISIONS))
    ap.add_argument("--weak", action="store_true", help="size^3 per GPU (z-extent x N)")
    ap.add_argument("--shape", default=None, help="explicit global lattice nx,ny,nz (overrides --size)")
    ap.add_argument("--block", default="0,0")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--glob-every-step", action="store_true",
                    help="globals on every step (a <Log Iterations=\"1\">-style run), not only the last")
    ap.add_argument("--loopback-dist", action="store_true",
                    help="1 rank through the multi-rank path (border/interior split + pack/unpack)")
    ap.add_argument("--transport", default=None, choices=["rccl", "copy", "ipc"],
                    help="halo transport of --loopback-dist (rccl: RCCL send/receive to itself)")
    ap.add_argument("--python-loop", action="store_true",
                    help="multi-rank steps from the Python step path instead of the native loop (A/B)")
    a = ap.parse_args()
    ws = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if ws == 0 and a.gpus is not None and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus, argv))
    if ws and a.gpus is not None and a.gpus != ws:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={ws} ranks", file=sys.stderr)
        sys.exit(2)
    if a.transport:
        os.environ["TCLB_DIST_TRANSPORT"] = a.transport
    if a.python_loop:
        os.environ["TCLB_DIST_NATIVE"] = "0"

    use_gpu = torch.cuda.is_available() and not a.cpu
    comm = init_distributed_from_env("cuda" if use_gpu else "cpu")
    if a.loopback_dist and comm.size == 1:
        from tclb_amd.parallel.comm import LoopbackComm
        comm = LoopbackComm(exercise_dist_path=True)
    rank, world = comm.rank, comm.size
    if use_gpu:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    n = a.size
    shape = (n, n, n * world) if a.weak else (n, n, n)
    if a.shape:
        shape = tuple(int(v) for v in a.shape.split(","))
    bx, by = (int(v) for v in a.block.split(","))
    lat = Lattice(a.model, shape, device=device, precision=a.precision, comm=comm, block=(bx, by),
                  overlap=None if not a.no_overlap else False)
    lat.set_flags(channel_flags(lat))
    lat.set_setting("nu", 0.02)
    lat.set_setting("ForceX", 1e-6)
    lat.init()
    mass0 = total_mass(lat, comm)

    def sync():
        if use_gpu:
            torch.cuda.synchronize()
        comm.barrier()

    lat.iterate(a.warmup, glob_last=False)
    if os.environ.get("TCLB_BENCH_FAIL_RANK") == str(rank):
        # failure drill (tests/test_bench_contract.py): this rank dies while the others
        # wait in the barrier below; the launcher must end the job, not hang
        raise SystemExit(f"bench.py: rank {rank} failing on purpose (TCLB_BENCH_FAIL_RANK)")
    sync()
    # host cost of a step on an idle queue: the enqueue time of a few steps (launches,
    # events, RCCL group calls) before the GPU has caught up — outside the timed window
    th = time.perf_counter()
    lat.iterate(4, glob_last=False)
    t_enqueue = (time.perf_counter() - th) / 4
    sync()
    it0 = lat.iter
    t0 = time.perf_counter()
    if a.glob_every_step:
        for _ in range(a.steps):
            lat.iterate(1, glob_last=True)
        t_host = time.perf_counter() - t0
    else:
        # exactly `steps` iterations in the window: steps - 1 plain ones, then the last
        # with the globals integrated (as Lattice::Iterate does on its last iteration)
        if a.steps > 1:
            lat.iterate(a.steps - 1, glob_last=False)
        t_host = time.perf_counter() - t0       # the host's enqueue time of the window
        lat.iterate(1, glob_last=True)
    sync()
    dt = time.perf_counter() - t0
    iters_timed = lat.iter - it0
    if iters_timed != a.steps:
        raise SystemExit(f"bench.py: {iters_timed} iterations in the timed window, expected {a.steps}")
    dt = comm.allreduce_scalar(dt, "max")
    t_host = comm.allreduce_scalar(t_host, "max")
    nodes = shape[0] * shape[1] * shape[2]
    mlups = nodes * a.steps / dt / 1e6
    chk = physics_checks(lat, comm, mass0, a.precision)
    ok = chk["globals_finite"] and chk["mass_ok"] and chk["z_invariant"] and chk["x_invariant"] and chk["collides"]
    if rank == 0:
        es = lat.snaps[0].element_size()
        nf = lat.nf
        bytes_node = 2 * nf * es + (2 if lat.model.flag_bits == 16 else 4)
        out = {
            "metric": METRIC,
            "value": float(f"{mlups:.8g}"),
            "unit": "MLUPS",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if a.weak else "strong",
            "vs_baseline": None,
            "dtype": {"double": "fp64", "float": "fp32", "float-shift": "fp32 (shifted storage)",
                      "mixed": "fp64-compute/fp32-storage", "mixed-shift": "fp64-compute/fp32-shifted-storage",
                      "half": "fp32-compute/fp16-storage",
                      "half-shift": "fp32-compute/fp16-shifted-storage"}[a.precision],
            "data": "synthetic (uniform init, channel walls + body force, random-free)",
            "config": {"model": a.model, "global_batch": nodes, "seq_len": shape[0],
                       "lattice": list(shape), "parallelism": f"zslab{world}" if world > 1 else "single",
                       "device": "cuda" if use_gpu else "cpu"},
            "effective_GBps_per_gpu": round(mlups * bytes_node / 1e3 / world, 1),
            "globals_finite": chk["globals_finite"],
            "checks": chk,
            "iterations_timed": iters_timed,
            "tile_split": lat.tile_split,
            "placement": lat.placement,
            "host_ms_per_step": round(t_host / max(1, a.steps - 1) * 1e3, 4) if not a.glob_every_step else None,
            "host_enqueue_ms_per_step": round(t_enqueue * 1e3, 4),
            "loop": ("native-dist/" + lat._dist.transport) if (lat._dist is not None and lat.comm.distributed) else
                    {"lib": "native", "loop": "native-loop", None: "python"}[lat._native_path("Iteration")],
            "baseline_note": "reference publishes no MLUPS (BASELINE.md); vs_baseline null",
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if not ok:
        print(f"bench.py: physics check failed on this run: {chk}", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
