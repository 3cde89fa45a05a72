#!/usr/bin/env python3
"""Per-dispatch timing of the headline stage by snapshot direction (A->B vs B->A).

The round-4 traces show the d3q27 fp64 512^3 collide alternating between two times on
some boxes (11.28 / 9.95 ms on one, 10.11 / 10.36 on another): one snapshot direction is
slower.  This probe times every dispatch of the plain stage separately (an event pair
around each single-step launch; the queue stays full because the host never waits) and
reports the even (snaps[0] -> snaps[1]) and odd (snaps[1] -> snaps[0]) medians for
several placements of the A/B pair:

  default           the two snapshots as Lattice allocates them (two torch allocations)
  swap              the same buffers with the roles exchanged (does the slow direction
                    follow a buffer?)
  one:<off>         both snapshots carved from ONE allocation, B starting <off> bytes
                    after the end of A (0, 4 KiB, 64 KiB, 2 MiB + 4 KiB, ...)
  fpad:<elems>      TCLB_FIELD_PAD (field planes staggered by <elems> elements)
  alloc:<mode>      each snapshot from the native allocator (csrc/device/snapalloc.hip):
                    hip, contiguous (one physically contiguous range) or vmm
  pair:<mode>       one native range holding both snapshots

and, for each placement, the 27-stream copy A->B and B->A of csrc/bench/stream_copy.hip
(the kernel's memory pattern without the arithmetic): if the copy shows the same
asymmetry, it is placement in the memory system, not the kernel.

    python tools/direction_probe.py [--n 512] [--steps 12] [--variants default,swap,one:0,...]
Prints one JSON line per variant.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _copy_fn():
    from tclb_amd.build import bench_lib_path
    p = bench_lib_path("stream_copy")
    if not os.path.exists(p):
        return None
    fn = ctypes.CDLL(p).tclb_stream_copy
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p]
    return fn


def _rw_fn():
    from tclb_amd.build import bench_lib_path
    fn = ctypes.CDLL(bench_lib_path("stream_copy")).tclb_stream_rw
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p]
    return fn


def time_rw(lat, reps: int = 4):
    """27-stream read-only and write-only time of each snapshot (ms): rA, rB, wA, wB"""
    fn = _rw_fn()
    s = ctypes.c_void_p(torch.cuda.current_stream(lat.device).cuda_stream)
    es = lat.snaps[0].element_size()
    sink = torch.zeros(16, dtype=lat.sdtype, device=lat.device)
    out = []
    for op in (1, 2):
        for buf in lat.snaps:
            src, dst = (buf.data_ptr(), sink.data_ptr()) if op == 1 else (0, buf.data_ptr())
            assert fn(src, dst, lat.fs, lat.fs, lat.nf, es, op, s) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn(src, dst, lat.fs, lat.fs, lat.nf, es, op, s)
            e1.record()
            torch.cuda.synchronize()
            out.append(round(e0.elapsed_time(e1) / reps, 4))
    return out


def make_lattice(n: int, model: str, precision: str, fpad: int = 0):
    import bench
    from tclb_amd.lattice import Lattice
    if fpad:
        os.environ["TCLB_FIELD_PAD"] = str(fpad)
    else:
        os.environ.pop("TCLB_FIELD_PAD", None)
    lat = Lattice(model, (n, n, n), device=torch.device("cuda", 0), precision=precision)
    os.environ.pop("TCLB_FIELD_PAD", None)
    lat.set_flags(bench.channel_flags(lat))
    lat.set_setting("nu", 0.02)
    lat.set_setting("ForceX", 1e-6)
    return lat


def carve_one(lat, off_bytes: int):
    """replace the A/B pair by two views of one allocation, B at A + size + off"""
    es = lat.snaps[0].element_size()
    per = lat.nf * lat.fs
    assert off_bytes % es == 0
    off = off_bytes // es
    lat.snaps = []
    torch.cuda.empty_cache()
    buf = torch.zeros(2 * per + off, dtype=lat.sdtype, device=lat.device)
    shape = (lat.nf, lat.NZ, lat.NY, lat.px)
    stride = (lat.fs, lat.NY * lat.px, lat.px, 1)
    lat.snaps = [buf.as_strided(shape, stride, 0), buf.as_strided(shape, stride, per + off)]
    lat._probe_buf = buf


def native_alloc(lat, mode: str, pair: bool, off_bytes: int = 0):
    """snapshots from the native allocator (tclb_amd/ops/device.py snap_buffer): one range
    per snapshot, or (pair) one range holding both, B at A + size + off"""
    from tclb_amd.ops.device import snap_buffer
    es = lat.snaps[0].element_size()
    per = lat.nf * lat.fs
    lat.snaps = []
    torch.cuda.empty_cache()
    shape = (lat.nf, lat.NZ, lat.NY, lat.px)
    stride = (lat.fs, lat.NY * lat.px, lat.px, 1)
    if pair:
        off = off_bytes // es
        buf = snap_buffer((2 * per + off) * es, mode, lat.device).view(lat.sdtype)
        buf.zero_()
        lat.snaps = [buf.as_strided(shape, stride, 0), buf.as_strided(shape, stride, per + off)]
        lat._probe_buf = buf
    else:
        bufs = [snap_buffer(per * es, mode, lat.device).view(lat.sdtype) for _ in range(2)]
        for b in bufs:
            b.zero_()
        lat.snaps = [b.as_strided(shape, stride, 0) for b in bufs]
        lat._probe_buf = bufs


def time_dispatches(lat, steps: int):
    lat.cur = 0
    lat.init()
    lat.iterate(2, glob_last=False)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    dirs = []
    ev[0].record()
    for i in range(steps):
        dirs.append(lat.cur)
        lat.iterate(1, glob_last=False)
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(steps)]
    a2b = [t for t, d in zip(ms, dirs) if d == 0]
    b2a = [t for t, d in zip(ms, dirs) if d == 1]
    return ms, statistics.median(a2b), statistics.median(b2a)


def time_copy(fn, lat, reps: int = 6):
    if fn is None:
        return None, None
    s = ctypes.c_void_p(torch.cuda.current_stream(lat.device).cuda_stream)
    es = lat.snaps[0].element_size()
    out = []
    for src, dst in ((lat.snaps[0], lat.snaps[1]), (lat.snaps[1], lat.snaps[0])):
        assert fn(src.data_ptr(), dst.data_ptr(), lat.fs, lat.fs, lat.nf, es, s) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn(src.data_ptr(), dst.data_ptr(), lat.fs, lat.fs, lat.nf, es, s)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return out[0], out[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--model", default="d3q27")
    ap.add_argument("--precision", default="double")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--variants", default="default,swap,one:0,one:4096,one:65536,one:2101248,fpad:512")
    ap.add_argument("--repeat", type=int, default=1, help="run the variant list this many times")
    ap.add_argument("--detail", action="store_true",
                    help="also time 27-stream read-only / write-only per snapshot and the tile-window "
                         "maps --splits on the same placement")
    ap.add_argument("--splits", default="0,1,2,3,4,5", help="log2 tile windows of --detail")
    a = ap.parse_args()
    a.splits = [int(k) for k in a.splits.split(",")]
    fn = _copy_fn()
    nodes = a.n ** 3
    for v in a.variants.split(",") * a.repeat:
        kind, _, arg = v.partition(":")
        lat = make_lattice(a.n, a.model, a.precision, fpad=int(arg) if kind == "fpad" else 0)
        if kind == "swap":
            lat.snaps = [lat.snaps[1], lat.snaps[0]]
        elif kind == "one":
            carve_one(lat, int(arg))
        elif kind in ("alloc", "pair"):
            native_alloc(lat, arg, kind == "pair")
        extra = {}
        if a.detail:
            # the rw probe overwrites the snapshots: before the kernel timing (which inits)
            extra["rA_rB_wA_wB_ms"] = time_rw(lat)
            # tile windows (executor_hip.hpp tile_id) on the same placement, interleaved
            for k in a.splits:
                lat.set_tile_split(k)
                _, x_ab, x_ba = time_dispatches(lat, a.steps)
                extra[f"split{k}_A2B_B2A"] = [round(x_ab, 4), round(x_ba, 4)]
            lat.set_tile_split(0)
        ms, m_ab, m_ba = time_dispatches(lat, a.steps)
        c_ab, c_ba = time_copy(fn, lat)
        pa, pb = lat.snaps[0].data_ptr(), lat.snaps[1].data_ptr()
        rec = {"variant": v, "n": a.n, "precision": a.precision, "ptr_A": hex(pa), "ptr_B": hex(pb),
               "B_minus_A": pb - pa, "ms": [round(t, 4) for t in ms], "med_A2B": round(m_ab, 4),
               "med_B2A": round(m_ba, 4), "ratio": round(max(m_ab, m_ba) / min(m_ab, m_ba), 4),
               "mlups_mean": round(nodes / ((m_ab + m_ba) / 2) / 1e3, 1),
               "copy_A2B_ms": None if c_ab is None else round(c_ab, 4),
               "copy_B2A_ms": None if c_ba is None else round(c_ba, 4), **extra}
        print(json.dumps(rec), flush=True)
        del lat
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
