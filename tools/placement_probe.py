#!/usr/bin/env python3
"""Streaming read / write speed of snapshot-sized allocations, buffer by buffer.

tools/direction_probe.py found the d3q27 fp64 512^3 collide running 9.5-11.8 ms per
dispatch depending only on where its two 29 GB snapshots landed, and that the slow
direction is the one WRITING into a "slow" buffer (27-stream non-temporal write of one
buffer: 4.3-5.6 ms from one allocation to the next, reads 4.5-4.8 ms).  This probe
allocates K such buffers at once (so each gets its own physical pages) and times, for
each, the 27-stream read and write of csrc/bench/stream_copy.hip — the numbers a
placement-aware allocator would rank candidates by.  Run it under
``rocprofv3 --pmc <counters>`` to get translation / channel counters per buffer (the
dispatches are in buffer order: K reads, then K writes, `reps` times).

    python tools/placement_probe.py [--k 4] [--gib 29] [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--n", type=int, default=512, help="field plane edge (elements n^3)")
    ap.add_argument("--fields", type=int, default=27)
    ap.add_argument("--elem", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", default="torch", help="torch | hip | contiguous | vmm (tclb_amd.ops.device)")
    a = ap.parse_args()
    from tclb_amd.build import bench_lib_path
    fn = ctypes.CDLL(bench_lib_path("stream_copy")).tclb_stream_rw
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    fs = a.n ** 3
    nbytes = a.fields * fs * a.elem
    dt = torch.float64 if a.elem == 8 else torch.float32
    bufs = []
    for _ in range(a.k):
        if a.mode == "torch":
            b = torch.zeros(a.fields * fs, dtype=dt, device=dev)
        else:
            from tclb_amd.ops.device import snap_buffer
            b = snap_buffer(nbytes, a.mode, dev).view(dt)
            b.zero_()
        bufs.append(b)
    sink = torch.zeros(16, dtype=dt, device=dev)
    s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    times = {i: {"r": [], "w": []} for i in range(a.k)}
    for _ in range(a.reps):
        for op, key in ((1, "r"), (2, "w")):
            for i, b in enumerate(bufs):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                src, dst = (b.data_ptr(), sink.data_ptr()) if op == 1 else (0, b.data_ptr())
                e0.record()
                assert fn(src, dst, fs, fs, a.fields, a.elem, op, s) == 0
                e1.record()
                torch.cuda.synchronize()
                times[i][key].append(e0.elapsed_time(e1))
    for i, b in enumerate(bufs):
        r, w = min(times[i]["r"]), min(times[i]["w"])
        print(json.dumps({"buffer": i, "ptr": hex(b.data_ptr()), "bytes": nbytes, "read_ms": round(r, 4),
                          "write_ms": round(w, 4), "read_TBps": round(nbytes / r / 1e9, 3),
                          "write_TBps": round(nbytes / w / 1e9, 3), "mode": a.mode}), flush=True)


if __name__ == "__main__":
    main()
