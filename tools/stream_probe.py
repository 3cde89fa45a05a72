#!/usr/bin/env python3
"""Copy ceilings of this box for the snapshot memory pattern (csrc/bench/stream_copy.hip).

The headline d3q27 fp64 bench moves the same bytes on every box, yet boxes differ by up
to ~15 % in MLUPS.  This probe separates the causes: a plain copy of one long array (the
box's copy ceiling), K = 27 streams 512^3 elements apart (the fp64 / fp32 snapshot
pattern: 27 read + 27 written field planes at once), and the same with the field planes
staggered by a pad.  If the 27-stream copy is slower than the one-stream copy on a box,
the many-stream pattern (page translation, channel aliasing) costs there, not the kernel.

    python tools/stream_probe.py [--n 512] [--reps 10]
Prints one JSON line per case (ms per copy, TB/s of read + written bytes).
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.build import bench_lib_path  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512, help="edge of the cubic field plane (elements = n^3)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--pads", default="0,2112", help="stagger of the field planes in elements")
    a = ap.parse_args()
    path = bench_lib_path("stream_copy")
    if not os.path.exists(path):
        raise SystemExit(f"{path} missing: build it first (python -c 'from tclb_amd import build; build.build_bench_libs()')")
    lib = ctypes.CDLL(path)
    fn = lib.tclb_stream_copy
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    plane = a.n ** 3
    pads = [int(p) for p in a.pads.split(",")]
    cases = [("fp64 1 stream (copy ceiling)", torch.float64, 1, 27 * plane, 0)]
    cases += [(f"fp64 27 streams pad {p}", torch.float64, 27, plane, p) for p in pads]
    cases += [(f"fp32 27 streams pad {p}", torch.float32, 27, plane, p) for p in pads]
    best = {}
    for _ in range(a.rounds):
        for label, dt, K, n, pad in cases:
            stride = n + pad
            src = torch.ones(K * stride, dtype=dt, device=dev)
            dst = torch.empty_like(src)
            eb = src.element_size()
            for _w in range(2):
                assert fn(src.data_ptr(), dst.data_ptr(), n, stride, K, eb, ctypes.c_void_p(stream)) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _r in range(a.reps):
                fn(src.data_ptr(), dst.data_ptr(), n, stride, K, eb, ctypes.c_void_p(stream))
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            best[label] = min(best.get(label, 1e30), ms)
            ok = bool(dst[:n].eq(1).all().item()) and bool(dst[(K - 1) * stride:(K - 1) * stride + n].eq(1).all().item())
            assert ok, label
            del src, dst
            torch.cuda.empty_cache()
    for label, dt, K, n, pad in cases:
        ms = best[label]
        nbytes = 2 * K * n * torch.tensor([], dtype=dt).element_size()
        print(json.dumps({"case": label, "streams": K, "elements_per_stream": n, "pad": pad, "ms": round(ms, 4),
                          "TBps": round(nbytes / ms / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
