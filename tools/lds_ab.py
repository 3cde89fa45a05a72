#!/usr/bin/env python3
"""LDS A/B of the 27-point stencil read pattern (csrc/bench/lds_stencil.hip).

Mode 0 reads the 27 neighbours straight from global memory (the model kernels' pattern,
L2 serves the x/y/z +-1 lines); mode 1 stages (64+2) x (4+2) tiles of a 3-plane ring
through LDS while marching 16 z planes per work-group.  Both write the same weighted
sum; the outputs are compared with each other and with a torch.roll reference.

    python tools/lds_ab.py --n 384 --reps 20
Prints one JSON line per mode: ms per sweep, GLUPS and the effective bandwidth of the
compulsory traffic (8 B read + 8 B written per node).  Run under tools/counters.py for
the HBM bytes each mode really moves.
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.build import bench_lib_path  # noqa: E402


def reference(phi: torch.Tensor) -> torch.Tensor:
    w = {0: -3.5, 1: 2.0 / 9.0, 2: 1.0 / 18.0, 3: 1.0 / 72.0}
    out = torch.zeros_like(phi)
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                out += w[dx * dx + dy * dy + dz * dz] * torch.roll(phi, shifts=(-dz, -dy, -dx), dims=(0, 1, 2))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=384)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    path = bench_lib_path("lds_stencil")
    if not os.path.exists(path):
        raise SystemExit(f"{path} missing: build it first (python -c 'from tclb_amd import build; build.build_bench_libs()')")
    if a.n % 64 or a.n % 16:
        raise SystemExit("--n must be a multiple of 64")
    lib = ctypes.CDLL(path)
    fn = lib.tclb_lds_ab_run
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.POINTER(ctypes.c_float)]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    phi = torch.rand((a.n, a.n, a.n), dtype=torch.float64, device=dev, generator=g)
    outs = [torch.empty_like(phi), torch.empty_like(phi)]
    stream = torch.cuda.current_stream(dev).cuda_stream
    ref = reference(phi)
    torch.cuda.synchronize()
    nodes = a.n ** 3
    best = {0: 1e30, 1: 1e30}
    for _ in range(a.rounds):                       # interleaved rounds
        for mode in (0, 1):
            ms = ctypes.c_float()
            rc = fn(mode, phi.data_ptr(), outs[mode].data_ptr(), a.n, a.reps, ctypes.c_void_p(stream), ctypes.byref(ms))
            if rc != 0:
                raise SystemExit(f"mode {mode}: error {rc}")
            best[mode] = min(best[mode], ms.value)
    torch.cuda.synchronize()
    err_ab = (outs[0] - outs[1]).abs().max().item()
    err_ref = (outs[0] - ref).abs().max().item()
    for mode, label in ((0, "global (L2-cached 27 loads)"), (1, "LDS tile 64x4, 16-plane z-march")):
        ms = best[mode]
        print(json.dumps({"mode": mode, "kernel": label, "n": a.n, "ms": round(ms, 4),
                          "GLUPS": round(nodes / ms / 1e6, 2), "compulsory_TBps": round(16 * nodes / ms / 1e9, 3),
                          "max_diff_vs_other": err_ab, "max_diff_vs_torch": err_ref}), flush=True)
    assert err_ab < 1e-12 and err_ref < 1e-12


if __name__ == "__main__":
    main()
