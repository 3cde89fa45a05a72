#!/usr/bin/env python3
"""Host overhead per step on a tiny lattice (launch-bound regime): d2q9 64x8, iterate(n)
through the native multi-step loop and through the per-step Python path."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.lattice import Lattice  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="d2q9")
    ap.add_argument("--shape", default="64,8,1")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()
    shape = tuple(int(v) for v in a.shape.split(","))
    for native in (True, False):
        lat = Lattice(a.model, shape, device=torch.device(a.device), native_loop=native)
        m = lat.model
        lat.set_flags(np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint16))
        lat.init()
        lat.iterate(10, glob_last=False)
        if a.device == "cuda":
            torch.cuda.synchronize()
        t = time.perf_counter()
        lat.iterate(a.steps, glob_last=False)
        if a.device == "cuda":
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.steps
        print(json.dumps({"model": a.model, "shape": shape, "device": a.device, "native_loop": native,
                          "us_per_step": round(dt * 1e6, 2),
                          "MLUPS": round(shape[0] * shape[1] * shape[2] / dt / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
