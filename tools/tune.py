#!/usr/bin/env python3
"""On-device A/B of kernel build variants and launch shapes (interleaved rounds in one
process, per cdna_hip_programming.md rule 24).  Also measures the device copy bandwidth
of one snapshot (torch copy) as the achievable-BW reference on the same GPU."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd import build as B  # noqa: E402
from tclb_amd.lattice import Lattice  # noqa: E402
from tclb_amd.ops import abi  # noqa: E402
from bench import channel_flags  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="d3q27")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--precision", default="double")
    ap.add_argument("--variants", default=",plain,nt,ntld")
    ap.add_argument("--blocks", default="256x1,128x2,64x4,128x1,64x2")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    variants = a.variants.split(",")
    libs = {v: abi.load(a.model, "hip", variant=v) for v in variants}
    n = a.size
    lat = Lattice(a.model, (n, n, n), device=dev, precision=a.precision)
    lat.set_flags(channel_flags(lat))
    lat.set_setting("nu", 0.02)
    lat.set_setting("ForceX", 1e-6)
    lat.init()
    es = 8 if a.precision == "double" else 4
    bpn = 2 * lat.nf * es + 2
    # copy-bandwidth reference
    src, dst = lat.snaps
    for _ in range(3):
        dst.copy_(src)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        dst.copy_(src)
    torch.cuda.synchronize()
    copy_bw = 2 * src.numel() * src.element_size() * 10 / (time.perf_counter() - t) / 1e9
    print(json.dumps({"copy_GBps": round(copy_bw, 1)}), flush=True)
    lat.init()
    res = {}
    for r in range(a.rounds):
        for v in variants:
            for blk in a.blocks.split(","):
                bx, by = (int(x) for x in blk.split("x"))
                lat.lib = libs[v]
                lat._L.block_x, lat._L.block_y = bx, by
                lat.iterate(2, glob_last=False)
                torch.cuda.synchronize()
                t = time.perf_counter()
                lat.iterate(a.steps, glob_last=False)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t) / a.steps
                key = f"{v or 'default'}/{blk}"
                res.setdefault(key, []).append(dt)
                print(json.dumps({"round": r, "cfg": key, "ms": round(dt * 1e3, 3),
                                  "MLUPS": round(n ** 3 / dt / 1e6, 1),
                                  "GBps": round(n ** 3 * bpn / dt / 1e9, 1)}), flush=True)
    print("== summary (median ms, MLUPS, GB/s)")
    for k, v in sorted(res.items(), key=lambda kv: np.median(kv[1])):
        m = float(np.median(v))
        print(f"{k:16s} {m * 1e3:8.3f} ms {n ** 3 / m / 1e6:9.1f} MLUPS {n ** 3 * bpn / m / 1e9:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
