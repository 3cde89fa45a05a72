#!/usr/bin/env python3
"""Cost of the first launch of a kernel instantiation (r06x: a 20-step window that held the
first globals step of the cavity lost ~4 ms).  Times iterate calls on a fresh lattice:
plain steps, then the first and later globals steps, each synchronised.

    python tools/first_launch_probe.py [model] [n]"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.lattice import Lattice  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "auto_d3q19_BGK"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    lat = Lattice(model, (n, n, n), device=torch.device("cuda", 0))
    lat.init()
    torch.cuda.synchronize()

    def t(label, **kw):
        t0 = time.perf_counter()
        lat.iterate(1, **kw)
        torch.cuda.synchronize()
        print(json.dumps({"model": model, "call": label, "ms": round((time.perf_counter() - t0) * 1e3, 3)}), flush=True)

    for i in range(3):
        t(f"plain {i}", glob_last=False)
    for i in range(3):
        t(f"globals {i}", glob_last=True)
    for i in range(2):
        t(f"plain again {i}", glob_last=False)


if __name__ == "__main__":
    main()
