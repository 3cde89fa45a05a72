#!/usr/bin/env python3
"""The part256 force stage with the particle changed (tools/bench_configs.py part256):
radius (default n/16) and position, to separate the cost of the nodes a particle covers
from the whole-lattice pass (profiles/README.md r06k-l).  Run under rocprofv3 --kernel-trace.

    python tools/calcf_probe.py --radius 2 --steps 20
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.lattice import Lattice  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--radius", type=float, default=0.0, help="0: n/16 as part256")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--nparticles", type=int, default=1)
    a = ap.parse_args()
    from tclb_amd.particles import SimplePart
    n = a.n
    shape = (n, n, n)
    lat = Lattice("auto_d3q19_part", shape, device=torch.device("cuda", 0))
    m = lat.model
    lat.set_flags(np.full((lat.NZ, lat.NY, n), m.node_type("MRT").value, dtype=np.uint32))
    lat.set_setting("Viscosity", 0.05)
    ps = SimplePart()
    r = a.radius or n / 16
    for k in range(a.nparticles):
        ps.add(x=(n / 2 + 3 * r * k, n / 2, n / 2), r=r, v=(0.01, 0, 0), m=2.0 * 4.0 / 3.0 * np.pi * r ** 3)
    ps.periodic[:] = True
    ps.period[:] = shape
    lat.particles = ps
    lat.init()
    lat.iterate(a.steps)
    torch.cuda.synchronize()
    print("ok", r, a.nparticles)


if __name__ == "__main__":
    main()
