#!/usr/bin/env python3
"""Timing of the unsteady adjoint (d3q19_adj porous duct) on the GPU adjoint executor:
primal steps/s, adjoint steps/s (each reverse step = checkpoint recompute + dual-number
sweep with the device adjoint push), and the gradient norm.

    python tools/bench_adjoint.py --size 128 --steps 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from tclb_amd.adjoint import Adjoint
    from tclb_amd.lattice import Lattice
    n = a.size
    dev = torch.device(a.device)
    lat = Lattice("d3q19_adj", (n, n, n), device=dev)
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, n), mrt, dtype=np.uint32)
    fl[:, :, 0] = m.node_type("WPressure").value | mrt
    fl[:, :, n - 1] = m.node_type("EPressure").value | mrt
    fl[:, :, n // 4 + 4] |= m.node_type("Outlet").value
    fl[:, :, 2:n // 4] |= m.node_type("DesignSpace").value
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    for k, v in {"nu": 0.1, "InletDensity": 1.01, "FluxInObj": 1.0, "Theta": 1.0}.items():
        lat.set_setting(k, v)
    lat.init()
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    f[wi, :, :, 2:n // 4] = 0.7
    lat.set_fields_interior(f)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    lat.iterate(a.steps)
    sync()
    tp = time.perf_counter() - t0
    ad = Adjoint(lat)
    sync()
    t0 = time.perf_counter()
    ad.unsteady(a.steps)
    sync()
    ta = time.perf_counter() - t0
    g = ad.field_gradient("w")
    nodes = n ** 3
    print(json.dumps({"case": f"d3q19_adj unsteady adjoint {n}^3", "device": a.device, "steps": a.steps,
                      "primal_ms_per_step": round(tp / a.steps * 1e3, 3),
                      "adjoint_ms_per_step": round(ta / a.steps * 1e3, 3),
                      "adjoint_MLUPS": round(nodes * a.steps / ta / 1e6, 2),
                      "J": ad.J, "grad_w_absmax": float(np.abs(g).max()),
                      "tangent_budget": ad.lib.tangents}), flush=True)


if __name__ == "__main__":
    main()
