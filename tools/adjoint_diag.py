#!/usr/bin/env python3
"""Locate a GPU adjoint fault node by node: one adjoint step (Adjoint.step_back) of the
d3q19_adj duct of tests/test_gpu_adjoint.py from a fixed random a_next, on the GPU
(TCLB_AD_VARIANT selects the adhip build, e.g. "row" = the primal's row accessors) and
on the CPU AD executor; prints one JSON line per (mode, repeat) with the error and where
it sits (node coordinates, node types, dual-list membership).

  python tools/adjoint_diag.py [--repeats 2]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from tclb_amd.adjoint import Adjoint  # noqa: E402


def one(dev, seeded: bool, reverse: bool, a_next_cpu):
    from test_gpu_adjoint import duct
    lat, wi = duct(torch.device(dev))
    ad = Adjoint(lat, settings=["InletDensity"] if seeded else [], reverse=reverse)
    a = ad.step_back(a_next_cpu.to(lat.device), state=None)
    if lat.is_gpu:
        torch.cuda.synchronize()
    return lat, ad, a.cpu()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=2)
    ap.add_argument("--modes", default="all", help="all | dual (the dual-only step alone)")
    a = ap.parse_args()
    variant = os.environ.get("TCLB_AD_VARIANT", "")
    from test_gpu_adjoint import duct
    ref_lat, _ = duct(torch.device("cpu"))
    g = torch.Generator().manual_seed(11)
    a_next = torch.rand(ref_lat.snaps[0].shape, generator=g, dtype=torch.float64)
    bad_all = 0
    modes = ((True, False, "dual-only (seeded setting)"), (False, False, "dual-only"),
             (False, True, "reverse + dual list"))
    if a.modes == "dual":
        modes = modes[1:2]
    for seeded, reverse, mode in modes:
        lc, adc, ac = one("cpu", seeded, reverse, a_next)
        for rep in range(a.repeats):
            lg, adg, ag = one("cuda", seeded, reverse, a_next)
            nx, ny, nz = lg.shape
            sl = (slice(None), slice(lg.gz, lg.gz + nz), slice(lg.gy, lg.gy + ny), slice(0, nx))
            d = (ag[sl] - ac[sl]).abs()
            scale = ac[sl].abs().max().item()
            node_err = d.amax(0)                       # (nz, ny, nx)
            bad = (node_err > 1e-10 * scale).nonzero().tolist()
            flags = lg.get_flags()
            m = lg.model
            kinds = {}
            for z, y, x in bad:
                fl = int(flags[z, y, x])
                names = [nt.name for nt in m.node_types if nt.value and (fl & nt.mask) == nt.value]
                key = "+".join(names) or "none"
                kinds[key] = kinds.get(key, 0) + 1
            out = {"variant": variant or "default", "mode": mode, "repeat": rep, "max_err": d.max().item(),
                   "scale": scale, "bad_nodes": len(bad), "nodes": nx * ny * nz, "bad_by_type": kinds,
                   "bad_first": bad[:12],
                   "bad_fields": (d.amax((1, 2, 3)) > 1e-10 * scale).nonzero().flatten().tolist()[:30]}
            if seeded:
                sg, sc = adg.setting_gradient("InletDensity"), adc.setting_gradient("InletDensity")
                out["setting_grad"] = [sg, sc]
            print(json.dumps(out), flush=True)
            bad_all += len(bad)
    sys.exit(1 if bad_all else 0)


if __name__ == "__main__":
    main()
