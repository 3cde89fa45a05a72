#!/usr/bin/env python3
"""MLUPS / effective bandwidth of every model on one GPU (catalog performance table)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.lattice import Lattice  # noqa: E402
from tclb_amd.models import registry  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="")
    ap.add_argument("--n3", type=int, default=256)
    ap.add_argument("--n2", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--precision", default="double")
    ap.add_argument("--variants", default="", help="comma list of HIP build variants to A/B (interleaved)")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--glob-every-step", action="store_true", help="globals integrated on every step")
    a = ap.parse_args()
    variants = a.variants.split(",") if a.variants else [None]
    names = a.models.split(",") if a.models else registry.names()
    dev = torch.device("cuda", 0)
    for name, variant, rnd in [(n, v, r) for n in names for r in range(a.rounds) for v in variants]:
        m = registry.get(name)
        shape = (a.n3, a.n3, a.n3) if m.dims == 3 else (a.n2, a.n2, 1)
        try:
            lat = Lattice(name, shape, device=dev, precision=a.precision, variant=variant)
            coll = next((n.value for n in m.node_types if n.group == "COLLISION"), 0)
            lat.set_flags(np.full((lat.NZ, lat.NY, shape[0]), coll, dtype=np.uint32))
            lat.init()
            lat.iterate(3, glob_last=False)
            torch.cuda.synchronize()
            t = time.perf_counter()
            if a.glob_every_step:
                for _ in range(a.steps):
                    lat.iterate(1, glob_last=True, reduce=False)
            else:
                lat.iterate(a.steps, glob_last=False)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / a.steps
            es = lat.snaps[0].element_size()
            nodes = shape[0] * shape[1] * shape[2]
            bpn = 2 * lat.nf * es + lat.flags.element_size()
            print(json.dumps({"model": name, "variant": variant, "round": rnd, "glob_every_step": a.glob_every_step, "shape": shape, "fields": lat.nf, "stages": len(m.stages),
                              "ms": round(dt * 1e3, 3), "MLUPS": round(nodes / dt / 1e6, 1),
                              "GBps_meter": round(nodes * bpn / dt / 1e9, 1)}), flush=True)
            del lat
            torch.cuda.empty_cache()
        except Exception as e:  # noqa
            print(json.dumps({"model": name, "error": str(e)[:300]}), flush=True)


if __name__ == "__main__":
    main()
