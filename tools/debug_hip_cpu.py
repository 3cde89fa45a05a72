#!/usr/bin/env python3
"""Step-by-step HIP vs CPU comparison of one model (first step / field / node that
differs), for diagnosing executor mismatches on a GPU box."""
import sys
import os

import numpy as np
import torch

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
from model_cases import make_case, perturb  # noqa: E402


def main():
    name = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    a = make_case(name, "cuda")
    b = make_case(name, "cpu")
    for lat in (a, b):
        lat.init()
    d = (a.fields_interior().cpu() - b.fields_interior()).abs()
    print("after init", d.max().item())
    for lat in (a, b):
        perturb(lat)
    for s in range(steps):
        for lat in (a, b):
            lat.iterate(1)
        fa, fb = a.fields_interior().cpu(), b.fields_interior()
        d = (fa - fb).abs()
        print(f"step {s + 1}: max diff {d.max().item():.3e}")
        if d.max().item() > 1e-12:
            per = d.reshape(d.shape[0], -1).max(dim=1).values
            for i, f in enumerate(a.model.fields):
                if per[i] > 1e-12:
                    idx = np.unravel_index(int(d[i].argmax()), d[i].shape)
                    print(f"  field {f.name}: {per[i].item():.3e} at (z,y,x)={idx} gpu={fa[i][idx].item():.15g} cpu={fb[i][idx].item():.15g}")
            break


if __name__ == "__main__":
    main()
