#!/usr/bin/env python3
"""One model's GPU step against the CPU executor, field by field (the probe that located
the r05m class-2 fault, profiles/README.md r05m).

    STEPS=2 MODE=each|noglob VARIANT=<hip build variant> python tools/split_probe.py <model> [nx,ny,nz]

The case is tests/model_cases.make_case (collision everywhere, a Wall plane at x = 0),
perturbed, then stepped STEPS times (MODE=each: one iterate call per step, so every step
integrates globals; noglob: no globals at all); for the native loop and the per-step
Python path it prints the largest difference to the CPU run and the fields and
coordinates of the nodes that differ by more than 1e-9 of the scale."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from model_cases import make_case, perturb  # noqa: E402


def main():
    name = sys.argv[1]
    shape = tuple(int(v) for v in sys.argv[2].split(",")) if len(sys.argv) > 2 else None
    steps = int(os.environ.get("STEPS", "1"))
    mode = os.environ.get("MODE", "")
    res = {}
    for dev, nl in (("cpu", True), ("cuda", True), ("cuda", False)):
        kw = {"variant": os.environ["VARIANT"]} if dev == "cuda" and os.environ.get("VARIANT") else {}
        lat = make_case(name, dev, shape=shape, native_loop=nl, **kw)
        lat.init()
        perturb(lat)
        if mode == "each":
            for _ in range(steps):
                lat.iterate(1)
        elif mode == "noglob":
            lat.iterate(steps, glob_last=False)
        else:
            lat.iterate(steps)
        res[(dev, nl)] = lat.fields_interior().cpu().double()
        print(dev, "native" if nl else "python", lat._native_path("Iteration"), lat.shape, flush=True)
    ref = res[("cpu", True)]
    for k, a in res.items():
        d = (a - ref).abs()
        bad = (d > 1e-9 * ref.abs().max()).nonzero()
        print(k, "max diff", d.max().item(), "nodes off", bad.shape[0], flush=True)
        if bad.shape[0]:
            for ax, lab in ((0, "fields"), (1, "z"), (2, "y"), (3, "x")):
                print(f"   {lab}", sorted(set(bad[:, ax].tolist()))[:24])


if __name__ == "__main__":
    main()
