#!/usr/bin/env python3
"""Race detector for stage data hazards (the reference's "permissive access" hazards,
src/conf.R:512-586): run each model's small catalog case on the OpenMP CPU executor with
1 thread and with N threads; any difference means some stage reads a field (through a
stencil) that other nodes of the same stage write.  Prints one JSON line per model.

    OMP_NUM_THREADS is set per child run:  python tools/race_check.py [models...]
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, torch
sys.path.insert(0, %r); sys.path.insert(0, %r)
from model_cases import run
lat = run(sys.argv[1], "cpu", steps=4)
torch.save(lat.fields_interior().clone(), sys.argv[2])
""" % (os.path.join(REPO, "tests"), REPO)


def main():
    import torch
    sys.path.insert(0, REPO)
    from tclb_amd.models import registry
    names = sys.argv[1:] or registry.names()
    bad = 0
    for n in names:
        outs = []
        for th in ("1", "8"):
            fn = f"/tmp/race_{n}_{th}.pt"
            r = subprocess.run([sys.executable, "-c", CHILD, n, fn], env={**os.environ, "OMP_NUM_THREADS": th},
                               capture_output=True, text=True)
            if r.returncode != 0:
                print(json.dumps({"model": n, "error": r.stderr[-300:]}), flush=True)
                break
            outs.append(torch.load(fn))
            os.unlink(fn)
        if len(outs) == 2:
            d = (outs[0] - outs[1]).abs().max().item()
            bad += d != 0
            print(json.dumps({"model": n, "max_diff_1_vs_8_threads": d}), flush=True)
    print(json.dumps({"models_with_races": bad}))


if __name__ == "__main__":
    main()
