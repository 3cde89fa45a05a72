#!/usr/bin/env python3
"""Stand-alone rigid-sphere integrator speaking the socket RFI protocol
(tclb_amd/particles/rfi.py) — the counterpart of the reference's `simplepart` program
(src/simplepart.cpp), and with --empty of its `empty` placeholder (src/empty.cpp: no
particles, just the exchange until the lattice stops).

    python tools/rfi_simplepart.py --address 127.0.0.1:5555 --config particles.json

config: {"particles": [{"x": [..], "r": .., "v": [..], "omega": [..], "m": .., "fixed": false}],
         "acc": [ax, ay, az], "periodic": [px, py, pz] (0 = not periodic)}   (lattice units)
--log writes Iteration and x/v/f of every particle per integrated step.
"""
import argparse
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.particles.rfi import IntegratorClient  # noqa: E402
from tclb_amd.particles.system import integrate_rigid  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--config", default=None)
    ap.add_argument("--empty", action="store_true")
    ap.add_argument("--log", default=None)
    a = ap.parse_args()
    cfg = json.load(open(a.config)) if a.config else {}
    ps = [] if a.empty else cfg.get("particles", [])
    n = len(ps)
    x = np.array([p["x"] for p in ps], float).reshape(n, 3)
    v = np.array([p.get("v", [0, 0, 0]) for p in ps], float).reshape(n, 3)
    w = np.array([p.get("omega", [0, 0, 0]) for p in ps], float).reshape(n, 3)
    r = np.array([p["r"] for p in ps], float)
    m = np.array([p.get("m") or 4.0 / 3.0 * math.pi * p["r"] ** 3 for p in ps], float)
    fixed = np.array([bool(p.get("fixed", False)) for p in ps])
    acc = np.asarray(cfg.get("acc", [0, 0, 0]), float)
    per = np.asarray(cfg.get("periodic", [0, 0, 0]), float)
    client = IntegratorClient(a.address)
    # the calculator's configuration (reference simplepart.cpp:100-145: "content" holds
    # the configuration, "output" names the log)
    if not a.config and client.has_var("content"):
        try:
            cfg = json.loads(client.get_var("content"))
        except ValueError:
            cfg = {}
        ps = [] if a.empty else cfg.get("particles", [])
        n = len(ps)
        x = np.array([p["x"] for p in ps], float).reshape(n, 3)
        v = np.array([p.get("v", [0, 0, 0]) for p in ps], float).reshape(n, 3)
        w = np.array([p.get("omega", [0, 0, 0]) for p in ps], float).reshape(n, 3)
        r = np.array([p["r"] for p in ps], float)
        m = np.array([p.get("m") or 4.0 / 3.0 * math.pi * p["r"] ** 3 for p in ps], float)
        fixed = np.array([bool(p.get("fixed", False)) for p in ps])
        acc = np.asarray(cfg.get("acc", [0, 0, 0]), float)
        per = np.asarray(cfg.get("periodic", [0, 0, 0]), float)
    if a.log is None and client.has_var("output") and n:
        a.log = client.get_var("output") + "_SP_Log.csv"
    log = open(a.log, "w") if a.log else None
    if log:
        log.write("Iteration," + ",".join(f"p{i}_{c}{d}" for i in range(n) for c in ("", "v", "f") for d in "xyz") + "\n")
    it = 0
    while True:
        res = client.exchange(x, v, w, r)
        if res is None:
            break
        integrate, f = res
        if integrate and n:
            integrate_rigid(x, v, w, r, m, fixed, f[:, 0:3], f[:, 3:6], acc, per > 0, per)
        if integrate:
            it += 1
            if log:
                row = [str(it)] + [f"{val:.10e}" for i in range(n) for arr in (x, v, f[:, 0:3]) for val in arr[i]]
                log.write(",".join(row) + "\n")
    client.close()
    if log:
        log.close()
    print(f"rfi_simplepart: {it} steps, {n} particle(s)")


if __name__ == "__main__":
    main()
