#!/usr/bin/env python3
"""MLUPS / effective bandwidth of every model on one GPU (catalog performance table)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from model_cases import case_settings  # noqa: E402
from tclb_amd.lattice import Lattice  # noqa: E402
from tclb_amd.models import registry  # noqa: E402
from tclb_amd.utils.guard import collision_check  # noqa: E402


def state_finite(lat) -> bool:
    """globals and every stored field finite (one field at a time, on the device)"""
    if not all(np.isfinite(v) for v in lat.globals.values()):
        return False
    s = lat.snaps[lat.cur]
    return all(bool(torch.isfinite(s[i]).all().item()) for i in range(lat.nf))


def collision_flag(m) -> int:
    """the node-type value of the collision the model's default build runs: MRT where the
    model has both BGK and MRT types and is not built with its BGK option (the first
    COLLISION type alone flagged d3q27_pf_velocity(_thermo) BGK, which their MRT build
    does not collide: those runs streamed only, profiles/README.md r04r)"""
    types = [n for n in m.node_types if n.group == "COLLISION"]
    if not types:
        return 0
    names = [n.name for n in types]
    if "MRT" in names and not (getattr(m, "options", None) or {}).get("BGK"):
        return types[names.index("MRT")].value
    return types[0].value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="")
    ap.add_argument("--n3", type=int, default=256)
    ap.add_argument("--n2", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=100, help="timed iterations (BASELINE.md: >= 100)")
    ap.add_argument("--precision", default="double")
    ap.add_argument("--variants", default="", help="comma list of HIP build variants to A/B (interleaved)")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--splits", default="", help="comma list of tile-window maps (Lattice.set_tile_split) to A/B")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--flag", default="", help="node type to flag every node with (default: the collision the "
                                               "model's default build runs, collision_flag)")
    ap.add_argument("--glob-every-step", action="store_true", help="globals integrated on every step")
    ap.add_argument("--allow-invalid", action="store_true", help="exit 0 even when a run went non-finite")
    a = ap.parse_args()
    invalid = []
    variants = a.variants.split(",") if a.variants else [None]
    splits = [int(k) for k in a.splits.split(",")] if a.splits else [None]
    names = a.models.split(",") if a.models else registry.names()
    dev = torch.device("cuda", 0) if a.device == "cuda" else torch.device(a.device)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    for name, variant, split, rnd in [(n, v, k, r) for n in names for r in range(a.rounds) for v in variants
                                      for k in splits]:
        m = registry.get(name)
        shape = (a.n3, a.n3, a.n3) if m.dims == 3 else (a.n2, a.n2, 1)
        try:
            lat = Lattice(name, shape, device=dev, precision=a.precision, variant=variant)
            if split is not None:
                lat.set_tile_split(split)
            cf = case_settings(name).get("_flag")
            coll = m.node_type(a.flag).value if a.flag else (m.node_type(cf).value if cf else collision_flag(m))
            lat.set_flags(np.full((lat.NZ, lat.NY, shape[0]), coll, dtype=np.uint32))
            # the model-family settings of the catalog tests (a physical case; some
            # defaults, e.g. zero densities of the phase-field models, are not)
            for k, v in case_settings(name).items():
                if not k.startswith("_") and m.setting(k) is not None:
                    lat.set_setting(k, v)
            lat.init()

            def window():
                if a.glob_every_step:
                    for _ in range(a.steps):
                        lat.iterate(1, glob_last=True, reduce=False)
                else:
                    lat.iterate(a.steps, glob_last=True)
            # warm-up: the exact timed sequence once (every instantiation the window
            # launches — the globals step included — has run before the clock starts;
            # round 5 timed advection_diffusion2D's first globals launch, 2.34 ms)
            window()
            sync()
            t = time.perf_counter()
            window()
            sync()
            dt = (time.perf_counter() - t) / a.steps
            ok = state_finite(lat)
            guard = collision_check(lat)
            ok = ok and guard["collides"]
            if not ok:
                invalid.append(name)
            es = lat.snaps[0].element_size()
            nodes = shape[0] * shape[1] * shape[2]
            bpn = 2 * lat.nf * es + lat.flags.element_size()
            print(json.dumps({"model": name, "variant": variant, "split": lat.tile_split, "round": rnd, "glob_every_step": a.glob_every_step, "shape": shape, "fields": lat.nf, "stages": len(m.stages),
                              "ms": round(dt * 1e3, 3), "MLUPS": round(nodes / dt / 1e6, 1),
                              "GBps_meter": round(nodes * bpn / dt / 1e9, 1), "valid": ok,
                              "collides": guard["collides"], "collision_rel_diff": guard["rel_diff"],
                              "collision_nodes": guard["collision_nodes"]}), flush=True)
            del lat
            torch.cuda.empty_cache()
        except Exception as e:  # noqa
            print(json.dumps({"model": name, "error": str(e)[:300]}), flush=True)
            invalid.append(name)
    if invalid and not a.allow_invalid:
        print(f"perf_models: {len(invalid)} run(s) not valid (non-finite state or error): {','.join(invalid)}",
              file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
