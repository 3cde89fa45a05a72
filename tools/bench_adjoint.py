#!/usr/bin/env python3
"""Timing of the unsteady adjoint of the ADJOINT models on the GPU adjoint executor:
primal steps/s, adjoint steps/s (each reverse step = checkpoint recompute + the node
adjoints: hand-written reverse sweeps where the model has them, Model.set_reverse, else
dual-number passes — --dual forces those everywhere), and the gradient norm.

    python tools/bench_adjoint.py --model d3q19_heat_adj --size 128 --steps 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def setup(model: str, n: int, dev):
    """a design-optimisation case of the model on an n^3 (3-D) or n^2 (2-D) lattice: inlet /
    outlet planes in x, a design block, objectives on; returns the lattice"""
    from tclb_amd.lattice import Lattice
    from tclb_amd.models import registry
    m = registry.get(model)
    shape = (n, n, n) if m.dims == 3 else (n, n, 1)
    lat = Lattice(model, shape, device=dev)
    m = lat.model
    nt = lambda name: m.node_type(name).value  # noqa: E731
    mrt = nt("MRT")
    fl = np.full((lat.NZ, lat.NY, n), mrt, dtype=np.uint32)
    settings = {}
    if model == "d3q19_adj":
        fl[:, :, 0] = nt("WPressure") | mrt
        fl[:, :, n - 1] = nt("EPressure") | mrt
        fl[:, :, n // 4 + 4] |= nt("Outlet")
        settings = {"nu": 0.1, "InletDensity": 1.01, "FluxInObj": 1.0, "Theta": 1.0}
    elif model in ("d3q19_heat_adj", "d3q19_heat_adj_art"):
        fl[:, 0, :] = nt("Wall")
        fl[:, n - 1, :] = nt("Wall")
        fl[:, 1:n // 8, n // 8] |= nt("Heater")
        fl[:, :, n // 4 + 4] |= nt("Outlet")
        if model == "d3q19_heat_adj_art":
            fl[:, 1:n - 1, 0] = nt("WVelocity") | mrt
        settings = {"nu": 0.1, "FluidAlpha": 0.05, "Velocity": 0.01, "Temperature": 1.2, "HeatFluxInObj": 1.0,
                    "FluxInObj": 0.2}
        if model == "d3q19_heat_adj_art":
            settings["SolidAlpha"] = 0.02
    elif model == "d3q19_heat_adj_prop":
        fl[:, 0, :] = nt("Wall")
        fl[:, n - 1, :] = nt("Wall")
        fl[:, 1:n - 1, 0] = nt("WVelocity") | mrt
        fl[:, 1:n // 8, n // 8] |= nt("Heater")
        fl[:, :, n // 4 + 4] |= nt("Outlet")
        fl[:, 1:n - 1, 3:n // 4] |= nt("Propagate")
        settings = {"nu": 0.1, "FluidAlpha": 0.05, "SolidAlpha": 0.02, "InletVelocity": 0.01,
                    "InletTemperature": 1.0, "HeaterTemperature": 1.2, "PropagateX": 0.2, "HeatFluxInObj": 1.0,
                    "FluxInObj": 0.2}
    elif model in ("d2q9_adj", "d2q9_heat_adj"):
        fl[:, 0, :] = nt("Wall")
        fl[:, n - 1, :] = nt("Wall")
        fl[:, 1:n - 1, 0] = nt("WVelocity") | mrt
        fl[:, 1:n - 1, n - 1] = nt("EPressure") | mrt
        fl[:, 1:n - 1, n // 4 + 4] |= nt("Outlet")
        if model == "d2q9_adj":
            settings = {"nu": 0.1, "Velocity": 0.01, "OutletFluxInObj": 1.0, "PressureLossInObj": 0.5}
        else:
            settings = {"nu0": 0.1, "InletVelocity": 0.01, "FluidAlpha": 0.05, "SolidAlpha": 0.02,
                        "HeatFluxInObj": 1.0}
    elif model == "d2q9_kuper_adj":
        fl[:, 0, :] = nt("Wall")
        fl[:, n - 1, :] = nt("Wall")
        fl[:, 2:n // 2, n // 4 + 4:n // 4 + 8] |= nt("Obj1")
        settings = {"InitDensity": 1.0, "WallDensity": 1.0, "Temperature": 0.56, "FAcc": 1.0, "Magic": 0.01,
                    "MagicA": -0.152, "MagicF": 1.0, "GravitationX": 1e-4, "nu": 0.1, "FluidVelocityXInObj": 1.0,
                    "Density1InObj": 0.1}
    elif model == "d2q9_optimalMixing":
        fl[:, 0, :] = nt("Wall")
        fl[:, :, 0] = nt("Wall")
        fl[:, :, n - 1] = nt("Wall")
        fl[:, n - 1, 1:n - 1] = nt("NMovingWall") | mrt
        settings = {"nu": 0.05, "K": 0.02, "MovingWallVelocity": 0.05, "Temperature": 1.0, "TotalTempSqrInObj": 1.0,
                    "MovingWallPowerInObj": 0.1}
    elif model == "d2q9_plate":
        fl[:, 0, :] = nt("Wall")
        fl[:, n - 1, :] = nt("Wall")
        fl[:, 1:n - 1, 0] = nt("WVelocity") | mrt
        fl[:, 1:n - 1, n - 1] = nt("EPressure") | mrt
        settings = {"nu": 0.02, "VelocityX": 0.02, "Smag": 0.1, "PRAD": n / 16, "SM": 2.0, "PX": n / 4, "PY": n / 2,
                    "ForceXInObj": 1.0, "PowerInObj": 0.5}
    else:
        raise SystemExit(f"no adjoint bench case for {model}")
    if m.node_type("DesignSpace") is not None:
        if m.dims == 3:
            fl[:, 1:n - 1, 2:n // 4] |= nt("DesignSpace")
        else:
            fl[:, 1:n - 1, 2:n // 4] |= nt("DesignSpace")
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    if any(fd.nicename == "w" for fd in m.fields):
        f[m.field_index("w"), :, :, 2:n // 4] = 0.7
    if model == "d2q9_optimalMixing":        # a temperature pattern to mix: T = 1 in the lower half
        for i in range(5):
            f[m.field_index(f"g[{i}]"), :, : n // 2] *= 2.0
    lat.set_fields_interior(f)
    return lat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="d3q19_adj")
    ap.add_argument("--size", type=int, default=128, help="n (n^3 for 3-D models, n^2 for 2-D)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--dual", action="store_true", help="dual-number passes everywhere (no reverse sweeps)")
    a = ap.parse_args()
    from tclb_amd.adjoint import Adjoint
    n = a.size
    dev = torch.device(a.device)
    lat = setup(a.model, n, dev)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    lat.iterate(2)
    sync()
    t0 = time.perf_counter()
    lat.iterate(a.steps)
    sync()
    tp = time.perf_counter() - t0
    ad = Adjoint(lat, reverse=not a.dual)
    sync()
    # first sweep cold (it allocates the checkpoint and segment snapshots, tunes the
    # tangent windows), then the timed warm sweep, as in an optimisation loop's later
    # iterations; both reported
    t0 = time.perf_counter()
    ad.unsteady(a.steps)
    sync()
    tc = time.perf_counter() - t0
    t0 = time.perf_counter()
    ad.unsteady(a.steps)
    sync()
    ta = time.perf_counter() - t0
    # models without a design field: the state adjoint of the initial condition
    g = ad.field_gradient("w") if any(fd.nicename == "w" for fd in lat.model.fields) else ad.a0.cpu().numpy()
    nodes = lat.nodes
    ok = bool(np.isfinite(ad.J) and np.all(np.isfinite(g)))
    print(json.dumps({"case": f"{a.model} unsteady adjoint {'x'.join(map(str, lat.gshape))}", "device": a.device,
                      "steps": a.steps, "reverse_sweeps": bool(ad.reverse),
                      "primal_ms_per_step": round(tp / a.steps * 1e3, 3),
                      "adjoint_ms_per_step": round(ta / a.steps * 1e3, 3),
                      "adjoint_over_primal": round(ta / tp, 2),
                      "adjoint_cold_ms_per_step": round(tc / a.steps * 1e3, 3),
                      "adjoint_cold_over_primal": round(tc / tp, 2),
                      "adjoint_MLUPS": round(nodes * a.steps / ta / 1e6, 2),
                      "J": ad.J, "grad_w_absmax": float(np.abs(g).max()), "finite": ok,
                      "tangent_budget": ad.lib.tangents, "native_segment_steps": ad.native_steps,
                      "native": os.environ.get("TCLB_AD_NATIVE", "1") != "0"}), flush=True)
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
