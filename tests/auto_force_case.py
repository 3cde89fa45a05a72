"""The auto (non-particle) case of tests/test_kept_fields.py: a small cavity with a body
force that changes mid-run; python tests/auto_force_case.py <out.npz> wrote
tests/data/auto_force_ref.npz with the model that still stored the Force fields."""
import sys, numpy as np, torch
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd.lattice import Lattice

def run(precision="double"):
    lat = Lattice("auto_d3q19_BGK", (12, 10, 8), device=torch.device("cpu"), precision=precision)
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, 12), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, lat.gy, :] = m.node_type("Wall").value
    fl[:, lat.gy + 9, 1:11] = m.node_type("NVelocity").value | m.node_type("MRT").value
    lat.set_flags(fl)
    lat.set_setting("Viscosity", 0.02)
    lat.set_setting("Velocity", 0.05)
    lat.set_setting("ForceX", 1e-5)
    lat.init()
    out = {}
    lat.iterate(3)
    out["f3"] = lat.fields_interior().double().numpy().copy()
    out["U3"] = lat.quantity("U").double().numpy().copy()
    lat.set_setting("ForceX", -2e-5)       # a mid-run <Param name="ForceX">
    lat.set_setting("ForceZ", 3e-6)
    lat.iterate(2)
    out["f5"] = lat.fields_interior().double().numpy().copy()
    out["U5"] = lat.quantity("U").double().numpy().copy()
    out["F5"] = lat.quantity("F").double().numpy().copy()
    out["Flux"] = np.array([lat.globals["Flux"]])
    return out

if __name__ == "__main__":
    res = {}
    for p in ("double", "mixed-shift"):
        for k, v in run(p).items():
            res[f"{p}_{k}"] = v
    np.savez(sys.argv[1], **res)
    print("saved", list(res))
