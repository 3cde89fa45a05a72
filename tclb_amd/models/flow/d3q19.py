"""d3q19 — d'Humieres MRT (19x19 moment matrix), Zou/He-type inlet/outlet, bounce-back,
slice/volume globals.  Reference: models/flow/d3q19/Dynamics.R, Dynamics.c.Rt,
src/lib/d3q19.R."""
import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.blocks import dense_transform, exprs_function
from ...emit.symbolic import d3q19_mrt


def mrt19_block(_m):
    r = d3q19_mrt()
    M = r.MAT
    parts = ["  // ---- d3q19 d'Humieres MRT (reference src/lib/d3q19.R)"]
    parts.append(dense_transform("mrt_moments", M, 19, 19, "R = f . MRTMAT"))
    parts.append(dense_transform("mrt_inverse", M.inv(), 19, 19, "f = R . MRTMAT^-1 (= t(MRTMAT)/Mw)"))
    rho, Jx, Jy, Jz = sp.symbols("rho Jx Jy Jz")
    parts.append(exprs_function("mrt_req", ["rho", "Jx", "Jy", "Jz"], r.Req))
    feq = list(sp.Matrix([r.Req]) * M.inv())
    parts.append(exprs_function("mrt_feq", ["rho", "Jx", "Jy", "Jz"], [sp.expand(e) for e in feq]))
    return "\n".join(parts)


def build(les: bool = False) -> Model:
    m = Model("d3q19", dims=3, family="flow", reference="models/flow/d3q19",
              description="D3Q19 MRT (d'Humieres) with velocity/pressure inlets and slice integrals")
    r = d3q19_mrt()
    U = r.U
    for i in range(19):
        m.add_density(f"f[{i}]", int(U[i, 0]), int(U[i, 1]), int(U[i, 2]), group="f", comment=f"density F{i}")
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_setting("omega", comment="One over relaxation time")
    m.add_setting("nu", default=0.16666666, comment="Viscosity", unit="1m2/s", omega="1.0/(3*nu + 0.5)")
    m.add_setting("InletVelocity", default="0m/s", comment="Inlet velocity", unit="1m/s")
    m.add_setting("InletPressure", default="0Pa", comment="Inlet pressure", unit="1Pa",
                  InletDensity="1.0+InletPressure*3")
    m.add_setting("InletDensity", default=1, comment="Inlet density", unit="1kg/m3")
    for a in "XYZ":
        m.add_setting(f"Force{a}", comment=f"Force {a}")
    m.add_global("Flux", comment="Volume flux", unit="m3/s")
    for n in ["XYslice", "XZslice", "YZslice"]:
        m.add_node_type(n, "ADDITIONALS")
    for pl in ("XY", "XZ", "YZ"):
        for q, u in (("vx", "m3/s"), ("vy", "m3/s"), ("vz", "m3/s"), ("rho", "kg/m"), ("area", "m2")):
            m.add_global(f"{pl}{q}", comment="slice integral", unit=u)
    for q, u in (("vx", "m4/s"), ("vy", "m4/s"), ("vz", "m4/s"), ("px", "mkg/s"), ("py", "mkg/s"), ("pz", "mkg/s"),
                 ("rho", "kg"), ("volume", "m3")):
        m.add_global(f"VOL{q}", comment="volume integral", unit=u)
    m.add_global("MaxV", comment="Max velocity", unit="m3", op="MAX")
    for n in ["EPressure", "Solid", "Wall", "WPressure", "WPressureL", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_codegen(mrt19_block)
    m.set_dynamics("flow/d3q19.inc")
    return m
