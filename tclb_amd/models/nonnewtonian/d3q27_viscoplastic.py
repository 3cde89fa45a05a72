"""d3q27_viscoplastic — Vikhansky's yield-stress (Bingham) LBM on D3Q27: regularised
non-equilibrium stress rescaling, apparent viscosity and yield status per node; Zou/He
inlets/outlets, symmetry planes, optional zero-gradient outlets (OutFlow).
Reference: models/nonnewtonian/d3q27_viscoplastic/{Dynamics.R, Dynamics.c}."""
from ..dsl import Model
from ..flow.d3q27_bgk import P, U, add_slice_globals


def build(outflow: bool = False) -> Model:
    m = Model("d3q27_viscoplastic" + ("_OutFlow" if outflow else ""), dims=3, family="nonnewtonian",
              reference="models/nonnewtonian/d3q27_viscoplastic",
              description="D3Q27 Vikhansky viscoplastic (Bingham) fluid")
    for k in range(27):
        m.add_density(f"f[{k}]", int(U[k, 0]), int(U[k, 1]), int(U[k, 2]), group="f",
                      comment=f"density F{P[k, 0]}{P[k, 1]}{P[k, 2]}")
    if outflow:
        for k in range(27):
            x, y, z = (int(v) for v in U[k])
            m.add_field(f"f[{k}]", dx=-x - 1, dy=-y, dz=-z)
            m.add_field(f"f[{k}]", dx=-x, dy=-y - 1, dz=-z)
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("nu_app", unit="m2/s")
    m.add_quantity("yield_stat")
    m.add_setting("nu", default=0.16666666, comment="Viscosity")
    m.add_setting("Velocity", default="0m/s", comment="Inlet velocity", zonal=True, unit="m/s")
    m.add_setting("Pressure", default="0Pa", comment="Inlet/Outlet pressure", zonal=True, unit="Pa")
    m.add_density("nu_app", 0, 0, 0, group="state", comment="apparent viscosity")
    m.add_density("yield_stat", 0, 0, 0, group="state", comment="1 if unyielded, 0 if yielded")
    for a in "XYZ":
        m.add_setting(f"Force{a}", default="0m/s2", comment=f"Force {a}", unit="m/s2")
    m.add_setting("YieldStress", default="0Pa", comment="Yield stress", unit="Pa")
    m.add_global("Flux", comment="Volume flux", unit="m3/s")
    for n in ("SymmetryY", "SymmetryZ", "NVelocity_ZouHe", "SVelocity_ZouHe", "EVelocity_ZouHe", "WVelocity_ZouHe",
              "NPressure_ZouHe", "SPressure_ZouHe", "EPressure_ZouHe", "WPressure_ZouHe"):
        m.add_node_type(n, "BOUNDARY")
    for n in ("XYslice1", "XZslice1", "YZslice1", "XYslice2", "XZslice2", "YZslice2"):
        m.add_node_type(n, "ADDITIONALS")
    if outflow:
        m.add_node_type("NeumannXP", "BOUNDARY")
        m.add_node_type("NeumannYP", "BOUNDARY")
    m.add_global("TotalRho", comment="Total mass", unit="kg")
    add_slice_globals(m)
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"OutFlow": outflow}
    m.set_dynamics("nonnewtonian/d3q27_viscoplastic.inc")
    return m
