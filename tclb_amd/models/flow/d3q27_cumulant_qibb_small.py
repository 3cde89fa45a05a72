"""d3q27_cumulant_qibb_small — D3Q27 cumulant flow (bulk rate 8(2-w)/(8-w), third-order
cumulants relaxed with it except c111 = 0, higher orders dropped, force per unit mass)
with the quadratic interpolated bounce-back (QIBB) of the reference's qibb experiments on
STL cuts, Zou/He planes, equilibrium / bounce-back velocity inlets, a zero-gradient east
outlet, symmetry planes and slice-integral globals.
Deviation (documented): the reference keeps its slice accumulation (XY/XZ/YZ slice
globals) inside a commented-out block, so those globals stay 0 there; here they are
integrated over the slice nodes.
Reference: models/flow/qibb/d3q27_cumulant_qibb_small/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model
from .d3q27_cumulant import P, U, _blocks


def build() -> Model:
    m = Model("d3q27_cumulant_qibb_small", dims=3, family="flow",
              reference="models/flow/qibb/d3q27_cumulant_qibb_small",
              description="D3Q27 cumulant LBM with quadratic interpolated bounce-back (QIBB)")
    for k in range(27):
        m.add_density(f"f[{k}]", int(U[k, 0]), int(U[k, 1]), int(U[k, 2]), group="f",
                      comment=f"density F{k}")
    for d in list(m.densities):
        m.add_field(d.field.name, dx=0, dy=0, dz=0)
        if d.dx < 0:
            m.add_field(d.field.name, dx=-1, dy=0, dz=0)
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    S = m.add_setting
    S("nu", default=0.16666666, comment="Viscosity")
    S("nubuffer", default=0.01, comment="Viscosity in the buffer layer")
    S("Velocity", default="0m/s", comment="Inlet velocity", zonal=True, unit="m/s")
    S("Pressure", default="0Pa", comment="Inlet pressure", zonal=True, unit="Pa")
    S("GalileanCorrection", default=1.0, comment="Galilean correction term")
    S("ForceX", default=0, comment="Force force X")
    S("ForceY", default=0, comment="Force force Y")
    S("ForceZ", default=0, comment="Force force Z")
    m.add_global("Flux", comment="Volume flux", unit="m3/s")
    for n in ("SymmetryY", "SymmetryZ", "TopSymmetry", "BottomSymmetry", "NVelocity", "SVelocity", "NPressure",
              "SPressure", "EOutlet", "WVelocityEq", "WVelocityBB"):
        m.add_node_type(n, "BOUNDARY")
    for n in ("XYslice1", "XZslice1", "YZslice1", "XYslice2", "XZslice2", "YZslice2"):
        m.add_node_type(n, "ADDITIONALS")
    m.add_node_type("QIBB", "HO_BOUNDARY")
    m.add_global("TotalRho", comment="Total mass", unit="kg")
    for p in ("XY", "XZ", "YZ"):
        for s, u in (("vx", "m3/s"), ("vy", "m3/s"), ("vz", "m3/s"), ("rho1", "kg/m"), ("rho2", "kg/m"), ("area", "m2")):
            m.add_global(f"{p}{s}", comment="Volume flux", unit=u)
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_codegen(_blocks)
    m.set_dynamics("flow/d3q27_cumulant_qibb_small.inc")
    return m
