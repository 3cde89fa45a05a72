"""d2q9_pf — conservative phase-field (Allen-Cahn) interface tracking coupled to the
d2q9 weighted-MRT flow solver.  Options (conf.mk OPT="no_bc+fd"): ``no_bc`` drops the
per-node BC velocity densities, ``fd`` computes the interface normal from a stored phase
field ``phi`` (extra CalcPhi stage, isotropic finite differences) instead of from the h
populations.  Reference: models/multiphase/d2q9_pf/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model
from ..flow.d2q9 import U9, d2q9_mrt_basis
from ...emit.blocks import mrt_block
from ...emit.symbolic import mrt_eq


def build(no_bc: bool = False, fd: bool = False) -> Model:
    m = Model("d2q9_pf", dims=2, family="multiphase", reference="models/multiphase/d2q9_pf",
              description="D2Q9 MRT flow + conservative phase-field (Allen-Cahn) LBM")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", int(x), int(y), 0, group="f")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"h[{i}]", int(x), int(y), 0, group="h")
    if not no_bc:
        m.add_density("BC[0]", group="BC", parameter=True)
        m.add_density("BC[1]", group="BC", parameter=True)
    if fd:
        m.add_field("phi", stencil2d=1)
        m.add_stage("BaseIteration", "Run", load_densities=["h", "f", "BC"], save_fields=["h", "f", "BC"])
        m.add_stage("CalcPhi", "CalcPhi", save_fields=["phi"], load_densities=["h"])
        m.add_stage("BaseInit", "Init", save_fields=["h", "f", "BC"])
        m.add_action("Iteration", ["BaseIteration", "CalcPhi"])
        m.add_action("Init", ["BaseInit", "CalcPhi"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("DEBUG", vector=True)
    m.add_quantity("Normal", unit="1/m", vector=True)
    m.add_quantity("PhaseField", unit="1")
    S = m.add_setting
    S("IntWidth", default=0.33333, comment="Interface width")
    S("Mobility", default=0.001, comment="Mobility")
    S("PhaseField", default=0.5, comment="Phase Field marker scalar", zonal=True)
    S("OverwriteVelocityField", default="0")
    S("PF_Advection_Switch", default=1.0, comment="Parameter to turn on/off advection of phase field - usefull for initialisation")
    S("RelaxationRate", comment="one over relaxation time", S2="1-RelaxationRate")
    S("Viscosity", default=0.16666666, comment="viscosity", RelaxationRate="1.0/(3*Viscosity + 0.5)")
    S("VelocityX", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("VelocityY", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default=0, comment="inlet/outlet/init density", zonal=True)
    S("GravitationX", default=0)
    S("GravitationY", default=0)
    S("S2", default="0", comment="MRT Sx")
    S("S3", default="0", comment="MRT Sx")
    S("S4", default="0", comment="MRT Sx")
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="pressure loss", unit="1m2/s")
    m.add_global("InletFlux", comment="pressure loss", unit="1m2/s")
    for n in ["NPressure", "SPressure", "WPressure", "EPressure", "WVelocity", "EVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"no_bc": no_bc, "fd": fd, "bc": not no_bc}
    eq = mrt_eq(U9, mat=d2q9_mrt_basis())
    m.add_codegen(lambda _m: mrt_block("mrt", eq))
    m.set_dynamics("multiphase/d2q9_pf.inc")
    return m
