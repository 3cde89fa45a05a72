"""d2q9_thin_film — depth-averaged (Hele-Shaw / thin film) flow: d2q9 MRT or cumulant
collision with a Brinkman drag K = 12 rho nu h_Z^2 from the local inverse film height
h_Z (parameter density).  Reference: models/flow/d2q9_thin_film/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model
from .d2q9 import U9, d2q9_mrt_basis
from ...emit.blocks import mrt_block
from ...emit.symbolic import mrt_eq


def build() -> Model:
    m = Model("d2q9_thin_film", dims=2, family="flow", reference="models/flow/d2q9_thin_film",
              description="D2Q9 thin-film (Brinkman-drag) flow, MRT or cumulant collision")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", int(x), int(y), 0, group="f")
    m.add_density("h_Z", 0, 0, 0, group="HZ", parameter=True)
    m.add_stage("BaseIteration", "Run", load_densities=["f", "HZ"], save_fields=["f", "HZ"])
    m.add_stage("BaseInit", "Init", save_fields=["f", "HZ"])
    m.add_action("Iteration", ["BaseIteration"])
    m.add_action("Init", ["BaseInit"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("H_Z")
    S = m.add_setting
    S("RelaxationRate", comment="one over relaxation time", S2="1-RelaxationRate")
    S("Viscosity", default=0.16666666, comment="viscosity", RelaxationRate="1.0/(3*Viscosity + 0.5)")
    S("VelocityX", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("VelocityY", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default=0, comment="inlet/outlet/init density", zonal=True)
    S("Height", default=1, comment="iinitial height in Z direction", zonal=True)
    S("BrinkmanHeightInv", default=0, zonal=True)
    S("GravitationX")
    S("GravitationY")
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="pressure loss", unit="1m2/s")
    m.add_global("InletFlux", comment="pressure loss", unit="1m2/s")
    S("S2", default="0", comment="MRT Sx")
    S("S3", default="0", comment="MRT Sx")
    S("S4", default="0", comment="MRT Sx")
    S("nubuffer", default=0.01, comment="Viscosity in the buffer layer (cumulant)")
    for n in ["EPressure", "WPressure", "NVelocity", "SVelocity", "WVelocity", "EVelocity", "NSymmetry", "SSymmetry"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Cumulant", "COLLISION")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    eq = mrt_eq(U9, mat=d2q9_mrt_basis())
    m.add_codegen(lambda _m: mrt_block("mrt", eq))
    m.set_dynamics("flow/d2q9_thin_film.inc")
    return m
