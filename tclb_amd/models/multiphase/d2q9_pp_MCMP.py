"""d2q9_pp_MCMP — Shan-Chen multi-component multiphase model (two D2Q9 populations: f,
the "wet" component, and g, the "dry" one) with cross-component interaction Gc,
fluid-wall adhesion Gad1/Gad2 through the wall potentials, a common velocity weighted by
the relaxation rates and the Shan-Chen velocity-shift forcing of each BGK collision.
Optional shear-layer initialisation (SL_*).
Reference: models/multiphase/experimental/d2q9_pp_MCMP/{Dynamics.R, Dynamics.c.Rt}
(the reference's unused MRT/LES/entropic routine is not carried over; quantity A is the
entropic-stabiliser ratio of the non-equilibrium part of f computed with the w-orthogonal
D2Q9 Hermite basis - parity unpinned).  The EoS constant ``R`` is the C++ member ``R_``.
"""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_pp_MCMP", dims=2, family="multiphase",
              reference="models/multiphase/experimental/d2q9_pp_MCMP",
              description="D2Q9 two-component Shan-Chen multiphase (velocity-shift forcing)")
    for grp in ("f", "g"):
        for i, (x, y) in enumerate(U9):
            m.add_density(f"{grp}[{i}]", x, y, 0, group=grp)
    m.add_field("psi_g", stencil2d=1)
    m.add_field("psi_f", stencil2d=1)
    m.add_stage("BaseIteration", "Run", save_fields=["f", "g"], load_densities=["f", "g"])
    m.add_stage("CalcPsi_f", "CalcPsi_f", save_fields=["psi_f"], load_densities=["f"])
    m.add_stage("CalcPsi_g", "CalcPsi_g", save_fields=["psi_g"], load_densities=["g"])
    m.add_stage("BaseInit", "Init", save_fields=["f", "g"], load_densities=["f", "g"])
    m.add_action("Iteration", ["BaseIteration", "CalcPsi_f", "CalcPsi_g"])
    m.add_action("Init", ["BaseInit", "CalcPsi_f", "CalcPsi_g"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("Rhof", unit="kg/m3")
    m.add_quantity("Rhog", unit="kg/m3")
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("A", unit="1", vector=True)
    m.add_quantity("Ff", unit="N", vector=True)
    m.add_quantity("Fg", unit="N", vector=True)
    S = m.add_setting
    S("omega", comment="one over relaxation time-wet")
    S("omega_g", comment="one over relaxation time-dry")
    S("nu", default=0.16666666, comment="viscosity-wet", omega="1.0/(3*nu + 0.5)")
    S("nu_g", default=0.16666666, comment="viscosity-dry", omega_g="1.0/(3*nu_g + 0.5)")
    S("Velocity_f", default=0, comment="inlet/outlet/init velocity 1st pop", zonal=True)
    S("Pressure_f", default=0, comment="inlet/outlet/init density 1st pop", zonal=True)
    S("Velocity_g", default=0, comment="inlet/outlet/init velocity 2nd pop", zonal=True)
    S("Pressure_g", default=0, comment="inlet/outlet/init density 2nd pop", zonal=True)
    S("Density", comment="higher density fluid - multiphase capable", zonal=True)
    S("Density_dry", comment="lower density fluid  - ideal gas assumption", zonal=True)
    S("Gc", comment="fluid1/2-fluid2/1 interation")
    S("Gad1", comment="fluid1-wall interation")
    S("Gad2", comment="fluid2-wall interation")
    S("R", default=1.0, comment="EoS gas const")
    S("T", default=1.0, comment="EoS reduced temp")
    S("a", default=1.0, comment="EoS a")
    S("b", default=4.0, comment="EoS b")
    S("Smag", comment="Smagorinsky constant")
    S("SL_U", comment="Shear Layer velocity")
    S("SL_lambda", comment="Shear Layer lambda")
    S("SL_delta", comment="Shear Layer disturbance")
    S("SL_L", comment="Shear Layer length scale")
    S("GravitationX", default=0.0, comment="Body Force")
    S("GravitationY", default=0.0, comment="Body Force")
    m.add_global("TotalDensity1", comment="quantity of fluid-1", unit="kg/m3")
    m.add_global("TotalDensity2", comment="quantity of fluid-2", unit="kg/m3")
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="pressure loss", unit="1m2/s")
    m.add_global("InletFlux", comment="pressure loss", unit="1m2/s")
    m.add_node_type("Smagorinsky", "LES")
    m.add_node_type("Stab", "ENTROPIC")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.set_dynamics("multiphase/d2q9_pp_MCMP.inc")
    return m
