"""d2q9_pf_pressureEvolution — mass-conserving phase-field LBM for immiscible two-phase
flow at large density ratios (Fakhari, Geier & Lee): a conservative Allen-Cahn phase field
h (D2Q9) and a pressure-evolution population f whose equilibrium is shifted by the
interfacial (mu grad phi) and body forces, with the mixed upwind/central directional
derivatives of the phase field (two-cell stencil field PhaseF).
Reference: models/multiphase/d2q9_pf_pressureEvolution/{Dynamics.R, Dynamics.c.Rt}
(the reference's velocity/pressure planes are empty placeholders and BGK is not
implemented there; both are kept as no-ops).
"""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_pf_pressureEvolution", dims=2, family="multiphase",
              reference="models/multiphase/d2q9_pf_pressureEvolution",
              description="D2Q9 conservative phase field + pressure-evolution hydrodynamics (MRT)")
    for grp in ("f", "h"):
        for i, (x, y) in enumerate(U9):
            m.add_density(f"{grp}[{i}]", x, y, 0, group=grp)
    m.add_field("PhaseF", stencil2d=2, group="phi")
    m.add_stage("PhaseInit", "Init", save_fields=["PhaseF"])
    m.add_stage("BaseInit", "Init_distributions", save_fields=["f", "h"])
    m.add_stage("calcPhase", "calcPhaseF", save_fields=["PhaseF"], load_densities=["h"])
    m.add_stage("BaseIter", "Run", save_fields=["f", "h"], load_densities=["f", "h"])
    m.add_action("Iteration", ["BaseIter", "calcPhase"])
    m.add_action("Init", ["PhaseInit", "BaseInit", "calcPhase"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("PhaseField", unit="1")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("P", unit="Pa")
    m.add_quantity("Mu", unit="1")
    m.add_quantity("Normal", unit="1/m", vector=True)
    m.add_quantity("InterfaceForce", unit="N", vector=True)
    S = m.add_setting
    S("Density_h", comment="High density")
    S("Density_l", comment="Low  density")
    S("PhaseField_h", default=1, comment="PhaseField in Liquid")
    S("PhaseField_l", default=0, comment="PhaseField gas")
    S("PhaseField", comment="Initial PhaseField distribution", zonal=True)
    S("W", default=4, comment="Anti-diffusivity coeff")
    S("M", default=0.05, comment="Mobility")
    S("sigma", comment="surface tension")
    S("omega_l", comment="one over relaxation time (low density fluid)")
    S("omega_h", comment="one over relaxation time (high density fluid)")
    S("Viscosity_l", default=0.16666666, comment="kinematic viscosity", omega_l="1.0/(3*Viscosity_l)")
    S("Viscosity_h", default=0.16666666, comment="kinematic viscosity", omega_h="1.0/(3*Viscosity_h)")
    S("VelocityX", default=0.0, comment="inlet/outlet/init velocity", zonal=True)
    S("VelocityY", default=0.0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default=0.0, comment="inlet/outlet/init density", zonal=True)
    S("GravitationX", default=0.0, comment="applied (rho)*GravitationX")
    S("GravitationY", default=0.0, comment="applied (rho)*GravitationY")
    S("BuoyancyX", default=0.0, comment="applied (rho-rho_h)*BuoyancyX")
    S("BuoyancyY", default=0.0, comment="applied (rho-rho_h)*BuoyancyY")
    S("GmatchedX", default=0.0, comment="applied (1-phi)*GmatchedX")
    S("GmatchedY", default=0.0, comment="applied (1-phi)*GmatchedY")
    S("Radius", default=0, comment="Radius of diffuse interface circle")
    S("CenterX", default=0, comment="Circle center x-coord")
    S("CenterY", default=0, comment="Circle Center y-coord")
    S("BubbleType", default=1, comment="Drop/bubble")
    for g, c, u in (("PressureLoss", "pressure loss", "1mPa"), ("OutletFlux", "pressure loss", "1m2/s"),
                    ("InletFlux", "pressure loss", "1m2/s"), ("TotalDensity", "Mass conservation check", "1kg/m3")):
        m.add_global(g, comment=c, unit=u)
    for g, c in (("BubbleVelocityX", "Bubble velocity in the x direction"),
                 ("BubbleVelocityY", "Bubble velocity in the y direction"),
                 ("BubbleVelocityZ", "Bubble velocity in the z direction"),
                 ("BubbleLocationY", "Bubble Location in the y direction"),
                 ("SumPhiGas", "Summation of (1-phi) in all gas cells")):
        m.add_global(g, comment=c)
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("multiphase/d2q9_pf_pressureEvolution.inc")
    return m
