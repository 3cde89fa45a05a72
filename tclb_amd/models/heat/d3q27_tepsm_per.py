"""d3q27_tePSM_per — thermal partially saturated method (PSM) for resolved particles in
periodic domains: D3Q27 BGK fluid with Guo forcing blended with a solid operator
(non-equilibrium bounce-back NEBB or superposition SUP) over the particle coverage, and a
D3Q27 total-energy distribution h (Guo et al. PRE 75 036704) with a conjugate
solid/fluid interface treatment (CollisionBGK_CHT).  Particle images across the periodic
box (DNx/DNy/DNz) enter the coverage.  Face boundaries: non-equilibrium extrapolation
walls (N/S/E/W/F/B Wall) and Zou/He pressure exits.

Reference: models/heat/d3q27_tePSM_per/{Dynamics.R, Dynamics.c.Rt},
OPT="(NEBB+SUP)*Isothermal".
"""
from ..dsl import Model

U27 = [[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1],
       [1, 1, 0], [-1, 1, 0], [1, -1, 0], [-1, -1, 0], [1, 0, 1], [-1, 0, 1], [1, 0, -1], [-1, 0, -1],
       [0, 1, 1], [0, -1, 1], [0, 1, -1], [0, -1, -1], [1, 1, 1], [-1, 1, 1], [1, -1, 1], [-1, -1, 1],
       [1, 1, -1], [-1, 1, -1], [1, -1, -1], [-1, -1, -1]]


def build(nebb: bool = False, sup: bool = False, isothermal: bool = False) -> Model:
    m = Model("d3q27_tePSM_per", dims=3, family="heat", reference="models/heat/d3q27_tePSM_per",
              description="thermal PSM (D3Q27 f + D3Q27 total-energy h) for periodic particle flows")
    for i, (x, y, z) in enumerate(U27):
        m.add_density(f"f[{i}]", x, y, z, group="f")
    if not isothermal:
        for i, (x, y, z) in enumerate(U27):
            m.add_density(f"h[{i}]", x, y, z, group="h")
    # every population readable at the 26 neighbours (face extrapolation, Dynamics.R:67-69)
    for d in list(m.densities):
        m.add_field(d.field.name, dx=(1, -1), dy=(1, -1), dz=(1, -1))
    for n in ("sol", "uPx", "uPy", "uPz"):
        m.add_density(n, 0, 0, 0, group="Force", parameter=True)
    m.add_quantity("Solid", unit="1")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Rho", unit="kg/m3")
    S = m.add_setting
    S("omegaF", comment="one over F relaxation time")
    S("omegaFplus", comment="one over F+ relaxation time for TRT")
    S("omegaFminus", comment="one over F- relaxation time for TRT")
    m.add_density("localOmegaF", 0, 0, 0, group="l", parameter=True)
    for a in "XYZ":
        S(f"WallVelocity{a}", default="0.0", zonal=True, comment=f"WallVelocity {a.lower()}-direction")
    for a in "XYZ":
        S(f"InitVelocity{a}", default="0.0", comment=f"Initialisation {a.lower()}-velocity")
    S("InletPressure", default="0Pa", comment="inlet pressure", InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, comment="inlet density")
    S("Pressure", default="0Pa", comment="Inlet pressure", zonal=True)
    for a in "XYZ":
        S(f"Gravitation{a}", default=0.0, comment=f"applied (rho)*Gravitation{a}")
    for a in "XYZ":
        S(f"Accel{a}", default=0.0, comment=f"body acceleration {a}")
    for a in "xyz":
        S(f"DN{a}", default=0, comment=f"Total nodes in {a.upper()} direction")
    m.add_global("TotalSVF", comment="Total of solids throughout domain")
    for f in "NEWSFB":
        m.add_node_type(f"{f}Wall", "BOUNDARY")
    for f in "NEWSFB":
        m.add_node_type(f"{f}Pressure", "BOUNDARY")
    groups = ["f", "Force"]
    calc_load = ["f", "Force"]
    if not isothermal:
        for n in ("TotEnergy", "Temperature", "rhoCp", "Conductivity", "mediaNum"):
            m.add_field(n, stencil3d=1, group="h")
        for n in ("localCv", "localConductivity", "localRho", "localOmegaH"):
            m.add_density(n, 0, 0, 0, group="l", parameter=True)
        for q in ("T", "T2", "TotEnergy", "TE2", "Cv"):
            m.add_quantity(q, unit="K" if q in ("T", "T2") else "1")
        S("omegaH", comment="one over H relaxation time")
        S("alpha", default=0.16666666, comment="Thermal Diffusivity")
        S("omegaHplus", comment="one over H+ relaxation time for TRT")
        S("omegaHminus", comment="one over H- relaxation time for TRT")
        S("ViscCoeff", default=0.0, comment="Thermoviscous coefficient")
        S("BoussinesqCoeff", default=0.0, comment="Boussinesq force coefficient")
        for mat in ("Fluid", "Solid"):
            S(f"{mat}Cv", default=1, comment="Thermal Cv")
            S(f"{mat}Rho", default=1, comment="Material density")
            S(f"{mat}Conductivity", default=1, comment="Thermal Conductivity")
        S("InitTemperature", default=1, zonal=True, comment="initial temperature")
        S("WallTemperatureGradient", default=0, zonal=True, comment="Gradient of temperature along wall")
        S("MediaNumber", default=1, zonal=True, comment="Media Number")
        m.add_node_type("Interface", "ADDITIONALS")
        m.add_node_type("Med2", "ADDITIONALS")
        groups = ["f", "h", "Force", "l"]
        calc_load = ["f", "Force", "l"]
    # the initial coverage (CalcPeriodicSolid in Init) needs the particles: particle stage
    m.add_stage("BaseInit", "Init", save_fields=groups, load_densities=groups, particle=True)
    # split: the interior collision and the face closures run as two kernels; defer: the
    # CHT interface closure of the interior collision runs as a third, over the tiles
    # whose nodes need it (they move with the particles)
    m.add_stage("BaseIteration", "Run", save_fields=groups, load_densities=groups, split=True,
                defer=not isothermal)
    # lazy: the populations are pulled only where a particle covers the node
    # (split + defer: the covered nodes' force pass is a kernel of its own on the GPU)
    m.add_stage("CalcF", "CalcF", save_fields=["Force"], load_densities=calc_load, particle=True, lazy_load=True,
                split=True, defer=True)
    m.add_action("Iteration", ["BaseIteration", "CalcF"])
    m.add_action("Init", ["BaseInit", "CalcF"])
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.options = {"NEBB": nebb, "SUP": sup, "Isothermal": isothermal}
    if not isothermal:
        m.add_codegen(lambda _m: f"  static constexpr int FI_H0 = {_m.field_index('h[0]')};")
    m.set_dynamics("heat/d3q27_tepsm_per.inc")
    m.glob_waves = 0          # 410-440 VGPRs: a 2-wave cap would spill heavily
    return m
