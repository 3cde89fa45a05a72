"""d2q9_lee — Lee's free-energy two-phase model ("Eliminating parasitic currents in the
lattice Boltzmann equation method for nonideal gases"): a D2Q9 population set with the
density and the chemical potential carried as two-cell stencil fields; the interfacial
force is split into a biased (upwind, ``fB``) and a central (``fC``) directional
derivative of rho and mu.  BGK and MRT collisions, Zou/He planes, moving / forced walls,
wet/dry wall densities.
Reference: models/multiphase/experimental/d2q9_lee/{Dynamics.R, Dynamics.c.Rt}.

Naming deviation (documented): the reference stores the chemical potential in a field
called ``nu`` next to the viscosity setting ``nu``; here the field is ``mu`` so that the
setting and the field do not share one identifier (quantity ``Nu`` still exports it).
"""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_lee", dims=2, family="multiphase", reference="models/multiphase/experimental/d2q9_lee",
              description="D2Q9 Lee free-energy two-phase model (biased/central force split)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_field("rho", stencil2d=2)
    m.add_field("mu", stencil2d=2)
    m.add_stage("BaseIteration", "Run", save_fields=["f"], load_densities=["f"])
    m.add_stage("CalcRho", "CalcRho", save_fields=["rho"], load_densities=["f"])
    m.add_stage("CalcNu", "CalcNu", save_fields=["mu"], load_densities=False)
    m.add_stage("InitRho", "InitRho", save_fields=["rho"], load_densities=False)
    m.add_stage("InitF", "InitF", save_fields=["f"], load_densities=False)
    m.add_stage("InitF2", "InitF2", save_fields=["f"], load_densities=False)
    m.add_action("Iteration", ["BaseIteration", "CalcRho", "CalcNu"])
    m.add_action("Init", ["InitF2", "CalcRho", "CalcNu"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Nu", unit="kg/m3")
    m.add_quantity("P", unit="Pa")
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("InletVelocity", default=0, comment="inlet velocity", zonal=True, unit="m/s")
    S("InletPressure", default=0, comment="inlet pressure", zonal=True, unit="Pa",
      InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, comment="inlet density", zonal=True)
    S("OutletDensity", default=1, comment="inlet density", zonal=True)
    S("InitDensity", comment="inlet density", zonal=True)
    S("WallDensity", comment="vapor/liquid density of wall", zonal=True)
    S("GravitationY", comment="Gravitation in the direction of y")
    S("GravitationX", comment="Gravitation in the direction of x")
    S("MovingWallVelocity", comment="Velocity of the MovingWall", zonal=True)
    S("WetDensity", comment="wet density", zonal=True)
    S("DryDensity", comment="dry density", zonal=True)
    S("Wetting", comment="wetting factor", zonal=True)
    S("LiquidDensity", comment="Density of liquid phase")
    S("VaporDensity", comment="Density of vapor phase")
    S("Beta", comment="Beta of Lee model")
    S("Kappa", comment="Capilarity")
    m.add_global("MomentumX", comment="momentum")
    m.add_global("MomentumY", comment="momentum")
    m.add_global("Mass", comment="mass")
    for n in ("MovingWall", "ForcedMovingWall"):
        m.add_node_type(n, "BOUNDARY")
    for n in ("Wet", "Dry"):
        m.add_node_type(n, "ADDITIONALS")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("multiphase/d2q9_lee.inc")
    return m
