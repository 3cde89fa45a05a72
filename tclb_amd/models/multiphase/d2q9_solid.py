"""d2q9_solid — dendritic solidification of a binary alloy: D2Q9 MRT flow (Boussinesq
buoyancy, solid fraction drag), D2Q9 temperature and solute sets, solid fraction fi_s
growing at the interface from the local equilibrium liquid concentration (Gibbs-Thomson
curvature with 4-fold anisotropy), solute rejection by the partition coefficient.
Reference: models/multiphase/solidification/d2q9_solid/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_solid", dims=2, family="multiphase", reference="models/multiphase/solidification/d2q9_solid",
              description="D2Q9 solidification (flow + temperature + solute, solid fraction growth)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    for q, u in (("Rho", "kg/m3"), ("T", "K"), ("C", "1"), ("Ct", "1"), ("Cl_eq", "1"), ("Solid", "1")):
        m.add_quantity(q, unit=u)
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("K", unit="1/m")
    m.add_quantity("Theta", unit="1")
    for g in ("g", "h"):
        for i, (x, y) in enumerate(U9):
            m.add_density(f"{g}[{i}]", x, y, 0, group=g)
    m.add_density("fi_s", 0, 0, 0, group="fi_s")
    m.add_field("fi_s", dx=(-1, 1), dy=(-1, 1), comment="solidification")
    m.add_density("Cs", 0, 0, 0, group="Cs")
    S = m.add_setting
    S("nu", comment="viscosity", unit="m2/s")
    S("FluidAlfa", default=1, comment="thermal diffusivity", unit="m2/s")
    S("SoluteDiffusion", comment="Solute diffusion coefficient in liquid", unit="m2/s")
    S("C0", comment="Concentration 0")
    S("T0", comment="Temperature 0", unit="K")
    S("Teq", comment="Equilibrium temperature at interface", unit="K")
    S("Velocity", default="0m/s", comment="fluid velocity", zonal=True, unit="m/s")
    S("Pressure", comment="pressure", zonal=True, unit="Pa")
    S("Temperature", comment="temperature", zonal=True, unit="K")
    S("Concentration", comment="concentration", zonal=True)
    S("Theta0", comment="Angle of preferential growth", zonal=True, unit="d")
    S("PartitionCoef", comment="Partition coefficient k")
    S("LiquidusSlope", comment="Liquidus slope m", unit="K")
    S("GTCoef", comment="Gibbs-Thomson coefficient gamma", unit="mK")
    S("SurfaceAnisotropy", comment="Degree of anisotropy of surface energy")
    S("SoluteCapillar", comment="Solutal capillary length d_0", unit="m")
    S("Buoyancy", comment="Buoyancy Boussinesq approximation", unit="m/s2K")
    m.add_global("OutFlux")
    m.add_global("Material")
    for n in ("Heater", "ForceTemperature", "ForceConcentration", "Seed"):
        m.add_node_type(n, "ADDITIONALS")
    m.add_node_type("Obj", "OBJECTIVE")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("multiphase/d2q9_solid.inc")
    return m
