"""d2q9_plate — a moving rigid plate / cylinder immersed in a D2Q9 MRT-Smagorinsky flow
through a smoothed penalisation field w(x, y) in the body frame; the body position and
angle are zonal settings (PX, PY, PR) whose time derivatives (PX_DT, ...) give the body
velocity, typically driven by a <Control> time series.  Reaction forces, moment, power
and volume are globals; the efficiency objectives EfficiencyX/Y = Force/Power are model
objective functions.  Reference: models/moving/d2q9_plate/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_plate", dims=2, family="moving", reference="models/moving/d2q9_plate",
              description="D2Q9 MRT-LES flow around a prescribed-motion plate (penalisation)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_density("avg_ux", 0, 0, 0, group="avg_u")
    m.add_density("avg_uy", 0, 0, 0, group="avg_u")
    m.add_density("avg_fx", 0, 0, 0, group="avg_f")
    m.add_density("avg_fy", 0, 0, 0, group="avg_f")
    m.add_node_type("NVelocity", "BOUNDARY")
    m.add_node_type("SPressure", "BOUNDARY")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("U_AVG", unit="m/s", vector=True)
    m.add_quantity("F_AVG", unit="N/m3", vector=True)
    m.add_quantity("Solid", unit="1")
    S = m.add_setting
    S("nu", default=0.16666666, comment="viscosity", zonal=True, unit="m2/s")
    S("VelocityY", default=0, comment="inlet/outlet/init velocity", zonal=True, unit="m/s")
    S("VelocityX", default=0, comment="inlet/outlet/init velocity", zonal=True, unit="m/s")
    S("Density", default=1, comment="inlet/outlet/init density", zonal=True, unit="kg/m3")
    S("Smag", default=1, comment="Smagorinsky constant")
    m.add_quantity("RhoB", adjoint=True, adjoint_of="f")
    m.add_quantity("UB", adjoint=True, vector=True)
    for g, c, u in (("ForceX", "reaction force X", "N/m"), ("ForceY", "reaction force Y", "N/m"),
                    ("Moment", "reaction moment", "N"), ("PowerX", "power X", "W/m"), ("PowerY", "power Y", "W/m"),
                    ("PowerR", "power of rotation", "W/m"), ("Power", "power", "W/m"), ("Power2", "power", "W/m"),
                    ("VolumeW", "Volume of moving body", "m2")):
        m.add_global(g, comment=c, unit=u)
    S("PDX", default=0, comment="plate diameter X", unit="m")
    S("PDY", default=0, comment="plate diameter Y", unit="m")
    S("PRAD", default=0, comment="cylinder radius", unit="m")
    S("SM", default=1, comment="smoothing diameter", unit="m")
    S("SM_M", default=0, comment="smoothing bias")
    S("EPSF", default=1, comment="boundary function, 0 - linear boundary, 1 - third order boundary")
    S("BF", default=0, comment="beta function bool")
    S("PX", default=0, comment="plate position X", zonal=True, unit="m")
    S("PY", default=0, comment="plate position Y", zonal=True, unit="m")
    S("PR", default=0, comment="plate angle", zonal=True)
    m.add_objective("EfficiencyX", "ForceX / Power")
    m.add_objective("EfficiencyY", "ForceY / Power")
    S("ExternalForceX", default=0, comment="external force x", zonal=True, unit="N/m3")
    S("ExternalForceY", default=0, comment="external force y", zonal=True, unit="N/m3")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("moving/d2q9_plate.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
