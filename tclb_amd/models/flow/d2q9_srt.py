"""d2q9_SRT — single-relaxation-time BGK tutorial model with Zou/He inlet/outlet.
Reference: models/flow/d2q9_SRT/Dynamics.R, Dynamics.c."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_SRT", dims=2, family="flow", reference="models/flow/d2q9_SRT",
              description="D2Q9 BGK (SRT) with Zou/He velocity/pressure boundaries")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_setting("omega", comment="inverse of relaxation time")
    m.add_setting("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu+0.5)")
    m.add_setting("Velocity", default=0, comment="inlet/outlet/init velocity", zonal=True)
    m.add_setting("Velocity_x", default=0, comment="inlet/outlet/init velocity in x", zonal=True)
    m.add_setting("Velocity_y", default=0, comment="inlet/outlet/init velocity in y", zonal=True)
    m.add_setting("GravitationX", default=0, comment="body/external acceleration", zonal=True)
    m.add_setting("GravitationY", default=0, comment="body/external acceleration", zonal=True)
    m.add_setting("Density", default=1, comment="Density")
    for n in ["EPressure", "WPressure", "WVelocity", "EVelocity", "Solid", "Wall"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.set_dynamics("flow/d2q9_srt.inc")
    return m
