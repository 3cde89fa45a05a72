"""d2q9_lbmpy — the reference's lbmpy-coupling example: a D2Q9 compressible cumulant
collision with a single relaxation rate omega (shear; bulk and higher orders at rate 1, the
lbmpy default for Method.CUMULANT with one rate) and body-force density G, Zou/He inlets
and outlets.  The reference generates the collision with lbmpy/pystencils at build time;
lbmpy is not available here, so the same method is written directly (the shared D2Q9
cumulant kernel).  Parity with lbmpy's generated code: unpinned (no lbmpy output in the
reference).  Reference: models/lbmpy/d2q9_lbmpy/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_lbmpy", dims=2, family="flow", reference="models/lbmpy/d2q9_lbmpy",
              description="D2Q9 cumulant (lbmpy method) with body force")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f", comment=f"f_{i}")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_setting("omega", comment="inverse of relaxation time")
    m.add_setting("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu+0.5)")
    for a in "XY":
        m.add_setting(f"Velocity{a}", default=0, comment=f"inlet/outlet/init velocity in {a.lower()}", zonal=True)
    for a in "XY":
        m.add_setting(f"Gravitation{a}", default=0, comment="body/external acceleration", zonal=True)
    m.add_setting("Density", default=1, comment="Density")
    for n in ("EPressure", "WPressure", "WVelocity", "EVelocity", "Solid", "Wall"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.set_dynamics("flow/d2q9_lbmpy.inc")
    return m
