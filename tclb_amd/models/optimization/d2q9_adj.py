"""d2q9_adj — porous-media topology optimisation model: d2q9 MRT flow whose velocity is
scaled by the local material parameter w (parameter density, the design variable on
DesignSpace nodes) through nw = w / (1 - gamma (1 - w)).  Gradients of the objective come
from the generic AD adjoint (no Tapenade).  Reference:
models/optimization/d2q9_adj/{Dynamics.R, Dynamics.c.Rt} (ADJOINT=1)."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_adj", dims=2, family="optimization", reference="models/optimization/d2q9_adj",
              description="D2Q9 MRT with a porosity design field w (topology optimisation)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_density("w", 0, 0, 0, group="w", parameter=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("W")
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1-1.0/(3*nu + 0.5)")
    S("Velocity", default="0m/s", comment="inlet velocity", zonal=True, unit="m/s")
    S("Pressure", default="0Pa", comment="inlet pressure", zonal=True, unit="Pa")
    S("ForceX", comment="Gravitation in the direction of x")
    S("ForceY", comment="Gravitation in the direction of y")
    for g, c in [("Drag", "pressure loss"), ("Lift", "pressure loss"), ("MaterialPenalty", "material penalty"),
                 ("Material", "material")]:
        m.add_global(g, comment=c)
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="pressure loss", unit="1m2/s")
    m.add_global("InletFlux", comment="pressure loss", unit="1m2/s")
    S("PorocityGamma", comment="gamma in hiperbolic transformation of porocity (-infty,1)")
    S("PorocityTheta", comment="theta in hiperbolic transformation of porocity", PorocityGamma="1.0 - exp(PorocityTheta)")
    S("Porocity", comment="initial porocity of Porous nodes", zonal=True)
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    for n in ["EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("DesignSpace", "DESIGNSPACE")
    m.set_dynamics("optimization/d2q9_adj.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
