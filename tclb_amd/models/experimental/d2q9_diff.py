"""d2q9_diff — D2Q9 diffusion (zero-velocity BGK) with a material parameter w blending
two diffusivities (nu0 on w=0, nu1 on w=1), pressure-type inlet/outlet, and a
difference objective between the Obj2-recorded and Obj1 densities.
Reference: models/experimental/d2q9_diff/{Dynamics.R, Dynamics.c.Rt} (ADJOINT=1)."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_diff", dims=2, family="experimental", reference="models/experimental/d2q9_diff",
              description="D2Q9 diffusion with a two-material parameter field (adjoint-ready)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_density("r", 0, 0, 0, group="r")
    m.add_density("w", 0, 0, 0, group="w", parameter=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("RhoB", adjoint=True)
    m.add_quantity("W")
    m.add_quantity("R")
    m.add_quantity("WB", adjoint=True)
    m.add_setting("nu0", default=0.16666666, comment="viscosity")
    m.add_setting("nu1", default=0.16666666, comment="viscosity")
    m.add_setting("InitDensity", default="0Pa", comment="initial density")
    m.add_setting("InletDensity", default="0Pa", comment="inlet density")
    m.add_setting("OutletDensity", default="0Pa", comment="outlet density")
    m.add_global("Diff", comment="difference objective")
    for n in ("EPressure", "Solid", "Wall", "WPressure"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("Obj1", "OBJECTIVE")
    m.add_node_type("Obj2", "OBJECTIVE")
    m.set_dynamics("experimental/d2q9_diff.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
