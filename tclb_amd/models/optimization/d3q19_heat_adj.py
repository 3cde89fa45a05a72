"""d3q19_heat_adj — D3Q19 MRT flow + D3Q7 MRT heat transport with a solid/fluid design
field w (heat-exchanger topology optimisation): heat-flux objectives on Outlet nodes,
temperature penalties on Thermometer nodes, Heater nodes pulling the temperature to the
zonal Temperature.  Equilibria are the reference's MRT_eq(d3q19, correction) /
MRT_eq(d3q7, order=1, sigma2=1/4) in the lattices' own moment matrices.

Deviations (documented): in the reference only EVelocity has a working boundary
closure (the W/E pressure and W velocity closures are commented out and reduce to
no-ops); the same holds here.  The reference collision reads momenta into undeclared
Jx/Jy/Jz variables; here the momentum is what the equilibria take.
Reference: models/optimization/d3q19_heat_adj/{Dynamics.R, Dynamics.c.Rt} (ADJOINT=1)."""
import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.blocks import dense_transform, exprs_function, vjp_function
from ...emit.symbolic import d3q19_mrtmat, d3q19_velocities, mrt_eq_mat

U7 = np.array([[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]])
# attr(d3q7, "MAT") of src/lib/lattice.R:36-43 (rows = directions)
MAT7 = [[1, 0, 0, 0, 0, 0, -6], [1, 1, 0, 0, 1, 1, 1], [1, -1, 0, 0, 1, 1, 1], [1, 0, 1, 0, -1, 1, 1],
        [1, 0, -1, 0, -1, 1, 1], [1, 0, 0, 1, 0, -2, 1], [1, 0, 0, -1, 0, -2, 1]]


def _blocks(_m):
    Jx, Jy, Jz = sp.symbols("Jx Jy Jz")
    U19 = d3q19_velocities()
    cor = [-Jz ** 2 / 6, -Jy ** 2 / 6, -Jx ** 2 / 6]
    f19 = mrt_eq_mat(U19, d3q19_mrtmat(), correction=cor)
    g7 = mrt_eq_mat(U7, sp.Matrix(MAT7), order=1, sigma2=sp.Rational(1, 4))
    out = []
    for pre, eq, n in (("m19", f19, 19), ("m7", g7, 7)):
        out.append(dense_transform(f"{pre}_moments", eq.mat, n, n, "moments = f . MAT"))
        out.append(dense_transform(f"{pre}_inverse", eq.mat.inv(), n, n, "f = moments . MAT^-1"))
        out.append(exprs_function(f"{pre}_req", ["rho", "Jx", "Jy", "Jz"], eq.Req))
        out.append(exprs_function(f"{pre}_feq", ["rho", "Jx", "Jy", "Jz"], eq.feq))
        ords = ", ".join(str(int(o)) for o in eq.order)
        out.append(f"  TCLB_FN static constexpr int {pre}_order(int k) {{ constexpr int o[{n}] = {{{ords}}}; return o[k]; }}")
        # transposes for the reverse sweep (rev_run): linear maps and the Jacobians of the
        # equilibria in (rho, J)
        out.append(dense_transform(f"{pre}_moments_T", eq.mat.T, n, n, "a_f = a_m . MAT^T"))
        out.append(dense_transform(f"{pre}_inverse_T", eq.mat.inv().T, n, n, "a_m = a_f . (MAT^-1)^T"))
        out.append(vjp_function(f"{pre}_req_T", ["rho", "Jx", "Jy", "Jz"], eq.Req))
        out.append(vjp_function(f"{pre}_feq_T", ["rho", "Jx", "Jy", "Jz"], eq.feq))
    return "\n".join(out)


def build() -> Model:
    m = Model("d3q19_heat_adj", dims=3, family="optimization", reference="models/optimization/d3q19_heat_adj",
              description="D3Q19 MRT flow + D3Q7 heat with a solid/fluid design field (adjoint-ready)")
    U = d3q19_velocities()
    for i in range(19):
        m.add_density(f"f[{i}]", int(U[i, 0]), int(U[i, 1]), int(U[i, 2]), group="f")
    for i in range(7):
        m.add_density(f"g[{i}]", int(U7[i, 0]), int(U7[i, 1]), int(U7[i, 2]), group="g")
    m.add_density("w", 0, 0, 0, group="w", parameter=True, comment="weight fluid-solid")
    m.add_quantity("W")
    m.add_quantity("WB", adjoint=True)
    m.add_quantity("Rho")
    m.add_quantity("T")
    m.add_quantity("U", vector=True)
    S = m.add_setting
    S("nu", default=0.16666666, comment="viscosity")
    S("Velocity", default="0m/s", comment="inlet velocity", zonal=True, unit="m/s")
    S("Pressure", default="0Pa", comment="inlet pressure", zonal=True, unit="Pa")
    S("Temperature", default=1, comment="inlet temperature", zonal=True)
    S("LimitTemperature", default=1, comment="temperature limit", zonal=True)
    S("FluidAlpha", default=1, comment="thermal diffusivity of the fluid")
    S("SolidAlpha", comment="Heat conductivity of solid")
    S("Buoyancy", comment="Buoyancy coefficient of temperature")
    S("PorocityGamma", comment="Gamma in hiperbolic transformation of porocity (-infty,1)")
    S("PorocityTheta", comment="Theta in hiperbolic transformation of porocity",
      PorocityGamma="1.0 - exp(PorocityTheta)")
    for g, c, u in (("HeatFlux", "Flux of heat", "Km3/s"), ("HeatSquareFlux", "Flux of temperature squered", "K2m3/s"),
                    ("Flux", "Volume flux", "m3/s"), ("TemperatureAtPoint", "Integral of temperature", "K"),
                    ("HighTemperature", "Penalty for high temperature", "1"),
                    ("LowTemperature", "Penalty for low temperature", "1"),
                    ("MaterialPenalty", "Quadratic penalty for intermediate material parameter", "m3")):
        m.add_global(g, comment=c, unit=u)
    m.add_node_type("Heater", "ADDITIONALS")
    m.add_node_type("HeatSource", "ADDITIONALS")
    m.add_node_type("Thermometer", "OBJECTIVE")
    for n in ("EPressure", "Solid", "Wall", "WPressure", "WPressureL", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("DesignSpace", "DESIGNSPACE")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.add_codegen(_blocks)
    m.set_dynamics("optimization/d3q19_heat_adj.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
