"""d3q19_heat_adj_prop — variant of the article heat-exchanger model in which the design
weight is *propagated* along x before use: on Propagate nodes the effective weight is
w0 = w - PropagateX (1 - w1), w1 being the effective weight streamed in from x - 1 (two
transport densities w0 / w1 moving in -x / +x), elsewhere w0 = w.  The flow momentum of the
post-collision equilibrium is scaled by w0 (w0 = 0 stops the fluid), the D3Q7 temperature
(sigma^2 = 1/4) has conductivity w0 FluidAlpha + (1 - w0) SolidAlpha; Heater nodes pin T to
HeaterTemperature, HeatSource nodes add HeatSource, Thermometer nodes integrate the
temperature and the penalties around LimitTemperature.
Reference: models/article/experimental/d3q19_heat_adj_prop/{Dynamics.R, Dynamics.c.Rt,
Dynamics_adj.c.Rt} (ADJOINT=1)."""
import numpy as np

from ..dsl import Model
from ...emit.symbolic import d3q19_velocities
from .d3q19_heat_adj_art import U7, _blocks


def build() -> Model:
    m = Model("d3q19_heat_adj_prop", dims=3, family="optimization",
              reference="models/article/experimental/d3q19_heat_adj_prop",
              description="D3Q19 MRT flow + D3Q7 heat, design weight propagated along x (adjoint)")
    U = d3q19_velocities()
    for i in range(19):
        m.add_density(f"f[{i}]", int(U[i, 0]), int(U[i, 1]), int(U[i, 2]), group="f", comment=f"density F{i}")
    for i in range(7):
        m.add_density(f"T[{i}]", int(U7[i, 0]), int(U7[i, 1]), int(U7[i, 2]), group="T", comment=f"density T{i}")
    m.add_density("w0", -1, 0, 0, group="wm", comment="weight fluid-solid moving in X")
    m.add_density("w1", 1, 0, 0, group="wm", comment="weight fluid-solid moving in X")
    m.add_density("w", 0, 0, 0, group="w", parameter=True, comment="weight fluid-solid")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("T", unit="K")
    m.add_quantity("W")
    m.add_quantity("W0")
    m.add_quantity("WB", adjoint=True)
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", omega="1.0/(3*nu + 0.5)", default=0.16666666, comment="viscosity")
    S("InletVelocity", default="0m/s", comment="inlet velocity", unit="m/s")
    S("InletPressure", InletDensity="1.0+InletPressure/3", default="0Pa", comment="inlet pressure", unit="Pa")
    S("InletDensity", default=1, comment="inlet density")
    S("InletTemperature", comment="inlet temperature")
    S("HeaterTemperature", comment="temperature of the heater")
    S("LimitTemperature", comment="temperature of the heater")
    S("FluidAlpha", comment="heat conductivity of fluid")
    S("SolidAlpha", comment="heat conductivity of fluid")
    S("HeatSource", comment="heat conductivity of fluid")
    S("Inertia", comment="inertia of the transport equation")
    for g, c in (("HeatFlux", "pressure loss"), ("HeatSquareFlux", "pressure loss"), ("Flux", "pressure loss"),
                 ("Temperature", "integral of temperature"), ("HighTemperature", "penalty for high temperature"),
                 ("LowTemperature", "penalty for low temperature"),
                 ("MaterialPenalty", "quadratic penalty for intermediate material parameter")):
        m.add_global(g, comment=c)
    S("PropagateX", comment="inertia of the transport equation")
    for n in ("EPressure", "Solid", "Wall", "WPressure", "WPressureL", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("DesignSpace", "DESIGNSPACE")
    m.add_node_type("Heater", "ADDITIONALS")
    m.add_node_type("HeatSource", "ADDITIONALS")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.add_node_type("Propagate", "ADDITIONALS")
    m.add_node_type("Thermometer", "OBJECTIVE")
    m.add_codegen(_blocks)
    m.set_dynamics("optimization/d3q19_heat_adj_prop.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
