"""d3q19_heat_adj_art — the heat-exchanger topology-optimisation model of the TCLB adjoint
article: D3Q19 MRT flow whose collision scales the momentum by (2 w - 1) (w = 1 fluid,
w = 0 reverses it like a bounce-back, w = 1/2 stops it) and a D3Q7 temperature (sigma^2 =
1/4) with conductivity w FluidAlpha + (1 - w) SolidAlpha.  Heater nodes pin T to the
zonal Temperature and report the injected heat (HeatInput); Outlet nodes integrate volume
/ heat / squared-heat fluxes, Thermometer nodes the temperature and penalties around
LimitTemperature; DesignSpace nodes the material penalty w (1 - w).
Only the five stress moments relax with omega = 1/(3 nu + 1/2); every other non-conserved
moment is set to its equilibrium (reference S-table).
Deviation (documented): the reference never initialises w on fluid nodes (the Init kernel
leaves the parameter density unset); here it starts at 1 (fluid), Solid nodes at 0.01.
Reference: models/article/d3q19_heat_adj_art/{Dynamics.R, Dynamics.c, Dynamics_adj.c.Rt}."""
import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.blocks import dense_transform
from ...emit.symbolic import d3q19_mrtmat, d3q19_velocities

U7 = np.array([[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]])


def _blocks(_m):
    M = d3q19_mrtmat()
    return "\n".join([dense_transform("art_moments", M, 19, 19, "moments = f . MRTMAT"),
                      dense_transform("art_inverse", M.inv(), 19, 19, "f = moments . MRTMAT^-1"),
                      # transposes for the reverse sweep (heat_adj_art_common.inc art_rev_collide)
                      dense_transform("art_moments_T", M.T, 19, 19, "a_f = a_m . MRTMAT^T"),
                      dense_transform("art_inverse_T", M.inv().T, 19, 19, "a_m = a_f . (MRTMAT^-1)^T")])


def build() -> Model:
    m = Model("d3q19_heat_adj_art", dims=3, family="optimization", reference="models/article/d3q19_heat_adj_art",
              description="D3Q19 MRT flow + D3Q7 heat, porosity design field (adjoint article model)")
    U = d3q19_velocities()
    for i in range(19):
        m.add_density(f"f[{i}]", int(U[i, 0]), int(U[i, 1]), int(U[i, 2]), group="f", comment=f"flow LB density F{i}")
    for i in range(7):
        m.add_density(f"T[{i}]", int(U7[i, 0]), int(U7[i, 1]), int(U7[i, 2]), group="T", comment=f"heat LB density G{i}")
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
    S("Temperature", default=1, comment="inlet density", zonal=True)
    S("LimitTemperature", default=1, comment="inlet density", zonal=True)
    S("FluidAlpha", default=1, comment="inlet density")
    S("SolidAlpha", comment="Heat conductivity of solid")
    S("Buoyancy", comment="Buoyancy coefficient of temperature")
    S("PorocityGamma", comment="Gamma in hiperbolic transformation of porocity (-infty,1)")
    S("PorocityTheta", comment="Theta in hiperbolic transformation of porocity",
      PorocityGamma="1.0 - exp(PorocityTheta)")
    for g, c, u in (("HeatInput", "Flux of heat into heater", "Km3/s"), ("HeatFlux", "Flux of heat", "Km3/s"),
                    ("HeatSquareFlux", "Flux of temperature squered", "K2m3/s"), ("Flux", "Volume flux", "m3/s"),
                    ("TemperatureAtPoint", "Integral of temperature", "K"),
                    ("HighTemperature", "Penalty for high temperature", "1"),
                    ("LowTemperature", "Penalty for low temperature", "1"),
                    ("MaterialPenalty", "Quadratic penalty for intermediate material parameter", "m3")):
        m.add_global(g, comment=c, unit=u)
    m.add_node_type("Heater", "ADDITIONALS")
    m.add_node_type("HeatSource", "ADDITIONALS")
    m.add_node_type("Thermometer", "OBJECTIVE")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    for n in ("EPressure", "Solid", "Wall", "WPressure", "WPressureL", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("DesignSpace", "DESIGNSPACE")
    m.add_codegen(_blocks)
    m.set_dynamics("optimization/d3q19_heat_adj_art.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
