"""d3q19_heat — D3Q19 flow (BGK in the d'Humieres moment basis) + D3Q7 advection-
diffusion of temperature with heater nodes.  Reference: models/heat/d3q19_heat."""
import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.blocks import exprs_function
from ...emit.symbolic import d3q19_mrtmat, d3q19_velocities, mrt_eq

D3Q7 = np.array([[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]])
D3Q7_MAT = sp.Matrix([[1, 0, 0, 0, 0, 0, -6], [1, 1, 0, 0, 1, 1, 1], [1, -1, 0, 0, 1, 1, 1],
                      [1, 0, 1, 0, -1, 1, 1], [1, 0, -1, 0, -1, 1, 1], [1, 0, 0, 1, 0, -2, 1],
                      [1, 0, 0, -1, 0, -2, 1]])


def _blocks(_m):
    U19 = d3q19_velocities()
    feq = mrt_eq(U19, mat=d3q19_mrtmat())
    geq = mrt_eq(D3Q7, mat=D3Q7_MAT, order=1, sigma2=sp.Rational(1, 4))
    return "\n".join([exprs_function("feq19", ["rho", "Jx", "Jy", "Jz"], feq.feq),
                      exprs_function("geq7", ["rho", "Jx", "Jy", "Jz"], geq.feq)])


def build() -> Model:
    m = Model("d3q19_heat", dims=3, family="heat", reference="models/heat/d3q19_heat",
              description="D3Q19 flow + D3Q7 temperature advection-diffusion")
    U19 = d3q19_velocities()
    for i in range(19):
        m.add_density(f"f[{i}]", *map(int, U19[i]), group="f", comment=f"flow LB density F{i}")
    for i in range(7):
        m.add_density(f"g[{i}]", *map(int, D3Q7[i]), group="g", comment=f"heat LB density G{i}")
    m.add_quantity("Rho")
    m.add_quantity("T")
    m.add_quantity("U", vector=True)
    m.add_setting("nu", default=0.16666666, comment="viscosity")
    m.add_setting("Velocity", default="0m/s", comment="inlet velocity", zonal=True, unit="m/s")
    m.add_setting("Pressure", default="0Pa", comment="inlet pressure", zonal=True, unit="Pa")
    m.add_setting("Temperature", default=1, comment="inlet temperature", zonal=True)
    m.add_setting("FluidAlpha", default=1, comment="thermal diffusivity")
    m.add_node_type("Heater", "ADDITIONALS")
    for n in ["EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.add_codegen(_blocks)
    m.set_dynamics("heat/d3q19_heat.inc")
    return m
