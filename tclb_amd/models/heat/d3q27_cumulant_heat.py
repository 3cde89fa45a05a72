"""d3q27_cumulant_heat — D3Q27 cumulant flow (Galilean-corrected, all third and higher
cumulants at equilibrium) coupled to a D3Q7 advection-diffusion temperature with uniform
relaxation (omegaT = 1/(3 Alpha + 1/2)), Boussinesq buoyancy on the y-momentum,
heater nodes, symmetry planes, Zou/He planes that also impose the temperature, and
time-correlated synthetic-turbulence inflow.
Reference: models/heat/experimental/d3q27_cumulant_heat/{Dynamics.R, Dynamics.c.Rt}.
"""
import numpy as np

from ..dsl import Model
from ...emit.blocks import feq_block, tensor_raw_transform
from ...emit.cumulants import cumulant_block

CV = (0, 1, -1)
P = np.array([[k % 3, (k // 3) % 3, k // 9] for k in range(27)])
U = np.array([[CV[a], CV[b], CV[c]] for a, b, c in P])
U7 = np.array([[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]])


def _blocks(_m):
    return "\n".join([
        tensor_raw_transform("raw_moments", U, P, inverse=False),
        tensor_raw_transform("raw_inverse", U, P, inverse=True),
        cumulant_block("cum", 3, drop_order_above=3),
        feq_block("geq7", U7, order=1),
    ])


def build() -> Model:
    m = Model("d3q27_cumulant_heat", dims=3, family="heat", reference="models/heat/experimental/d3q27_cumulant_heat",
              description="D3Q27 cumulant flow + D3Q7 temperature (Boussinesq)")
    for k in range(27):
        m.add_density(f"f[{k}]", int(U[k, 0]), int(U[k, 1]), int(U[k, 2]), group="f",
                      comment=f"density F{P[k, 0]}{P[k, 1]}{P[k, 2]}")
    for i, c in enumerate(U7):
        m.add_density(f"g[{i}]", int(c[0]), int(c[1]), int(c[2]), group="g", comment=f"heat LB density G{i}")
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("T", unit="K")
    S = m.add_setting
    S("nu", default=0.16666666, comment="Viscosity")
    S("nubuffer", default=0.01, comment="Viscosity in the buffer layer")
    S("Velocity", default=0, comment="Inlet velocity", zonal=True, unit="m/s")
    S("Pressure", default=0, comment="Inlet pressure", zonal=True, unit="Pa")
    S("Turbulence", comment="Turbulence intensity", zonal=True)
    S("Temperature", comment="Temperature", zonal=True)
    S("Alpha", zonal=True)
    S("Buoyancy", unit="N/K")
    S("BuoyancyT0", unit="K")
    S("GalileanCorrection", default=0.0, comment="Galilean correction term")
    for a in "XYZ":
        S(f"Force{a}", default=0, comment=f"Force force {a}")
    m.add_global("HeatFlux", comment="Heat flux", unit="Km3/s")
    for n in ("WVelocityTurbulent", "NSymmetry", "SSymmetry", "ISymmetry", "OSymmetry", "NVelocity", "SVelocity",
              "NPressure", "SPressure"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Heater", "ADDITIONALS")
    m.add_node_type("SamplingPlane", "ADDITIONALS")
    for n in ("SynthTX", "SynthTY", "SynthTZ"):
        m.add_density(n, 0, 0, 0, group="SynthT")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_codegen(_blocks)
    m.set_dynamics("heat/d3q27_cumulant_heat.inc")
    return m
