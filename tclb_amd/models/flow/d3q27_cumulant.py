"""d3q27_cumulant — cumulant collision (Geier et al.) with Galilean correction, optional
Smagorinsky (SMAG), running averages (AVG) and interpolated bounce-back (IB, STL cuts).
Reference: models/flow/d3q27_cumulant/Dynamics.R, Dynamics.c.Rt (OPT="AVG*IB*SMAG")."""
import numpy as np

from ..dsl import Model
from ...emit.blocks import tensor_raw_transform
from ...emit.cumulants import cumulant_block

CV = (0, 1, -1)
# reference order: expand.grid(x=c(0,1,-1), y=.., z=..); index k = px + 3 py + 9 pz
P = np.array([[k % 3, (k // 3) % 3, k // 9] for k in range(27)])
U = np.array([[CV[a], CV[b], CV[c]] for a, b, c in P])


def _blocks(_m):
    return "\n".join([
        tensor_raw_transform("raw_moments", U, P, inverse=False),
        tensor_raw_transform("raw_inverse", U, P, inverse=True),
        cumulant_block("cum", 3, drop_order_above=3),
    ])


def build(avg: bool = False, ib: bool = False, smag: bool = False, part: bool = False) -> Model:
    """``part``: the d3q27_cumulant_part variant (reference models/flow/d3q27_cumulant_part):
    a particle stage CalcF writes the coupling force density (fx,fy,fz,sol) that the
    next collision applies instead of the uniform ForceX/Y/Z."""
    name = "d3q27_cumulant_part" if part else "d3q27_cumulant"
    m = Model(name, dims=3, family="flow", reference=f"models/flow/{name}",
              description="D3Q27 cumulant LBM with Galilean correction (+SMAG/AVG/IB options)"
              + (", particle coupling (CalcF stage)" if part else ""))
    for k in range(27):
        m.add_density(f"f[{k}]", int(U[k, 0]), int(U[k, 1]), int(U[k, 2]), group="f",
                      comment=f"density F{P[k, 0]}{P[k, 1]}{P[k, 2]}")
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Solid", unit="1")
    if part:
        for n in ("fx", "fy", "fz", "sol"):
            m.add_density(n, 0, 0, 0, group="Force", parameter=True)
        m.add_quantity("F", unit="N/m3", vector=True)
        m.add_setting("ParticleVelocityLimit", default=0.05, unit="m/s",
                      comment="(local) particle velocity limit")
        m.add_stage("BaseIteration", "Run", save_fields=["f", "Force", "avg"], load_densities=["f", "Force", "avg"])
        m.add_stage("BaseInit", "Init", save_fields=["f", "Force", "avg"])
        # lazy: the populations are pulled only within reach of a particle
        m.add_stage("CalcF", "CalcF", save_fields=["Force"], load_densities=["f", "Force"], particle=True,
                    lazy_load=True)
        m.add_action("Iteration", ["BaseIteration", "CalcF"])
        m.add_action("Init", ["BaseInit", "CalcF"])
    m.add_setting("nu", default=0.16666666, comment="Viscosity")
    m.add_setting("nubuffer", default=0.01, comment="Viscosity in the buffer layer")
    m.add_setting("Velocity", default="0m/s", comment="Inlet velocity", zonal=True, unit="m/s")
    m.add_setting("Pressure", default="0Pa", comment="Inlet pressure", zonal=True, unit="Pa")
    m.add_setting("Turbulence", comment="Turbulence intensity", zonal=True)
    m.add_setting("GalileanCorrection", default=1.0, comment="Galilean correction term")
    for a in "XYZ":
        m.add_setting(f"Force{a}", default=0, comment=f"Force {a}")
    m.add_setting("Omega", default=1, comment="relaxation rate for 3rd order cumulants")
    if part:
        m.add_setting("Smag", default=0, comment="Smagorinsky coefficient for SGS modeling")
    else:
        m.add_global("Density", comment="system density", unit="kg/m3")
    m.add_global("Flux", comment="Volume flux", unit="m3/s")
    m.add_global("Drag", comment="Force exerted on body in X-direction", unit="N")
    m.add_global("Lift", comment="Force exerted on body in Z-direction", unit="N")
    m.add_global("Lateral", comment="Force exerted on body in Y-direction", unit="N")
    if not part:
        m.add_global("Mass", comment="Integral of density over the domain", unit="kg")
        for a in "XYZ":
            m.add_global(f"{a}Momentum", comment=f"Integral of momentum in {a}", unit="kgm/s")
    for n in (["WVelocityTurbulent", "NVelocity", "SVelocity", "NPressure", "SPressure"] if part else
              ["Buffer", "WVelocityTurbulent", "NVelocity", "SVelocity", "NPressure", "SPressure"]):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("NSymmetry", "ADDITIONALS")
    m.add_node_type("SSymmetry", "ADDITIONALS")
    m.add_node_type("Body", "BODY")
    if smag:
        m.add_setting("Smag", default=0, comment="Smagorinsky coefficient for SGS modeling")
    if ib:
        m.add_node_type("IB", "HO_BOUNDARY")
    if avg:
        m.add_quantity("KinE", comment="Turbulent kinetic energy")
        m.add_quantity("ReStr", comment="Reynolds stress off-diagonal component", vector=True)
        m.add_quantity("Dissipation", comment="Dissipation e")
        m.add_quantity("avgU", unit="m/s", vector=True)
        m.add_quantity("varU", vector=True)
        m.add_quantity("averageP", unit="Pa")
        for n in ["avgP", "varUX", "varUY", "varUZ", "varUXUY", "varUXUZ", "varUYUZ", "avgdxu2", "avgdyv2",
                  "avgdzw2", "avgUX", "avgUY", "avgUZ"]:
            m.add_density(n, 0, 0, 0, group="avg", average=True)
        m.add_field("avgUX", dx=(-1, 1), average=True)
        m.add_field("avgUY", dy=(-1, 1), average=True)
        m.add_field("avgUZ", dz=(-1, 1), average=True)
    for n in (["EPressure", "EVelocity", "Wall", "WPressure", "WVelocity"] if part else
              ["EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"]):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"AVG": avg, "IB": ib, "SMAG": smag, "PART": part}
    m.add_codegen(_blocks)
    m.set_dynamics("flow/d3q27_cumulant.inc")
    return m
