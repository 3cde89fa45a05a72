"""d3q27q7_cm_cht — conjugate heat transfer on D3Q27 x D3Q7: cumulant hydrodynamics
(Galilean-corrected, third cumulants relaxed with Omegafor3rdCumulants, optional
Smagorinsky) with Boussinesq buoyancy about T_ref = 10 and a Darcy stopper in solids,
coupled to an enthalpy population h (H = rho cp T) on D3Q7 relaxed in central moments
(CM: odd moments about the fluid velocity, CM_PROB: equilibrium about a velocity blended
from the h and fluid velocities, BGK: single relaxation to the central-moment
equilibrium). Dirichlet (equilibrium / anti-bounce-back / interpolated ABB) and Neumann
heat-flux heaters, heat sources, force and flux measurement zones, non-equilibrium
bounce-back W/E planes that impose the inflow temperature.
Options (reference OPT="OutFlowConvective*OutFlowNeumann*AVG*IBB*SMAG*CHT"):
  CHT  sigma^2 = h_stability_enhancement / (3 cp rho) in the heat equilibria;
  IBB  interpolated (anti-)bounce-back on STL cuts; AVG running averages;
  SMAG Smagorinsky eddy viscosity; OutFlowConvective / OutFlowNeumann east outlets.
heat_q=27 (d3q27q27_cm_cht): CM_HIGHER_PROB, CM_HIGHER_PROB_M_EQ and the cumulant heat
collisions normalise by H = sum(h) (k[1]/k[0], cum_raw2cum), as the reference does
(h100/h000): a node with H = 0 (the default InitTemperature = 0) turns NaN and spreads it
by streaming.  Initialise a nonzero temperature before using them.
Reference: models/heat/d3q27q7_cm_cht/{Dynamics.R:1-224, Dynamics.c.Rt:247-1487}.
"""
import numpy as np

from ..dsl import Model
from ...emit.blocks import tensor_raw_transform
from ...emit.cumulants import cumulant_block

CV = (0, 1, -1)
P = np.array([[k % 3, (k // 3) % 3, k // 9] for k in range(27)])
U = np.array([[CV[a], CV[b], CV[c]] for a, b, c in P])
# reference hname order h000 h100 h200 h010 h020 h001 h002 (lib/lattice.R d3q7)
U7 = np.array([[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]])


def _blocks(_m):
    return "\n".join([
        tensor_raw_transform("raw_moments", U, P, inverse=False),
        tensor_raw_transform("raw_inverse", U, P, inverse=True),
        cumulant_block("cum", 3, drop_order_above=3),
    ])


def build(outflowconvective=False, outflowneumann=False, avg=False, ibb=False, smag=False, cht=False,
          heat_q=7) -> Model:
    """heat_q = 7: d3q27q7_cm_cht; heat_q = 27: d3q27q27_cm_cht (reference
    models/heat/d3q27q27_cm_cht/Dynamics.R, same settings/globals/zones, D3Q27 heat set and
    the CM_HIGHER / CM_HIGHER_PROB / CM_HIGHER_PROB_M_EQ / Cumulants / Cumulants_HIGHER
    collisions)."""
    name = f"d3q27q{heat_q}_cm_cht"
    m = Model(name, dims=3, family="heat", reference=f"models/heat/{name}",
              description=f"D3Q27xD3Q{heat_q} conjugate heat transfer (cumulant flow, central-moment heat)")
    HU = U7 if heat_q == 7 else U
    for k in range(27):
        m.add_density(f"f[{k}]", int(U[k, 0]), int(U[k, 1]), int(U[k, 2]), group="f",
                      comment=f"flow LB density F{P[k, 0]}{P[k, 1]}{P[k, 2]}")
    for i, c in enumerate(HU):
        m.add_density(f"h[{i}]", int(c[0]), int(c[1]), int(c[2]), group="h", comment=f"heat LB density H{i}")
    S = m.add_setting
    for a in "XYZ":
        S(f"Velocity{a}", default=0, comment=f"inlet/outlet/init {a.lower()}-velocity component", zonal=True,
          unit="m/s")
    S("Pressure", default=0, comment="inlet/outlet/init pressure", zonal=True, unit="Pa")
    for a in "XYZ":
        S(f"Gravitation{a}", default=0.0, comment=f"applied rho*Gravitation{a}")
    S("nu", default=0.16666666, comment="kinematic viscosity")
    S("GalileanCorrection", default=1.0, comment="Galilean correction term")
    S("nu_buffer", default=0.01, comment="kinematic viscosity in the buffer layer")
    S("conductivity_buffer", default=0.01, comment="thermal conductivity in the buffer layer")
    S("Omegafor3rdCumulants", default=1, comment="relaxation rate for 3rd order cumulants")
    S("h_stability_enhancement", default=1.0, comment="magic stability enhancement")
    S("InitTemperature", default=0, comment="Initial/Inflow temperature distribution", zonal=True)
    S("InitHeatFlux", default=0, comment="Initial/Inflow heat flux through boundary", zonal=True)
    S("conductivity", default=0.16666666, comment="thermal conductivity of fluid (W/(m K))", zonal=True)
    S("material_density", default=1.0, comment="density of material [kg/m3]", zonal=True)
    S("cp", default=1.0, comment="specific heat capacity at constant pressure of fluid (J/(kg K))", zonal=True)
    S("BoussinesqCoeff", default=1.0, comment="BoussinesqCoeff=rho_0*thermal_exp_coeff")
    for g, c, u in (("FDrag", "Force exerted on body in X-direction", "N"),
                    ("FLateral", "Force exerted on body in Y-direction", "N"),
                    ("FLift", "Force exerted on body in Z-direction", "N"),
                    ("XHydroFLux", "Momentum flux in X-direction", "kg/s"),
                    ("YHydroFLux", "Momentum flux in Y-direction", "kg/s"),
                    ("ZHydroFLux", "Momentum flux in Z-direction", "kg/s"),
                    ("XHydroFLux2", "Momentum flux (2nd logger) in X-direction", "kg/s"),
                    ("YHydroFLux2", "Momentum flux (2nd logger) in Y-direction", "kg/s"),
                    ("ZHydroFLux2", "Momentum flux (2nd logger) in Z-direction", "kg/s"),
                    ("HeatFluxX", "Heat flux in X-direction", "W"), ("HeatFluxY", "Heat flux in Y-direction", "W"),
                    ("HeatFluxZ", "Heat flux in Z-direction", "W"),
                    ("HeatFluxX2", "Heat flux (2nd logger) in X-direction", "W"),
                    ("HeatFluxY2", "Heat flux (2nd logger) in Y-direction", "W"),
                    ("HeatFluxZ2", "Heat flux (2nd logger) in Z-direction", "W"),
                    ("HeatSource", "Total Heat flux from body", "W")):
        m.add_global(g, comment=c, unit=u)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("H", unit="J")
    m.add_quantity("T", unit="K")
    m.add_quantity("m00_F")
    m.add_quantity("material_density", unit="kg/m3")
    m.add_quantity("cp", unit="J/kg/K")
    m.add_quantity("conductivity", unit="W/m/K")
    m.add_quantity("RawU", unit="m/s", vector=True)
    m.add_node_type("ForceMeasurmentZone", "OBJECTIVEFORCE")
    m.add_node_type("FluxMeasurmentZone1", "OBJECTIVEFLUX")
    m.add_node_type("FluxMeasurmentZone2", "OBJECTIVEFLUX")
    m.add_node_type("DarcySolid", "ADDITIONALS")
    m.add_node_type("Smoothing", "ADDITIONALS")
    for n in ("HeaterDirichletTemperatureEQ", "HeaterDirichletTemperatureABB", "HeaterSource",
              "HeaterNeumannHeatFluxCylinder", "HeaterNeumannHeatFluxEast"):
        m.add_node_type(n, "ADDITIONALS_HEAT")
    if heat_q == 7:
        m.add_node_type("CM", "COLLISION")
        m.add_node_type("CM_PROB", "COLLISION")
    else:
        # reference registration order (models/heat/d3q27q27_cm_cht/Dynamics.R:114-119):
        # flag values follow it, so raw NodeType dumps match the reference's
        for n in ("CM", "CM_HIGHER", "CM_HIGHER_PROB", "CM_HIGHER_PROB_M_EQ", "Cumulants", "Cumulants_HIGHER"):
            m.add_node_type(n, "COLLISION")
    S("CylinderCenterX", default=0, comment="X coord of cylinder with imposed heat flux")
    S("CylinderCenterY", default=0, comment="Y coord of cylinder with imposed heat flux")
    S("CylinderCenterX_GH", default=0, comment="X coord of Gaussian Hill")
    S("CylinderCenterY_GH", default=0, comment="Y coord of Gaussian Hill")
    S("Sigma_GH", default=1, comment="Initial width of the Gaussian Hill", zonal=True)
    if ibb:
        m.add_node_type("HeaterDirichletTemperatureIABB", "HO_BOUNDARY_HEAT")
        m.add_node_type("ThermalIBB", "HO_BOUNDARY_HEAT")
        m.add_node_type("HydroIBB", "HO_BOUNDARY_HYDRO")
    if smag:
        S("Smag", default=0, comment="Smagorinsky coefficient for SGS modeling")
    m.add_density("U", 0, 0, 0, group="Vel")
    if outflowconvective:
        for k in range(heat_q):
            m.add_density(f"hold[{k}]", 0, 0, 0, group="hold", comment=f"heat LB density H{k}")
        for k in range(27):
            m.add_density(f"fold[{k}]", 0, 0, 0, group="fold", comment=f"flow LB density F{k}")
        for d in list(m.densities):
            m.add_field(d.field.name, dx=-d.dx - 1, dy=-d.dy, dz=-d.dz)
        m.add_field("U", dx=(-1, 0))
        m.add_node_type("EConvective", "BOUNDARY")
    if outflowneumann:
        for d in list(m.densities):
            m.add_field(d.field.name, dx=-d.dx - 1, dy=-d.dy, dz=-d.dz)
        m.add_node_type("ENeumann", "BOUNDARY")
    if avg:
        for q, u, v in (("KinE", None, False), ("ReStr", None, True), ("Dissipation", None, False),
                        ("averageU", "m/s", True), ("varU", None, True), ("averageP", "Pa", False),
                        ("averageT", "K", False)):
            m.add_quantity(q, unit=u or "1", vector=v)
        for n in ("avgT", "avgP", "varUX", "varUY", "varUZ", "varUXUY", "varUXUZ", "varUYUZ", "avgdxu2",
                  "avgdyv2", "avgdzw2", "avgUX", "avgUY", "avgUZ"):
            m.add_density(n, 0, 0, 0, group="avg", average=True)
        m.add_field("avgUX", dx=(-1, 1), average=True)
        m.add_field("avgUY", dy=(-1, 1), average=True)
        m.add_field("avgUZ", dz=(-1, 1), average=True)
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("Body", "BODY")
    m.options = {"OutFlowConvective": outflowconvective, "OutFlowNeumann": outflowneumann, "AVG": avg,
                 "IBB": ibb, "SMAG": smag, "CHT": cht}
    m.add_codegen(_blocks)
    m.set_dynamics(f"heat/{name}.inc")
    # no cap: the globals kernels sit at 256+ VGPRs, a 2-wave cap spilled 8-116 B/lane
    # (profiles/README.md r03s); with LDS accumulators they cost what the plain ones do
    m.glob_waves = 0
    return m
