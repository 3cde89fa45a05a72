"""d2q9q9_cm_cht — conjugate heat transfer on D2Q9 x D2Q9: cumulant hydrodynamics with
Boussinesq buoyancy and a Darcy stopper in solids, an enthalpy-like population h
(H = rho cp T) relaxed in central moments (CM_HIGHER, CM_HIGHER_PROB,
CM_HIGHER_PROB_M_EQ) or cumulants; Dirichlet (equilibrium / anti-bounce-back /
interpolated ABB) and Neumann heat-flux boundaries, heat sources, flux and force
measurement zones.
Options (reference OPT="OutFlowConvective*OutFlowNeumann*AVG*IBB*SMAG*CHT"):
  CHT  sigma^2 = h_stability_enhancement / (3 cp rho) in the heat equilibria;
  IBB  interpolated (anti-)bounce-back on STL cuts; AVG running averages;
  SMAG Smagorinsky setting; OutFlowConvective / OutFlowNeumann east outlets.
Reference: models/heat/d2q9q9_cm_cht/{Dynamics.R, Dynamics.c.Rt}.
"""
from ..dsl import Model

CV = (0, 1, -1)


def build(outflowconvective=False, outflowneumann=False, avg=False, ibb=False, smag=False, cht=False) -> Model:
    m = Model("d2q9q9_cm_cht", dims=2, family="heat", reference="models/heat/d2q9q9_cm_cht",
              description="D2Q9xD2Q9 conjugate heat transfer (cumulant flow, central-moment heat)")
    for grp, c in (("f", "flow LB density F"), ("h", "heat LB density H")):
        for k in range(9):
            px, py = k % 3, k // 3
            m.add_density(f"{grp}[{k}]", CV[px], CV[py], 0, group=grp, comment=f"{c}{px}{py}0")
    S = m.add_setting
    S("VelocityX", default=0, comment="inlet/outlet/init x-velocity component", zonal=True, unit="m/s")
    S("VelocityY", default=0, comment="inlet/outlet/init y-velocity component", zonal=True, unit="m/s")
    S("Pressure", default=0, comment="inlet/outlet/init pressure", zonal=True, unit="Pa")
    S("GravitationX", default=0.0, comment="applied rho*GravitationX")
    S("GravitationY", default=0.0, comment="applied rho*GravitationY")
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
                    ("FLift", "Force exerted on body in Y-direction", "N"),
                    ("XHydroFLux", "Momentum flux in X-direction", "kg/s"),
                    ("YHydroFLux", "Momentum flux in Y-direction", "kg/s"),
                    ("XHydroFLux2", "Momentum flux (2nd logger) in X-direction", "kg/s"),
                    ("YHydroFLux2", "Momentum flux (2nd logger) in Y-direction", "kg/s"),
                    ("HeatFluxX", "Heat flux in X-direction", "W"), ("HeatFluxY", "Heat flux in Y-direction", "W"),
                    ("HeatFluxX2", "Heat flux (2nd logger) in X-direction", "W"),
                    ("HeatFluxY2", "Heat flux (2nd logger) in Y-direction", "W"),
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
    for n in ("CM", "CM_HIGHER", "CM_HIGHER_PROB", "CM_HIGHER_PROB_M_EQ", "Cumulants"):
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
        for grp in ("hold", "fold"):
            for k in range(9):
                m.add_density(f"{grp}{k}", 0, 0, 0, group=grp)
        for d in list(m.densities):
            m.add_field(d.field.name, dx=-d.dx - 1, dy=-d.dy)
        m.add_field("U", dx=(-1, 0))
        m.add_node_type("EConvective", "BOUNDARY")
    if outflowneumann:
        for d in list(m.densities):
            m.add_field(d.field.name, dx=-d.dx - 1, dy=-d.dy)
        m.add_node_type("ENeumann", "BOUNDARY")
    if avg:
        for q, u, v in (("KinE", None, False), ("ReStr", None, True), ("Dissipation", None, False),
                        ("averageU", "m/s", True), ("varU", None, True), ("averageP", "Pa", False),
                        ("averageT", "K", False)):
            m.add_quantity(q, unit=u or "1", vector=v)
        for n in ("avgT", "avgP", "varUX", "varUY", "varUXUY", "avgdxu2", "avgdyv2", "avgUX", "avgUY"):
            m.add_density(n, 0, 0, 0, group="avg", average=True)
        m.add_field("avgUX", dx=(-1, 1), average=True)
        m.add_field("avgUY", dy=(-1, 1), average=True)
    for n in ("EPressure", "Solid", "Wall", "WVelocity", "Lid"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Body", "BODY")
    m.options = {"OutFlowConvective": outflowconvective, "OutFlowNeumann": outflowneumann, "AVG": avg,
                 "IBB": ibb, "SMAG": smag, "CHT": cht}
    m.set_dynamics("heat/d2q9q9_cm_cht.inc")
    return m
