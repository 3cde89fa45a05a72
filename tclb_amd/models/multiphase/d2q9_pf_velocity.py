"""d2q9_pf_velocity — conservative phase-field (Allen-Cahn, h) + velocity-based
pressure-evolution hydrodynamics (g) on D2Q9 for high-density-ratio two-phase flow
(Fakhari, Mitchell, Leonardi, Bolster, PRE 96 053301), with geometric wetting (wall
normals from the solid mask, contact angle radAngle), moving walls, Zu-He style
velocity inlets, drag/lift on Body nodes and interface trackers.
Options (reference OPT="(GF+RT+Outflow+GuoCM+debug+BGK+CM)*autosym"):
  GF  higher-order (Guo) forcing of g;   RT  Ren's temporal term in the phase equilibrium;
  Outflow  convective / Neumann outlets (extra old-population densities);
  debug  momentum and force-budget globals;  BGK  single relaxation time;
  CM  central-moment collisions;  GuoCM  no-op in the reference (accepted);
  autosym  symmetry node types.
Reference: models/multiphase/d2q9_pf_velocity/{Dynamics.R, Dynamics.c.Rt}.
"""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build(gf=False, rt=False, outflow=False, debug=False, bgk=False, cm=False, guocm=False, autosym=0) -> Model:
    m = Model("d2q9_pf_velocity", dims=2, family="multiphase", reference="models/multiphase/d2q9_pf_velocity",
              description="D2Q9 phase-field + velocity-based pressure evolution (high density ratio)")
    for grp in ("g", "h"):
        for i, (x, y) in enumerate(U9):
            m.add_density(f"{grp}[{i}]", x, y, 0, group=grp)
    if outflow:
        for grp in ("gold", "hold"):
            for i in range(9):
                m.add_density(f"{grp}{i}", 0, 0, 0, group=grp)
    m.add_density("nw_x", 0, 0, 0, group="nw", comment="phase field normal at the wall in x direction, pointing into fluid")
    m.add_density("nw_y", 0, 0, 0, group="nw")
    m.add_density("U", 0, 0, 0, group="Vel")
    m.add_density("V", 0, 0, 0, group="Vel")
    m.add_field("PhaseF", stencil2d=1, group="PF")
    if outflow:
        for d in list(m.densities):
            m.add_field(d.field.name, dx=-d.dx - 1, dy=-d.dy)
            m.add_field(d.field.name, dx=-d.dx, dy=-d.dy - 1)
        m.add_field("U", dx=(-1, 0))
        m.add_field("V", dy=(0, -1))
    if rt:
        m.add_field("PhaseOld", group="PF")
        # nw is constant after Init; it is saved every iteration so both buffers hold it
        m.add_stage("PhaseInit", "Init_phase", save_fields=["PF"])
        m.add_stage("WallInit", "Init_wallNorm", save_fields=["nw"])
        m.add_stage("BaseInit", "Init_distributions", save_fields=["g", "h", "Vel"])
        m.add_stage("BaseIter", "calcHydroIter", save_fields=["g", "h", "Vel", "nw"],
                    load_densities=["g", "h", "Vel", "nw"])
        m.add_stage("PhaseIter", "calcPhaseFIter", save_fields=["PhaseF", "PhaseOld"], load_densities=["h"])
        m.add_stage("WallIter", "calcWallPhaseIter", save_fields=["PF"], load_densities=["nw"])
    elif outflow:
        sv = ["g", "h", "Vel", "nw", "gold", "hold"]
        m.add_stage("PhaseInit", "Init_phase", save_fields=["PF"])
        m.add_stage("WallInit", "Init_wallNorm", save_fields=["nw"])
        m.add_stage("BaseInit", "Init_distributions", save_fields=["g", "h", "Vel", "gold", "hold"])
        m.add_stage("BaseIter", "calcHydroIter", save_fields=sv, load_densities=sv)
        m.add_stage("PhaseIter", "calcPhaseFIter", save_fields=["PF"], load_densities=sv)
        m.add_stage("WallIter", "calcWallPhaseIter", save_fields=["PF"], load_densities=["nw"])
    else:
        sv = ["g", "h", "Vel", "nw"]
        m.add_stage("PhaseInit", "Init_phase", save_fields=["PF"])
        m.add_stage("WallInit", "Init_wallNorm", save_fields=["nw"])
        m.add_stage("BaseInit", "Init_distributions", save_fields=["g", "h", "Vel"])
        # keep: the wall normals are written by WallInit only (the reference stores them
        # again in every iteration)
        m.add_stage("BaseIter", "calcHydroIter", save_fields=sv, load_densities=sv, keep=["nw"])
        # lazy: a node without a boundary condition sums its pulled h populations and
        # reads nothing else (PF2_LAZY in the node code); boundary nodes pull every
        # declared density for BC_Switcher, as before
        m.add_stage("PhaseIter", "calcPhaseFIter", save_fields=["PF"], load_densities=sv, lazy_load=True)
        # split: on the GPU only the wall nodes run (node_class_ 2); every other node would
        # store the PhaseF it reads, in place (the stage is never an action's first)
        m.add_stage("WallIter", "calcWallPhaseIter", save_fields=["PF"], load_densities=["nw"], split=True)
        m.defines["PF2_LAZY"] = "1"
        m.add_codegen(lambda _m: "\n".join(f"  static constexpr int FI_{a.upper()}0 = "
                                           f"{[i for i, f in enumerate(_m.fields) if f.array == a][0]};"
                                           for a in ("h",)))
    m.add_action("Iteration", ["BaseIter", "PhaseIter", "WallIter"])
    m.add_action("Init", ["PhaseInit", "WallInit", "WallIter", "BaseInit"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("PhaseField", unit="1")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("NormalizedPressure", unit="Pa")
    m.add_quantity("Pressure", unit="Pa")
    m.add_quantity("Normal", unit="1", vector=True)
    S = m.add_setting
    S("Period", default=0, comment="Number of cells per cos wave")
    S("Perturbation", default=0, comment="Size of wave perturbation, Perturbation Period")
    S("MidPoint", default=0, comment="height of RTI centerline")
    S("Wave", default=0, comment="Used for gravity and capillary wave benchmarks")
    S("Radius", default=0, comment="Radius of diffuse interface circle")
    S("CenterX", default=0, comment="Circle center x-coord")
    S("CenterY", default=0, comment="Circle Center y-coord")
    S("BubbleType", default=1, comment="Drop/bubble")
    S("Density_h", comment="High density fluid")
    S("Density_l", comment="Low  density fluid")
    S("PhaseField_h", default=1, comment="PhaseField in high density fluid")
    S("PhaseField_l", default=0, comment="PhaseField in low density fluid")
    S("PhaseField_init", comment="Initial/Inflow PhaseField distribution", zonal=True)
    S("W", default=4, comment="Anti-diffusivity coeff (phase interfacial thickness) ")
    S("omega_phi", comment="one over relaxation time (phase field)")
    S("M", default=0.02, comment="Mobility", omega_phi="1.0/(3*M+0.5)")
    S("sigma", comment="surface tension")
    S("radAngle", default=1.570796, comment="Contact angle in radians, can use units -> 90d where d=2pi/360",
      zonal=True)
    S("tau_l", comment="relaxation time (low density fluid)")
    S("tau_h", comment="relaxation time (high density fluid)")
    S("Viscosity_l", default=0.16666666, comment="kinematic viscosity", tau_l="(3*Viscosity_l)")
    S("Viscosity_h", default=0.16666666, comment="kinematic viscosity", tau_h="(3*Viscosity_h)")
    S("omega_bulk", default=1.0, comment="inverse of bulk relaxation time")
    S("bulk_visc", comment="bulk viscosity", omega_bulk="1.0/(3*bulk_visc+0.5)")
    S("VelocityX", default=0.0, comment="inlet/outlet/init velocity", zonal=True)
    S("VelocityY", default=0.0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default=0.0, comment="inlet/outlet/init density", zonal=True)
    S("GravitationX", default=0.0, comment="applied (rho)*GravitationX", zonal=True)
    S("GravitationY", default=0.0, comment="applied (rho)*GravitationY", zonal=True)
    S("BuoyancyX", default=0.0, comment="applied (rho-rho_h)*BuoyancyX")
    S("BuoyancyY", default=0.0, comment="applied (rho-rho_h)*BuoyancyY")
    S("fixedIterator", default=2.0, comment="fixed iterator for velocity calculation")
    for g, c, u in (("PressureLoss", "pressure loss", "1mPa"), ("OutletFlux", "pressure loss", "1m2/s"),
                    ("InletFlux", "pressure loss", "1m2/s"), ("TotalDensity", "Mass conservation check", "1kg/m3")):
        m.add_global(g, comment=c, unit=u)
    for n in ("SpikeTrack", "BubbleTrack", "WaveTrack"):
        m.add_node_type(n, "ADDITIONALS")
    m.add_global("RTIBubble", comment="Bubble Tracker", op="MAX")
    m.add_global("RTISpike", comment="Spike Tracker", op="MAX")
    m.add_global("WaveLocation", comment="Wave", op="MAX")
    m.add_global("NMovingWallForce", comment="force exerted on the N Moving Wall")
    m.add_global("NMovingWallPower", comment="implented: Vx* incoming momentum (precollision)")
    for g, c in (("BubbleVelocityX", "Bubble velocity in the x direction"),
                 ("BubbleVelocityY", "Bubble velocity in the y direction"),
                 ("BubbleVelocityZ", "Bubble velocity in the z direction"),
                 ("BubbleLocationY", "Bubble Location in the y direction"),
                 ("SumPhiGas", "Summation of (1-phi) in all gas cells")):
        m.add_global(g, comment=c)
    if debug:
        for g in ("MomentumX", "MomentumY", "MomentumX_afterCol", "MomentumY_afterCol", "F_pressureX", "F_pressureY",
                  "F_bodyX", "F_bodyY", "F_surf_tensionX", "F_surf_tensionY", "F_muX", "F_muY",
                  "F_total_hydroX", "F_total_hydroY", "F_phiX", "F_phiY"):
            m.add_global(g)
    if cm:
        m.add_node_type("CM", "COLLISION")
    m.add_node_type("Smoothing", "ADDITIONALS")
    for n in ("MovingWall_N", "MovingWall_S", "NVelocity", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Body", "BODY")
    m.add_global("FDrag", comment="Force exerted on body in X-direction", unit="N")
    m.add_global("FLift", comment="Force exerted on body in Y-direction", unit="N")
    m.add_global("FTotal", comment="Force exerted on body in X+Y -direction", unit="N")
    if outflow:
        for n in ("Convective_E", "Convective_N", "Neumann_E"):
            m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"GF": gf, "RT": rt, "Outflow": outflow, "GuoCM": guocm, "debug": debug, "BGK": bgk, "CM": cm,
                 "autosym": autosym}
    m.set_color("getPhaseField()")  # reference Color(): PhaseF
    m.set_dynamics("multiphase/d2q9_pf_velocity.inc")
    return m
