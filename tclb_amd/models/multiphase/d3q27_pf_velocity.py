"""d3q27_pf_velocity — conservative phase-field (Allen-Cahn) + velocity-based
pressure-evolution LBM for high-density-ratio two-phase flow: hydrodynamics on D3Q27
(weighted-MRT in the 27-moment basis of the reference), interface on D3Q15 (or D3Q27
with ``q27``).  Two distribution sets g (27) and h (15/27) + macroscopic/wall fields.

Reference: models/multiphase/d3q27_pf_velocity/{Dynamics.R, model.R, Dynamics.c.Rt,
Boundary.c.Rt, thermocapillary.R, thermo.c.Rt}.  Implemented options: ``q27``, ``BGK``,
``OutFlow`` (Neumann / convective E,W outflow with the gold/hold history sets),
``thermo`` (temperature field by explicit RK4 with phase-dependent conductivity and heat
capacity; surface tension sigma(T) enters the chemical potential and a Marangoni force),
``planarBenchmark`` (heated-wall layered benchmark initialisation, with ``thermo``) and
``autosym`` (1/2), and the wetting-boundary options of Boundary.c.Rt: ``geometric``
(geometric contact-angle condition from the tangential phase gradient extrapolated from
two nodes along the wall normal, with the gradient stages calcPhaseGrad[_init]),
``staircaseimp`` (the wall normal is the exact surface normal, extended to the D3Q27 cube
surface; values along it are interpolated barycentrically on the hit triangle of the cube
face), ``isograd`` (isotropic gradients near walls from the previous iteration) and
``tprec`` (a second, smaller triangle for the second interpolation point).

Build-time derivations (sympy, replacing the reference's R polynomial algebra):
* the 27x27 moment matrix M factorises as M = C . Mraw, Mraw the raw-monomial
  tensor transform (3 axis passes) and C a 75-non-zero coefficient matrix, so the
  moment transforms cost O(Q D) + 75 FMAs instead of 2 x 416;
* equilibrium moments in the M basis (MRT_eq(..., mat=t(M)), Req[0] <- p);
* stress of the non-equilibrium part (second moments of M^-1 m) as a 6-row map;
* the 12 face boundary conditions (velocity / pressure on N,E,S,W,F,B) for g and h,
  straight-line and CSE'd, exactly as Boundary.c.Rt:31-108 assembles them.
"""
import itertools

import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.blocks import dense_transform, exprs_function, tensor_raw_transform
from ...emit.cprint import assign_block
from ...emit.symbolic import mrt_eq

# reference lattice.R ordering (g0..g26; h uses the first 15 or all 27)
U27 = np.array([[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1],
                [1, 1, 1], [-1, 1, 1], [1, -1, 1], [-1, -1, 1], [1, 1, -1], [-1, 1, -1], [1, -1, -1],
                [-1, -1, -1], [1, 1, 0], [-1, 1, 0], [1, -1, 0], [-1, -1, 0], [1, 0, 1], [-1, 0, 1],
                [1, 0, -1], [-1, 0, -1], [0, 1, 1], [0, -1, 1], [0, 1, -1], [0, -1, -1]])
FACES = [("N", (0, 1, 0)), ("E", (1, 0, 0)), ("S", (0, -1, 0)), ("W", (-1, 0, 0)),
         ("F", (0, 0, 1)), ("B", (0, 0, -1))]


def moment_matrix() -> sp.Matrix:
    """rows m0..m26 of model.R:16-44 evaluated on U27 (M[k, i])."""
    X, Y, Z = sp.symbols("x y z")
    a2 = X ** 2 + Y ** 2 + Z ** 2
    h = sp.Rational(1, 2)
    rows = [sp.Integer(1), X, Y, Z, X * Y, Y * Z, Z * X, 3 * X ** 2 - a2, Y ** 2 - Z ** 2, a2 - 1,
            X * (3 * a2 - 5), Y * (3 * a2 - 5), Z * (3 * a2 - 5),
            X * (Y ** 2 - Z ** 2), Y * (Z ** 2 - X ** 2), Z * (X ** 2 - Y ** 2), X * Y * Z,
            h * (3 * a2 ** 2 - 7 * a2 + 2), (3 * a2 - 4) * (3 * X ** 2 - a2), (3 * a2 - 4) * (Y ** 2 - Z ** 2),
            X * Y * (3 * a2 - 7), Y * Z * (3 * a2 - 7), Z * X * (3 * a2 - 7),
            h * X * (9 * a2 ** 2 - 33 * a2 + 26), h * Y * (9 * a2 ** 2 - 33 * a2 + 26),
            h * Z * (9 * a2 ** 2 - 33 * a2 + 26), h * (9 * a2 ** 3 - 36 * a2 ** 2 + 33 * a2 - 2)]
    return sp.Matrix([[r.subs({X: int(u[0]), Y: int(u[1]), Z: int(u[2])}) for u in U27] for r in rows])


def _raw_basis():
    P = np.array([p for p in itertools.product(range(3), repeat=3)])[:, ::-1]   # a fastest
    Mraw = sp.Matrix([[int(np.prod([int(u[d]) ** int(p[d]) for d in range(3)])) for u in U27] for p in P])
    return P, Mraw


def _bounce(U):
    idx = {tuple(r): i for i, r in enumerate(U.tolist())}
    return [idx[tuple((-np.array(r)).tolist())] for r in U.tolist()]


def build(q27: bool = False, bgk: bool = False, thermo: bool = False, planarbenchmark: bool = False,
          outflow: bool = False, autosym: int = 0, geometric: bool = False, staircaseimp: bool = False,
          isograd: bool = False, tprec: bool = False) -> Model:
    if thermo and geometric:
        # Dynamics.R:155-169: with thermo the actions use the surface-energy stages
        # (WallInit, calcWall), which geometric renames to *_CA: no buildable variant
        raise NotImplementedError("thermo with geometric has no actions in the reference (Dynamics.R:155-169)")
    m = Model("d3q27_pf_velocity", dims=3, family="multiphase", reference="models/multiphase/d3q27_pf_velocity",
              description="phase-field (D3Q15/D3Q27 h) + velocity-based hydrodynamics (D3Q27 g), "
                          "weighted-MRT, high density ratio")
    Qh = 27 if q27 else 15
    # ---- densities / fields (Dynamics.R:11-96, lattice.R)
    for n in ("Init_UX_External", "Init_UY_External", "Init_UZ_External", "Init_PhaseField_External"):
        m.add_density(n, 0, 0, 0, group="init", parameter=True)
    for n in ("pnorm", "U", "V", "W"):
        m.add_density(n, 0, 0, 0, group="Vel")
    for n in ("nw_x", "nw_y", "nw_z"):
        m.add_density(n, 0, 0, 0, group="nw")
    extra_save, extra_load, extra_phase, extra_bc = [], [], [], []
    if staircaseimp:        # Dynamics.R:36-61
        for n in ("nw_actual_x", "nw_actual_y", "nw_actual_z"):
            m.add_density(n, 0, 0, 0, group="nw_actual")
        for n in ("coeff_v1", "coeff_v2", "coeff_v3", "triangle_index"):
            m.add_density(n, 0, 0, 0, group="st_interpolation")
        if tprec:
            for n in ("coeff2_v1", "coeff2_v2", "coeff2_v3", "triangle_index2"):
                m.add_density(n, 0, 0, 0, group="st_interpolation")
        extra_save = ["nw_actual", "st_interpolation"]
        extra_load = ["nw_actual", "st_interpolation"]
        extra_phase = ["nw_actual"]
        extra_bc = ["nw_actual", "st_interpolation"]
    m.add_density("IsSpecialBoundaryPoint", 0, 0, 0, group="solid_boundary")
    m.add_quantity("SpecialBoundaryPoint", unit="1")
    m.add_field("IsBoundary", stencil3d=2 if geometric else 1, group="solid_boundary")
    if geometric:           # Dynamics.R:93-109: gradients read two nodes along the normal
        for n in ("gradPhiVal_x", "gradPhiVal_y", "gradPhiVal_z"):
            m.add_field(n, stencil3d=2, group="gradPhi")
        m.add_field("gradPhi_PhaseF", stencil3d=1, group="gradPhi")
    m.add_field("PhaseF", stencil3d=2 if geometric else 1, group="PF")
    for i, u in enumerate(U27):
        m.add_density(f"g[{i}]", int(u[0]), int(u[1]), int(u[2]), group="g")
    for i, u in enumerate(U27[:Qh]):
        m.add_density(f"h[{i}]", int(u[0]), int(u[1]), int(u[2]), group="h")

    save_initial_PF = ["PF", "Vel"]
    save_initial = ["g", "h", "PF"]
    save_iteration = ["g", "h", "Vel", "nw", "solid_boundary"] + extra_save
    load_iteration = ["g", "h", "Vel", "nw", "solid_boundary"] + extra_load
    load_phase = ["g", "h", "Vel", "nw", "solid_boundary"] + extra_phase
    if outflow:
        # Dynamics.R:65-79 + lattice.R:63-66: every density readable one node east/west of
        # its pull location (Neumann / convective outflow), U readable at x+-1, and the
        # previous post-collision populations (gold/hold) carried for the convective BC
        for d in list(m.densities):
            m.add_field(d.field.name, dx=-d.dx - 1, dy=-d.dy, dz=-d.dz)
            m.add_field(d.field.name, dx=-d.dx + 1, dy=-d.dy, dz=-d.dz)
        m.add_field("U", dx=(-1, 1))
        for i in range(27):
            m.add_density(f"gold[{i}]", 0, 0, 0, group="gold")
        for i in range(Qh):
            m.add_density(f"hold[{i}]", 0, 0, 0, group="hold")
        save_initial += ["gold", "hold"]
        save_iteration += ["gold", "hold"]
        load_iteration += ["gold", "hold"]
        load_phase += ["gold", "hold"]
    if thermo:
        _thermo_declarations(m, planarbenchmark)
        save_initial_PF = save_initial_PF + ["Thermal"]
        # the collision stores the temperature and surface tension that the RK stages of
        # the same step read; it keeps (does not store) the conductivity, set at
        # initialisation only, and the RK iterates, which the RK stages rewrite before any read
        save_iteration += ["Temp", "SurfaceTension", "Cond", "RK1", "RK2", "RK3"]
        load_iteration += ["Thermal"]
    m.add_stage("PhaseInit", "Init", save_fields=save_initial_PF)
    m.add_stage("BaseInit", "Init_distributions", save_fields=save_initial)
    m.add_stage("calcPhase", "calcPhaseF", save_fields=["PhaseF"], load_densities=load_phase, lazy_load=True)
    # (the collision's PhaseF stencil stays on global loads: an LDS tile of it made the
    # latency-bound collision 7-10 % slower, profiles/README.md r04a)
    # lazy: Run pulls the populations where the interior MRT collision needs them; split:
    # that path and the boundary closures run as two kernels (their own register budgets)
    # keep: the wall normals and boundary markers are set by the wall-init stages only
    # (Init_wallNorm); the collision reads them where it needs them and never stores them
    m.add_stage("BaseIter", "Run", save_fields=save_iteration, load_densities=load_iteration, lazy_load=True,
                split=not (bgk or outflow or autosym or staircaseimp),   # = PF_LAZY_INTERIOR
                keep=["nw", "solid_boundary"] + (["Cond", "RK1", "RK2", "RK3"] if thermo else []))
    m.add_stage("InitFromFieldsStage", "InitFromFieldsStage", save_fields=save_initial_PF, load_densities=["init"])
    if geometric:           # Dynamics.R:129-135
        m.add_stage("WallInit_CA", "Init_wallNorm", save_fields=["nw", "solid_boundary"] + extra_bc)
        m.add_stage("calcWall_CA", "calcWallPhase", save_fields=["PhaseF"],
                    load_densities=["nw", "gradPhi", "PF", "solid_boundary"] + extra_bc, lazy_load=True)
        m.add_stage("calcPhaseGrad", "calcPhaseGrad", save_fields=["gradPhi"],
                    load_densities=["nw", "PF", "solid_boundary"])
        m.add_stage("calcPhaseGrad_init", "calcPhaseGrad_init", save_fields=["gradPhi"],
                    load_densities=["nw", "PF", "solid_boundary"])
    else:
        m.add_stage("WallInit", "Init_wallNorm", save_fields=["nw", "solid_boundary"] + extra_bc)
        m.add_stage("calcWall", "calcWallPhase", save_fields=["PhaseF"],
                    load_densities=["nw", "solid_boundary"] + extra_bc, lazy_load=True)
    m.add_stage("calcWallPhase_correction", "calcWallPhase_correction", save_fields=["PhaseF"],
                load_densities=["nw", "solid_boundary"], lazy_load=True)
    if thermo:
        # the thermal collide runs 7 % faster with the row-form addressing in its plain
        # kernels too (profiles/README.md r04s; build.py _cmd model flags)
        m.hip_flags = ["-DTCLB_ROW_ADDR_PLAIN=1"]
        # Dynamics.R:124-134, 142-147 (explicit RK4 of the energy equation)
        T3 = ["Temp", "Cond", "SurfaceTension"]
        m.add_stage("CopyDistributions", "TempCopy", save_fields=["g", "h", "Vel", "nw", "PF", "Thermal"])
        m.add_stage("CopyThermal", "ThermalCopy", save_fields=T3, load_densities=T3)
        # the RK stages are two 27-point stencils (the stage's temperature iterate and the
        # conductivity) per node: both staged in LDS tiles on the GPU
        m.add_stage("RK_1", "TempUpdate1", save_fields=["RK1"], load_densities=["U", "V", "W", "Cond", "Temp"],
                    lds=["Temp", "Cond"])
        m.add_stage("RK_2", "TempUpdate2", save_fields=["RK2"],
                    load_densities=["U", "V", "W", "RK1", "Cond", "Temp"], lds=["RK1", "Cond"])
        m.add_stage("RK_3", "TempUpdate3", save_fields=["RK3"],
                    load_densities=["U", "V", "W", "RK1", "RK2", "Cond", "Temp"], lds=["RK2", "Cond"])
        m.add_stage("RK_4", "TempUpdate4", save_fields=["Temp", "SurfaceTension"],
                    load_densities=["U", "V", "W", "RK1", "RK2", "RK3", "Cond", "Temp"], lds=["RK3", "Cond"])
        # split: on the GPU the stage runs on the EAdiabatic nodes only (node_class_)
        m.add_stage("NonLocalTemp", "BoundUpdate", save_fields=["Temp", "SurfaceTension"], load_densities=["Temp"],
                    split=True)
        rk = ["RK_1", "RK_2", "RK_3", "RK_4", "NonLocalTemp"]
        m.add_action("TempToSteadyState", ["CopyDistributions"] + rk)
        m.add_action("Iteration", ["BaseIter", "calcPhase", "calcWall"] + rk)
        m.add_action("IterationConstantTemp", ["BaseIter", "calcPhase", "calcWall", "CopyThermal"])
        m.add_action("Init", ["PhaseInit", "WallInit", "calcWall", "BaseInit"])
    elif geometric:         # Dynamics.R:160-164
        grad = "calcPhaseGrad" if isograd else "calcPhaseGrad_init"
        m.add_action("Iteration", ["BaseIter", "calcPhase", grad, "calcWall_CA", "calcWallPhase_correction"])
        m.add_action("Init", ["PhaseInit", "WallInit_CA", "calcPhaseGrad_init", "calcWall_CA",
                              "calcWallPhase_correction", "BaseInit"])
        m.add_action("InitFields", ["InitFromFieldsStage", "WallInit_CA", "calcPhaseGrad_init", "calcWall_CA",
                                    "calcWallPhase_correction", "BaseInit"])
    else:
        m.add_action("Iteration", ["BaseIter", "calcPhase", "calcWall", "calcWallPhase_correction"])
        m.add_action("Init", ["PhaseInit", "WallInit", "calcWall", "calcWallPhase_correction", "BaseInit"])
        m.add_action("InitFields", ["InitFromFieldsStage", "WallInit", "calcWall", "calcWallPhase_correction",
                                    "BaseInit"])
    # ---- quantities
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("PhaseField", unit="1")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("P", unit="Pa")
    m.add_quantity("Pstar", unit="1")
    m.add_quantity("Normal", unit="1", vector=True)
    m.add_quantity("IsItBoundary", unit="1")
    if geometric:
        m.add_quantity("GradPhi", unit="1", vector=True)
    if staircaseimp:
        m.add_quantity("ActualNormal", unit="1", vector=True)
    # ---- settings (Dynamics.R:185-245)
    S = m.add_setting
    S("Density_h", comment="High density")
    S("Density_l", comment="Low  density")
    S("PhaseField_h", default=1, comment="PhaseField in Liquid")
    S("PhaseField_l", default=0, comment="PhaseField gas")
    S("PhaseField", comment="Initial PhaseField distribution", zonal=True)
    S("IntWidth", default=4, comment="Anti-diffusivity coeff")
    S("omega_phi", comment="one over relaxation time (phase field)")
    S("M", default=0.02, comment="Mobility", omega_phi="1.0/(3*M+0.5)")
    S("sigma", comment="surface tension")
    S("force_fixed_iterator", default=2, comment="to resolve implicit relation of viscous force")
    S("Washburn_start", default=0, comment="Start of washburn gas phase")
    S("Washburn_end", default=0, comment="End of washburn gas phase")
    S("radAngle", default="1.570796", comment="Contact angle in radians, can use units -> 90d where d=2pi/360",
      zonal=True)
    S("minGradient", default="1e-8", comment="if the phase gradient is less than this, set phase normals to zero")
    S("RTI_Characteristic_Length", default=-999, comment="Use for RTI instability")
    S("pseudo2D", default=0, comment="if 1, assume model is pseduo2D")
    S("Radius", default=0.0, comment="Diffuse Sphere Radius")
    S("CenterX", default=0.0, comment="Diffuse sphere center_x")
    S("CenterY", default=0.0, comment="Diffuse sphere center_y")
    S("CenterZ", default=0.0, comment="Diffuse sphere center_z")
    S("BubbleType", default=1.0, comment="droplet(1.0) or bubble(-1.0)?!")
    S("DonutTime", default=0.0, comment="Radius of a Torus - initialised to travel along x-axis")
    S("Donut_h", default=0.0, comment="Half donut thickness, i.e. the radius of the cross-section")
    S("Donut_D", default=0.0, comment="Dilation factor along the x-axis")
    S("Donut_x0", default=0.0, comment="Position along x-axis")
    S("HEIGHT", default=0, comment="Height of channel for 2D Poiseuille flow")
    S("Uavg", default=0, zonal=True, comment="Average velocity of channel for 2D Poiseuille flow")
    S("developedFlow", default=0, comment="set greater than 0 for fully developed flow in the domain (x-direction)")
    S("developedPipeFlow", default=0, comment="set greater than 0 for fully developed pipe flow in the inlets")
    S("developedPipeFlow_X", default=0,
      comment="set greater than 0 for fully developed pipe flow in the domain (x-direction-only)")
    S("pipeRadius", default=0, comment="radius of pipe for developed pipe flow")
    S("pipeCentre_Y", default=0, comment="pipe centre Y co-ord for developed pipe flow")
    S("pipeCentre_Z", default=0, comment="pipe centre Z co-ord for developed pipe flow")
    S("tau_l", comment="relaxation time (low density fluid)")
    S("tau_h", comment="relaxation time (high density fluid)")
    S("tauUpdate", default=1, comment="Interpolation: 1-linear, 2- inverse, 3- dyn viscosity")
    S("Viscosity_l", default=0.16666666, comment="kinematic viscosity", tau_l="(3*Viscosity_l)")
    S("Viscosity_h", default=0.16666666, comment="kinematic viscosity", tau_h="(3*Viscosity_h)")
    for a in "XYZ":
        S(f"Velocity{a}", default=0.0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default=0.0, comment="inlet/outlet/init density", zonal=True)
    for a in "XYZ":
        S(f"Gravitation{a}", default=0.0, comment=f"applied (rho)*Gravitation{a}")
    for a in "XYZ":
        S(f"Buoyancy{a}", default=0.0, comment=f"applied (rho_h-rho)*Buoyancy{a}")
    S("xyzTrack", default=1, comment="x<-1, y<-2, z<-3")
    # ---- node types
    for n in ("Centerline", "Spiketrack", "Saddletrack", "Bubbletrack"):
        m.add_node_type(n, "ADDITIONALS")
    # ---- globals (order of the reference)
    m.add_global("InterfacePosition", op="MAX", comment="trackPosition")
    m.add_global("InterfaceYTop", op="MAX", comment="Track top position of the interface in Y direction")
    m.add_global("Vfront", comment="velocity infront of bubble")
    m.add_global("Vback", comment="velocity behind bubble")
    m.add_global("RTISpike", op="MAX", comment="SpikeTracker ")
    m.add_global("RTIBubble", op="MAX", comment="BubbleTracker")
    m.add_global("RTISaddle", op="MAX", comment="SaddleTracker")
    m.add_global("XLocation", comment="tracking of x-centroid of the gas regions in domain", unit="m")
    m.add_global("DropFront", op="MAX", comment="Highest location of droplet", unit="m")
    m.add_node_type("Smoothing", "ADDITIONALS")
    m.add_node_type("flux_nodes", "ADDITIONALS")
    for f, _ in FACES:
        m.add_node_type(f"{f}Velocity", "BOUNDARY")
        m.add_node_type(f"{f}Pressure", "BOUNDARY")
    for n in ("MovingWall_N", "MovingWall_S", "Solid", "Wall"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    if outflow:
        for n in ("ENeumann", "WNeumann", "EConvect", "WConvect"):
            m.add_node_type(n, "BOUNDARY")
    for g, u in [("PressureLoss", "1mPa"), ("OutletFlux", "1m2/s"), ("InletFlux", "1m2/s"),
                 ("TotalDensity", "1kg/m3"), ("KineticEnergy", "J"), ("GasTotalVelocity", "m/s"),
                 ("GasTotalVelocityX", "m/s"), ("GasTotalVelocityY", "m/s"), ("GasTotalVelocityZ", "m/s"),
                 ("GasTotalPhase", "1"), ("LiqTotalVelocity", "m/s"), ("LiqTotalVelocityX", "m/s"),
                 ("LiqTotalVelocityY", "m/s"), ("LiqTotalVelocityZ", "m/s"), ("NumFluidCells", "1"),
                 ("NumSpecialPoints", "1"), ("NumWallBoundaryPoints", "1"), ("NumBoundaryPoints", "1"),
                 ("LiqTotalPhase", "1"), ("FluxNodeCount", "1"), ("FluxX", "1"), ("FluxY", "1"), ("FluxZ", "1")]:
        m.add_global(g, unit=u)
    m.options = {"q27": q27, "BGK": bgk, "OutFlow": outflow, "thermo": thermo,
                 "planarBenchmark": planarbenchmark, "autosym": autosym, "geometric": geometric,
                 "staircaseimp": staircaseimp, "isograd": isograd, "tprec": tprec}
    m.defines["hPops"] = str(Qh)
    m.add_codegen(lambda _m: codegen(Qh))
    m.add_codegen(_field_index_block)
    m.set_color("getPhaseField()")  # reference Color(): PhaseF, 0 on Solid
    m.set_dynamics("multiphase/d3q27_pf_velocity.inc")
    # GLOB kernels of the thermo / OutFlow variants need 310-370 VGPRs: a 2-wave cap would
    # spill a quarter of them; the plain pf_velocity (250-266) gains 1.5x from it
    # no occupancy cap on the globals kernels: with the accumulators in LDS they need about
    # the VGPRs of the plain kernels (226 vs 197); a 2-wave cap made the BGK and q27
    # variants spill 12-92 B/lane (profiles/README.md r03s)
    m.glob_waves = 0
    return m


def _field_index_block(m: Model) -> str:
    """field indices of the first g / h / gold / hold population (runtime-indexed reads)"""
    out = []
    for arr in ("g", "h", "gold", "hold"):
        idx = [i for i, f in enumerate(m.fields) if f.array == arr]
        if idx:
            assert idx == list(range(idx[0], idx[0] + len(idx)))
            out.append(f"  static constexpr int FI_{arr.upper()}0 = {idx[0]};")
    # the node-local values of the collision stage (d3q27_pf_velocity.inc Run, lazy pulls)
    names = {f.name: i for i, f in enumerate(m.fields)}
    for n in ("pnorm", "U", "V", "W", "nw_x", "nw_y", "nw_z", "IsSpecialBoundaryPoint"):
        if n in names:
            out.append(f"  static constexpr int FI_{n.upper()} = {names[n]};")
    return "\n".join(out)


def _thermo_declarations(m: Model, planar: bool):
    """thermocapillary.R (sourced by Dynamics.R:112-118 before the stages)"""
    for n in ("Temp", "Cond", "SurfaceTension"):
        m.add_density(n, 0, 0, 0, group="Thermal")
    for n in ("Temp", "Cond", "SurfaceTension"):
        m.add_field(n, stencil3d=1, group="Thermal")
    m.add_quantity("T", unit="K")
    m.add_quantity("ST", unit="N/m")
    S = m.add_setting
    S("surfPower", default=1, comment="Use for parabolic representation of surface tension")
    S("sigma_T", comment="Derivative describing how surface tension changes with temp unit=[N/m2]")
    S("sigma_TT", comment="Derivative describing how surface tension changes with temp unit=[N/m3]")
    S("T_ref", comment="Reference temperature at which sigma is set unit=[K]")
    S("T_init", zonal=True, comment="Initial temperature field unit=[K]")
    S("cp_h", comment="specific heat for heavy phase unit=[J/kg/K]")
    S("cp_l", comment="specific heat for light phase unit=[J/kg/K]")
    S("k_h", comment="thermal conductivity for heavy phase unit=[W/m/K]")
    S("k_l", comment="thermal conductivity for light phase unit=[W/m/K]")
    S("dT", comment="Application of vertical temp gradient to speed up initialisation unit=[K]")
    S("dTx", default=0, comment="Application of horizontal temp gradient to speed up initialisation unit=[K]")
    S("stabiliser", default=1, comment="If not solving flow field, can adjust temperature timestep")
    m.add_global("TempChange")
    if planar:
        for n, v in (("T_c", 10), ("T_h", 20), ("T_0", 4), ("myL", 100), ("MIDPOINT", 51), ("PLUSMINUS", 1)):
            S(n, default=v)
        m.add_node_type("BWall", "ADDITIONALS")
        m.add_node_type("TWall", "ADDITIONALS")
    for n in ("RK1", "RK2", "RK3"):
        m.add_density(n, 0, 0, 0, group="Thermal")
        m.add_field(n, stencil3d=1, group="Thermal")
    m.add_node_type("ConstantTemp", "ADDITIONALS")
    m.add_node_type("EAdiabatic", "ADDITIONALS")


def codegen(Qh: int) -> str:
    M = moment_matrix()
    Minv = M.inv()
    P, Mraw = _raw_basis()
    C = M * Mraw.inv()
    Cinv = C.inv()
    uu = sp.symbols("U V W")
    p = sp.Symbol("p")
    out = [f"  // ---- d3q27_pf_velocity moment algebra (model.R:16-46), M = C . Mraw"]
    out.append(tensor_raw_transform("pf_raw", U27, P))
    out.append(tensor_raw_transform("pf_rawinv", U27, P, inverse=True))
    # low moments m0..m9 from raw moments (only these enter relaxation / stress)
    out.append(dense_transform("pf_r2m_lo", C.T, 27, 10, "m[k<10] = C[k,:] . raw"))
    out.append(dense_transform("pf_m2r", Cinv.T, 27, 27, "raw = C^-1 m"))
    eq = mrt_eq(U27, rho=sp.Integer(1), J=uu, mat=M.T)
    req = list(eq.Req)
    req[0] = p
    out.append(exprs_function("pf_req", ["p", "U", "V", "W"], req))
    # stress of M^-1 m: s_ab = sum_i c_ia c_ib (M^-1 m)_i
    pairs = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]
    Srows = sp.Matrix([[sum(int(U27[i, a]) * int(U27[i, b]) * Minv[i, k] for i in range(27)) for k in range(27)]
                       for a, b in pairs])
    out.append(dense_transform("pf_stress", Srows.T, 27, 6, "stress = c c (M^-1 m)"))
    Uh = U27[:Qh]
    eqh = mrt_eq(Uh, rho=sp.Integer(1), J=uu)
    out.append(exprs_function("pf_heq", ["U", "V", "W"], eqh.feq))
    # ---- face boundary conditions (Boundary.c.Rt:31-108)
    gs = [sp.Symbol(f"g_{i}") for i in range(27)]
    hs = [sp.Symbol(f"h_{i}") for i in range(Qh)]
    ren = {s: f"g[{i}]" for i, s in enumerate(gs)}
    ren.update({s: f"h[{i}]" for i, s in enumerate(hs)})
    bg = _bounce(U27)
    bh = _bounce(Uh)
    geq_vel = [sp.expand(e) for e in Minv * sp.Matrix(req)]   # feq with Req[0]=p (p cancels below)
    feq1 = list(eq.feq)                                        # feq with Req[0]=1
    w_g = [sp.nsimplify(e.subs({uu[0]: 0, uu[1]: 0, uu[2]: 0})) for e in feq1]
    pstar = sp.Symbol("pstar")
    pf = sp.Symbol("pf")
    heq_bc = [pf * e for e in (eqh.feq if Qh == 27 else
                               mrt_eq(Uh, rho=sp.Integer(1), J=(0, 0, 0)).feq)]
    for name, n in FACES:
        n = np.array(n)
        # g, velocity type
        cn = U27 @ n
        sel = [i for i in range(27) if cn[i] < 0]
        sel2 = [i for i in range(27) if cn[i] == 0]
        exM = sp.Matrix([[sum((gs[i] - geq_vel[i]) * int(U27[i, d]) for i in sel2) for d in range(3)]])
        Us = sp.Matrix(U27[sel].tolist())
        Nmat = Us.T * Us
        corr = exM * Nmat.inv() * sp.Matrix(U27.tolist()).T
        exprs = [sp.expand(gs[bg[i]] + (geq_vel[i] - geq_vel[bg[i]]) - sp.Rational(1, 2) * corr[0, i]) for i in sel]
        if any(sp.Symbol("p") in e.free_symbols for e in exprs):
            raise AssertionError("pressure term must cancel in the velocity boundary condition")
        out.append(f"  TCLB_FN void pf_bc_vel_g_{name}() {{")
        out.append(assign_block([f"g[{i}]" for i in sel], exprs, rename=ren, tmp_prefix="b_"))
        out.append("  }")
        # g, pressure type
        geq = [pstar * w_g[i] + (feq1[i] - w_g[i]) for i in range(27)]
        exS = sum(gs[i] - geq[i] for i in sel2)
        exprs = [sp.expand(geq[i] + geq[bg[i]] - gs[bg[i]] - sp.Rational(1, 2) * sp.Rational(1, len(sel)) * exS)
                 for i in sel]
        out.append(f"  TCLB_FN void pf_bc_press_g_{name}(R pstar) {{")
        out.append(assign_block([f"g[{i}]" for i in sel], exprs, rename=ren, tmp_prefix="b_"))
        out.append("  }")
        # h (same for velocity and pressure type)
        cn = Uh @ n
        sel = [i for i in range(Qh) if cn[i] < 0]
        sel2 = [i for i in range(Qh) if cn[i] == 0]
        exS = sum(hs[i] - heq_bc[i] for i in sel2)
        exprs = [sp.expand(heq_bc[i] + heq_bc[bh[i]] - hs[bh[i]] - sp.Rational(1, 2) * sp.Rational(1, len(sel)) * exS)
                 for i in sel]
        out.append(f"  TCLB_FN void pf_bc_h_{name}(R pf) {{")
        out.append(assign_block([f"h[{i}]" for i in sel], exprs, rename=ren, tmp_prefix="b_"))
        out.append("  }")
    return "\n".join(out)
