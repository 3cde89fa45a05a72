"""d2q9_scmp — single-component multiphase pseudopotential model with a Carnahan-Starling
equation of state (Kupershtokh EoS scaling), selectable forcing, collision operator and
wall treatment.  Reference: models/multiphase/d2q9_scmp/{Dynamics.R, Dynamics.c.Rt},
OPT="(LycettLuo+Kupershtokh)*VirtualRhoWBC*ViscositySmooth*(TRT+BGK+WMRT+CUM)*FMT*HiOrd-1".

Options:
  Kupershtokh     exact-difference-method forcing (J += F + rho g before the equilibrium)
  LycettLuo       Lycett-Brown/Luo forcing term (with the reference's zero Phi tensor)
  VirtualRhoWBC   virtual wall density from the weighted fluid neighbours (contact angle
                  via LVRho_phi_dr and the LVRho_ulimit/llimit clamps; wall rho_n < 0 marks)
  ViscositySmooth viscosity interpolated in dynamic viscosity between density_v and
                  density_l (else a step at rho = 1)
  TRT/BGK/WMRT    collision basis (default MRT in raw moments); CUM: D2Q9 cumulant collision
  FMT, HiOrd      tensor-factorised moment transform / order-12 equilibrium
A variant with neither forcing option (the formula allows it) has no interaction force;
the reference does not compile those (its collision refers to an undefined dF).
"""
import numpy as np
import sympy as sp

from ..dsl import Model
from ..flow.auto import wmrt_matrix
from ...emit.blocks import dense_transform, exprs_function, tensor_raw_transform
from ...emit.symbolic import mrt_eq, poly_matrix

U9 = np.array([[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]])


def build(lycettluo=False, kupershtokh=False, virtualrhowbc=False, viscositysmooth=False, trt=False, bgk=False,
          wmrt=False, cum=False, fmt=False, hiord=False) -> Model:
    m = Model("d2q9_scmp", dims=2, family="multiphase", reference="models/multiphase/d2q9_scmp",
              description="D2Q9 pseudopotential multiphase (C-S EoS, EDM / Lycett-Brown-Luo forcing)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", int(x), int(y), 0, group="f")
    m.add_field("rho_n", stencil2d=1, group="rho_n")
    m.add_stage("BaseIteration", "Run", save_fields=["f", "nw"], load_densities=["f"])
    # VirtualRhoWBC wall nodes average the neighbours' rho_n while fluid nodes overwrite
    # rho_n in the same stage: read the pre-stage values (the reference races here)
    m.add_stage("CalcRhoSC", "CalcRhoSC", save_fields=["rho_n"], load_densities=["f"],
                snapshot_reads=virtualrhowbc)
    m.add_stage("BaseInit", "Init", save_fields=["f", "rho_n"], load_densities=["f"])
    m.add_action("Init", ["BaseInit"])
    m.add_action("Iteration", ["BaseIteration", "CalcRhoSC"])
    for q, u, v in (("Rho", "kg/m3", False), ("U", "m/s", True), ("P", "Pa", False), ("F", "N", True),
                    ("Finternal", "N", True), ("DEBUG", "1", True)):
        m.add_quantity(q, unit=u, vector=v)
    S = m.add_setting
    if viscositysmooth:
        S("omega_l", default=1, comment="relaxation factor", nu_l="(1./omega_l - 0.5) / 3.")
        S("omega_v", default=1, comment="relaxation factor", nu_v="(1./omega_v - 0.5) / 3.")
        S("nu_l", default=1 / 6, comment="viscosity")
        S("nu_v", default=1 / 6, comment="viscosity")
    else:
        S("omega_l", default=1, comment="relaxation factor")
        S("omega_v", default=1, comment="relaxation factor")
        S("nu_l", comment="viscosity", omega_l="1.0/(3*nu_l + 0.5)")
        S("nu_v", comment="viscosity", omega_v="1.0/(3*nu_v + 0.5)")
    S("Magic", default=3 / 16, comment="Magic parameter")
    S("Velocity", default="0m/s", unit="m/s", comment="inlet velocity")
    S("Temperature", comment="temperature of the liquid/gas")
    S("LVRho_phi_dr", default=1, zonal=True, comment="wetting toning parameter (DOI 10.1103/PhysRevE.100.053313)")
    S("LVRho_ulimit", default=0.01, zonal=True, comment="Upper limiting value of rho_w")
    S("LVRho_llimit", default=3.2, zonal=True, comment="Lower limiting value of rho_w")
    S("Kupershtokh_K", default="0.01", comment="C-S EOS multiplying param")
    S("Kupershtokh_A", default="-0.152" if kupershtokh else "0",
      comment="A in force calculation - type of stencil (0 for psi*sum(psi(ei)))")
    S("LBL_kappa", default="0", comment="kappa - int width parameter (0 is safe value)")
    S("LBL_epsilon0", default="2", comment="epsilon0 param - se original paper (2 is safe value)")
    S("GravitationY", comment="Gravitation in the direction of y")
    S("GravitationX", comment="Gravitation in the direction of x")
    S("MovingWallVelocity", comment="Velocity of the MovingWall")
    S("Density", comment="zonal density", zonal=True)
    S("Wetting", comment="wetting factor")
    S("density_l", comment="density for omega= omega_l")
    S("density_v", comment="density for omega= omega_l")
    S("nubuffer", comment="Wall buffer density for cumulant")
    for g, c in (("Pressure1", "pressure at Obj1"), ("Pressure2", "pressure at Obj2"),
                 ("Pressure3", "pressure at Obj3"), ("Density1", "density at Obj1"),
                 ("Density2", "density at Obj2"), ("Density3", "density at Obj3"), ("SumUsqr", "Sumo o U**2"),
                 ("WallForce1X", "force x"), ("WallForce1Y", "force y"), ("WallForce2X", "force x"),
                 ("WallForce2Y", "force y"), ("WallForce3X", "force x"), ("WallForce3Y", "force y")):
        m.add_global(g, comment=c)
    for n in ("NMovingWall", "MovingWall", "ESymmetry", "NSymmetry", "SSymmetry"):
        m.add_node_type(n, "BOUNDARY")
    for n in ("SolidBoundary1", "SolidBoundary2", "SolidBoundary3"):
        m.add_node_type(n, "OBJECTIVE")
    # default node types of the reference (src/conf.R: Wall, Solid, MRT, BGK, E/W P/V ...)
    for n in ("Wall", "Solid", "EVelocity", "WPressure", "WVelocity", "EPressure"):
        m.add_node_type(n, "BOUNDARY")
    for n in ("BGK", "MRT"):
        m.add_node_type(n, "COLLISION")
    coll = "TRT" if trt else ("BGK" if bgk else ("WMRT" if wmrt else "MRT"))
    m.options = {"LycettLuo": lycettluo, "Kupershtokh": kupershtokh, "VirtualRhoWBC": virtualrhowbc,
                 "ViscositySmooth": viscositysmooth, "TRT": trt, "BGK": bgk, "WMRT": wmrt, "CUM": cum,
                 "FMT": fmt, "HiOrd": hiord}

    def blocks(_m):
        raw12 = mrt_eq(U9, orthogonal=False, order=12)     # EQ_NO
        if coll == "BGK":
            M = sp.eye(9)
        elif coll == "WMRT":
            M = wmrt_matrix(raw12)
        else:
            M = raw12.mat
        eq = mrt_eq(U9, mat=M, order=12 if hiord else 2)
        om = []
        for o in eq.order:
            o = int(o)
            if o < 2:
                om.append("1")
            elif coll == "TRT" and o % 2 == 1:
                om.append("2")
            elif coll == "MRT" and o > 2:
                om.append("1")
            else:
                om.append("0")
        out = [f"  TCLB_FN static constexpr int om_kind(int k) {{ constexpr int o[9] = {{{', '.join(om)}}}; return o[k]; }}"]
        if fmt:
            pm = poly_matrix(U9)
            out.append(tensor_raw_transform("sc_raw", U9, pm.p))
            out.append(tensor_raw_transform("sc_rawinv", U9, pm.p, inverse=True))
            out.append(dense_transform("sc_r2m", pm.mat.inv() * eq.mat, 9, 9, "m = raw . Mraw^-1 M"))
            out.append(dense_transform("sc_m2r", eq.mat.inv() * pm.mat, 9, 9, "raw = m . M^-1 Mraw"))
            out.append("  TCLB_FN static void sc_moments(const R* f, R* m) { R r[9]; sc_raw(f, r); sc_r2m(r, m); }")
            out.append("  TCLB_FN static void sc_inverse(const R* m, R* f) { R r[9]; sc_m2r(m, r); sc_rawinv(r, f); }")
        else:
            out.append(dense_transform("sc_moments", eq.mat, 9, 9, "m = f . M"))
            out.append(dense_transform("sc_inverse", eq.mat.inv(), 9, 9, "f = m . M^-1"))
        rho, Jx, Jy = sp.symbols("rho Jx Jy")
        e2 = mrt_eq(U9, rho=rho, J=(Jx, Jy), mat=M, order=12 if hiord else 2)
        out.append(exprs_function("sc_req", ["rho", "Jx", "Jy"], e2.Req))
        out.append(exprs_function("sc_feq", ["rho", "Jx", "Jy"], e2.feq))
        return "\n".join(out)
    m.add_codegen(blocks)
    m.set_dynamics("multiphase/d2q9_scmp.inc")
    return m
