"""d2q9_csf — conservative phase-field interface tracking (h populations, phase field in
[-1/2, 1/2]) with continuum-surface-force surface tension: curvature and gradient from a
local least-squares fit over the four 2x2 boxes around a node (optionally WENO-weighted),
wall wetting through smoothed wall normals (fixed-point CalcWallNormall stage), Brinkman
(Hele-Shaw) friction from h_Z, flow in a Cholesky-weighted moment basis or by a cumulant
collision.  Reference: models/multiphase/d2q9_csf/{Dynamics.R, Dynamics.c.Rt},
OPT="(bc+bcinit)*noflow*weno*viscstep*cumulant".

Options: bc (velocity/force field from the BC[0..1] parameter densities), bcinit (initial
phase field from BC[0]), noflow (prescribed velocity, no momentum solve), weno (WENO
weights of the box gradients), viscstep (tanh viscosity step), cumulant (cumulant flow
collision).
"""
import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.blocks import dense_transform, exprs_function
from ...emit.symbolic import mrt_eq, weights_from_eq

U9 = np.array([[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]])


def csf_basis():
    """B = M . H^T with H the (reversed-order) Cholesky factor of M^-1 diag(1/w) M^-T,
    rows scaled as in Dynamics.c.Rt:16-29"""
    eq = mrt_eq(U9, orthogonal=False)
    w = weights_from_eq(eq)
    Minv = eq.mat.inv()
    W0 = Minv * sp.diag(*[1 / wi for wi in w]) * Minv.T
    n = W0.shape[0]
    rev = list(range(n))[::-1]
    Wr = W0.extract(rev, rev)
    Lr = Wr.cholesky(hermitian=False)      # Wr = Lr Lr^T; R's chol() is the upper factor Lr^T
    H = Lr.T.extract(rev, rev)
    scale = [1, sp.sqrt(3) / 3, sp.sqrt(3) / 3, sp.sqrt(2), sp.sqrt(2), 1, sp.sqrt(6) / 3, sp.sqrt(6) / 3, 2]
    H = sp.Matrix(n, n, lambda r, c: sp.nsimplify(H[r, c] * scale[r]))
    B = sp.simplify(eq.mat * H.T)
    return B, w


def build(bc=False, bcinit=False, noflow=False, weno=False, viscstep=False, cumulant=False) -> Model:
    m = Model("d2q9_csf", dims=2, family="multiphase", reference="models/multiphase/d2q9_csf",
              description="conservative phase field + CSF surface tension, Brinkman friction")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", int(x), int(y), 0, group="f")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"h[{i}]", int(x), int(y), 0, group="h")
    m.add_density("h_Z", 0, 0, 0, group="HZ")
    if bc:
        m.add_setting("OverwriteVelocityField", default="0")
        m.add_density("BC[0]", 0, 0, 0, group="BC", parameter=True)
        m.add_density("BC[1]", 0, 0, 0, group="BC", parameter=True)
    if bcinit and not bc:
        m.add_density("BC[0]", 0, 0, 0, group="BC", parameter=True)
    m.add_field("nw_x", stencil2d=1, group="nw")
    m.add_field("nw_y", stencil2d=1, group="nw")
    m.add_field("phi", stencil2d=1)
    # keep: the wall normals are set by the fixed-point CalcWallNormall of Init only; Run
    # reads them and stores them back unchanged (the reference stores them every step)
    m.add_stage("BaseIteration", "Run", load_densities=["f", "h", "HZ", "BC"], save_fields=["f", "h", "nw", "HZ"],
                keep=["nw"])
    m.add_stage("CalcPhi", "CalcPhi", save_fields=["phi"], load_densities=["h"])
    m.add_stage("BaseInit", "Init", load_densities=["BC"], save_fields=["f", "h", "HZ"])
    m.add_stage("CalcWallNormall", "CalcNormal", save_fields=["nw"], fixed_point=True)
    m.add_action("Iteration", ["BaseIteration", "CalcPhi"])
    m.add_action("Init", ["BaseInit", "CalcPhi", "CalcWallNormall"])
    m.add_quantity("H_Z")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Normal", unit="1/m", vector=True)
    m.add_quantity("PhaseField", unit="1")
    m.add_quantity("Curvature", unit="1")
    m.add_quantity("InterfaceForce", unit="1", vector=True)
    m.add_quantity("DEBUG", vector=True)
    m.add_quantity("WallNormal", vector=True)
    S = m.add_setting
    S("PF_Advection_Switch", default=1.0, comment="Parameter to turn on/off advection of phase field")
    S("omega", comment="one over relaxation time")
    S("omega2_ph", default="1", comment="one over relaxation time - second for phase field")
    S("omega_l", comment="one over relaxation time, light phase")
    S("Viscosity", default=0.16666666, comment="viscosity", omega="1.0/(3*Viscosity + 0.5)")
    S("Viscosity_l", default=0.16666666, comment="viscosity", omega_l="1.0/(3*Viscosity_l + 0.5)")
    S("VelocityX", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("VelocityY", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default=0, comment="inlet/outlet/init density", zonal=True)
    S("Mobility", default=0.05, comment="Mobility")
    S("PhaseField", default=0.5, comment="Phase Field marker scalar", zonal=True)
    S("GravitationX", default=0)
    S("GravitationY", default=0)
    if viscstep:
        S("ViscosityStepWidth", default=1)
        S("IntWidth", comment="Viscous step width wrt interface width")
    else:
        S("IntWidth", default=0.333, comment="1/(PF interface width)")
    S("GravitationX_l", default=0)
    S("GravitationY_l", default=0)
    S("SurfaceTensionDecay", default=0.248)
    S("SurfaceTensionRate", default=0.1)
    S("WettingAngle", default=0, zonal=True)
    S("WallAdhesionDecay", default=0, zonal=True)
    S("S2", default="0", comment="MRT Sx")
    S("S3", default="0", comment="MRT Sx")
    S("S4", default="0", comment="MRT Sx")
    S("BrinkmanHeightInv", default=0, zonal=True)
    S("nubuffer", default=0.01, comment="Viscosity in the buffer layer in cumulant collision model")
    S("WallSmoothingMagic", default=0.12, comment="Wall normal smoothing parameter, higher - more smoothed")
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="pressure loss", unit="1m2/s")
    m.add_global("InletFlux", comment="pressure loss", unit="1m2/s")
    for n in ("NSymmetry", "SSymmetry", "EPressure", "WPressure", "EVelocity", "WVelocity", "NVelocity",
              "SVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"bc": bc, "bcinit": bcinit, "noflow": noflow, "weno": weno, "viscstep": viscstep,
                 "cumulant": cumulant}

    def blocks(_m):
        B, w = csf_basis()
        rho, Jx, Jy = sp.symbols("rho Jx Jy")
        eq = mrt_eq(U9, rho=rho, J=(Jx, Jy), mat=B)
        for k in range(3):   # conserved moments must be rho, Jx, Jy themselves
            assert sp.simplify(eq.Req[k] - (rho, Jx, Jy)[k]) == 0
        kinds = []
        for o in eq.order:
            o = int(o)
            kinds.append({0: 0, 1: 0, 2: 2, 3: 3, 4: 4}[o])
        out = [f"  TCLB_FN static constexpr int csf_order(int k) {{ constexpr int o[9] = {{{', '.join(map(str, kinds))}}}; return o[k]; }}"]
        Bn = B.evalf(20)
        out.append(dense_transform("csf_moments", Bn, 9, 9, "R = f . B"))
        out.append(dense_transform("csf_inverse", B.inv().evalf(20), 9, 9, "f = R . B^-1"))
        out.append(exprs_function("csf_req", ["rho", "Jx", "Jy"], [sp.N(e, 20) for e in eq.Req]))
        out.append(exprs_function("csf_feq", ["rho", "Jx", "Jy"], eq.feq))
        out.append("  TCLB_FN static constexpr double csf_w(int i) { constexpr double a[9] = {"
                   + ", ".join(f"{float(x)!r}" for x in w) + "}; return a[i]; }")
        return "\n".join(out)
    m.add_codegen(blocks)
    m.set_dynamics("multiphase/d2q9_csf.inc")
    m.glob_waves = 0 if weno else 2                  # WENO/cumulant: 326-334 VGPRs
    if not (cumulant or weno):
        # 2-wave occupancy floor on the stage kernels: the collision lands at 262 registers
        # (1 wave/SIMD, latency-bound on its fp64 divisions and square roots); capped at
        # 256 it spills 12 bytes and runs 0.613 -> 0.434 ms per 2048^2 step
        # (profiles/README.md r06i).  The cumulant / WENO builds sit far above 256: a cap
        # would spill heavily.
        m.hip_flags = ["-DTCLB_STAGE_WAVES=2"]
    return m
