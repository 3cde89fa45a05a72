"""auto — generic raw-moment LBM on D3Q27 or D3Q19 with MRT / BGK / TRT collision and an
optional particle-coupling stage (CalcF).  Reference: models/flow/auto/Dynamics.R,
Dynamics.c.Rt (OPT="d3q19*part*(TRT+BGK+WMRT)*FMT*HiOrd*autosym").

Deviation (documented): with ``part`` the coupling force field (fx,fy,fz) written by
the particle stage is added to the momentum in the collision (ForceX + fx), so the
fluid feels the particles (two-way coupling); the reference variant only reports it."""
import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.blocks import dense_transform, exprs_function, tensor_raw_transform
from ...emit.symbolic import mrt_eq, poly_matrix

CV = (0, 1, -1)


def lattice(q19: bool):
    P = [(a, b, c) for c in range(3) for b in range(3) for a in range(3)]
    U = [(CV[a], CV[b], CV[c]) for a, b, c in P]
    sel = [sum(abs(v) for v in u) < 3 for u in U] if q19 else [True] * 27
    P = [p for p, s in zip(P, sel) if s]
    U = np.array([u for u, s in zip(U, sel) if s])
    return P, U


def wmrt_matrix(raw) -> sp.Matrix:
    """WMRT basis of the reference (Dynamics.c.Rt:43-67): A[monomial, moment] holds the
    coefficients of the order-12 raw equilibrium moments as polynomials in (rho, J);
    R = qr.R(A) with rows scaled to a unit diagonal; M = mat . R^-1.  R is computed by exact
    Gram-Schmidt: R[i, j] = <v_i, a_j> / <v_i, v_i> (v_i the orthogonalised columns),
    which equals qr.R(A)[i, j] / qr.R(A)[i, i] for a full-rank A (no pivoting)."""
    Req = raw.Req
    monos = []
    coef = []
    for e in Req:
        d = sp.expand(e).as_coefficients_dict()
        coef.append(d)
        for mono in d:
            if mono not in monos:
                monos.append(mono)
    Q = len(Req)
    A = sp.Matrix(len(monos), Q, lambda r, c: coef[c].get(monos[r], 0))
    if A.shape[0] > Q or A.rank() < Q:
        raise ValueError("WMRT: equilibrium coefficient matrix is not of full column rank")
    R = sp.eye(Q)
    V = []
    for j in range(Q):
        v = A[:, j]
        for i, vi in enumerate(V):
            v = v - vi * ((vi.T * A[:, j])[0] / (vi.T * vi)[0])
        V.append(v)
    for i in range(Q):
        nrm = (V[i].T * V[i])[0]
        for j in range(i, Q):
            R[i, j] = (V[i].T * A[:, j])[0] / nrm
    return raw.mat * R.inv()


def build(q19: bool = False, part: bool = False, coll: str = "MRT", fmt: bool = False, hiord: bool = False,
          autosym: int = 0) -> Model:
    """coll: MRT (default), BGK, TRT or WMRT; fmt: fast (tensor-factorised) moment
    transform; hiord: order-12 (untruncated) equilibrium moments; autosym: symmetry
    node types (reference OPT="d3q19*part*(TRT+BGK+WMRT)*FMT*HiOrd*autosym")."""
    name = "auto"
    m = Model(name, dims=3, family="flow", reference="models/flow/auto",
              description=f"raw-moment {'D3Q19' if q19 else 'D3Q27'} LBM, {coll} collision"
                          f"{', particle coupling' if part else ''}")
    P, U = lattice(q19)
    Q = len(U)
    for k in range(Q):
        m.add_density(f"f[{k}]", int(U[k, 0]), int(U[k, 1]), int(U[k, 2]), group="f",
                      comment="density f%d%d%d" % P[k])
    for n in ("fx", "fy", "fz", "sol"):
        m.add_density(n, 0, 0, 0, group="Force", parameter=True)
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Solid", unit="1")
    m.add_quantity("F", unit="N/m3", vector=True)
    m.add_setting("Viscosity", default=0.16666666, comment="Viscosity")
    m.add_setting("Magic", default=3 / 16, comment="Magic parameter")
    m.add_setting("Velocity", default="0m/s", comment="Inlet velocity", zonal=True, unit="m/s")
    m.add_setting("Pressure", default="0Pa", comment="Inlet pressure", zonal=True, unit="Pa")
    m.add_setting("Turbulence", comment="Turbulence intensity", zonal=True)
    m.add_setting("GalileanCorrection", default=1.0, comment="Galilean correction term")
    for a in "XYZ":
        m.add_setting(f"Force{a}", default=0, comment=f"Force {a}")
    m.add_global("Flux", comment="Volume flux", unit="m3/s")
    m.add_global("Drag", comment="Force exerted on body in X-direction", unit="N")
    m.add_global("Lift", comment="Force exerted on body in Z-direction", unit="N")
    m.add_global("Lateral", comment="Force exerted on body in Y-direction", unit="N")
    for n in ["WVelocityTurbulent", "NVelocity", "SVelocity", "NPressure", "SPressure"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Body", "BODY")
    if part:
        m.add_stage("BaseIteration", "Run", save_fields=["f"], load_densities=["f", "Force"])
        m.add_stage("BaseInit", "Init", save_fields=["f", "Force"])
        # the densities are pulled only on the nodes a particle covers (auto.inc CalcF);
        # on the GPU those nodes run in a deferred kernel of their own (split + defer), so
        # the zero-force pass over the rest of the lattice keeps a small register budget
        m.add_stage("CalcF", "CalcF", save_fields=["Force"], load_densities=["f"], particle=True,
                    lazy_load=True, split=True, defer=True)
        m.add_action("Iteration", ["BaseIteration", "CalcF"])
        m.add_action("Init", ["BaseInit", "CalcF"])
    else:
        # without particles Run only sets the Force fields to the body force (reference
        # Dynamics.c.Rt Run: fx = ForceX ... sol = 0, densities Dynamics.R:24-27) and
        # nothing in the step reads them: the iteration neither loads nor stores them
        # (keep); the lattice fills both snapshots from the settings before the steps of
        # every iterate call in which they changed (Lattice._mirror_kept)
        m.add_stage("BaseIteration", "Run", load_densities=["f"], save_fields=["f", "Force"], keep=["Force"])
        m.setting_fields = {"fx": "ForceX", "fy": "ForceY", "fz": "ForceZ", "sol": 0.0}
    for n in ["EPressure", "EVelocity", "Wall", "WPressure", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"d3q19": q19, "part": part, "TRT": coll == "TRT", "BGK": coll == "BGK", "WMRT": coll == "WMRT",
                 "FMT": fmt, "HiOrd": hiord, "autosym": autosym}

    raw12 = mrt_eq(U, orthogonal=False, order=12)          # EQ_NO of the reference
    if coll == "BGK":
        M = sp.eye(Q)
    elif coll == "WMRT":
        M = wmrt_matrix(raw12)
    else:
        M = raw12.mat
    eq = mrt_eq(U, mat=M, order=12 if hiord else 2)
    orders = [int(o) for o in eq.order]

    def blocks(_m):
        om = []
        for o in orders:
            if o < 2:
                om.append("1")            # conserved
            elif coll == "TRT" and o % 2 == 1:
                om.append("2")            # omega2
            elif coll == "MRT" and o > 2:
                om.append("1")            # relaxed to equilibrium (WMRT: all at omega)
            else:
                om.append("0")            # omega
        out = [f"  TCLB_FN static constexpr int om_kind(int k) {{ constexpr int o[{Q}] = {{{', '.join(om)}}}; return o[k]; }}"]
        if fmt and Q == 27:
            # FMT: raw moments by three 1-D axis passes, then the (sparse) change of basis
            # to M (identity for MRT): m = raw . (Mraw^-1 M), f = raw^-1(m . (M^-1 Mraw))
            pm = poly_matrix(U)
            T = pm.mat.inv() * eq.mat
            Ti = eq.mat.inv() * pm.mat
            out.append(tensor_raw_transform("am_raw", U, pm.p))
            out.append(tensor_raw_transform("am_rawinv", U, pm.p, inverse=True))
            out.append(dense_transform("am_r2m", T, Q, Q, "m = raw . Mraw^-1 M"))
            out.append(dense_transform("am_m2r", Ti, Q, Q, "raw = m . M^-1 Mraw"))
            out.append("  TCLB_FN static void am_moments(const R* f, R* m) { R r[27]; am_raw(f, r); am_r2m(r, m); }")
            out.append("  TCLB_FN static void am_inverse(const R* m, R* f) { R r[27]; am_m2r(m, r); am_rawinv(r, f); }")
        else:
            # D3Q19 (or no FMT): dense straight-line transforms (the tensor factorisation
            # needs the full 27-velocity lattice; the moments are the same)
            out.append(dense_transform("am_moments", eq.mat, Q, Q, "m = f . M"))
            out.append(dense_transform("am_inverse", eq.mat.inv(), Q, Q, "f = m . M^-1"))
        out.append(exprs_function("am_req", ["rho", "Jx", "Jy", "Jz"], eq.Req))
        out.append(exprs_function("am_feq", ["rho", "Jx", "Jy", "Jz"], eq.feq))
        return "\n".join(out)
    m.add_codegen(blocks)
    m.defines["AUTO_Q"] = str(Q)
    m.set_dynamics("flow/auto.inc")
    return m
