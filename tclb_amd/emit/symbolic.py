"""Symbolic LBM algebra used by the static per-model emitter.

Re-derives (with sympy, at build time) the moment-space building blocks that the
reference generates with its R polynomial algebra:

* ``poly_matrix``      ~ MRT_polyMatrix   (reference: src/lib/feq.R:9-21)
* ``integer_orthogonal`` ~ MRT_integerOrtogonal (src/lib/feq.R:23-36)
* ``mrt_eq``           ~ MRT_eq           (src/lib/feq.R:38-82)
* ``d3q19_mrt``        ~ d3q19_MRT        (src/lib/d3q19.R:24-96)

Everything here produces exact rational matrices / sympy expressions which are then
printed as straight-line C++ by :mod:`tclb_amd.emit.cprint`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from fractions import Fraction
from typing import List, Optional, Sequence

import numpy as np
import sympy as sp


def _u_matrix(U) -> np.ndarray:
    U = np.asarray(U, dtype=int)
    if U.ndim != 2:
        raise ValueError("U must be (Q, D)")
    if (np.abs(U) > 1).any():
        raise ValueError("Too high velocities in poly_matrix")
    return U


@dataclass
class PolyMatrix:
    order: np.ndarray   # (Q,) polynomial order of every moment (sorted)
    mat: sp.Matrix      # (Q, Q) mat[i, k] = monomial_k(c_i)
    p: np.ndarray       # (Q, D) exponent of every moment
    canonical: np.ndarray


def poly_matrix(U) -> PolyMatrix:
    """Raw monomial moment basis.  Exponent 2 is used for velocity -1 so that every
    lattice direction maps to exactly one monomial (c_x^p_x c_y^p_y ...)."""
    U = _u_matrix(U)
    p = np.where(U < 0, 2, U)
    sums = p.sum(axis=1)
    can = np.argsort(sums, kind="stable")
    p = p[can]
    Q, D = U.shape
    W = sp.zeros(Q, Q)
    for k in range(Q):
        for i in range(Q):
            v = 1
            for d in range(D):
                v *= int(U[i, d]) ** int(p[k, d])
            W[i, k] = v
    return PolyMatrix(order=p.sum(axis=1), mat=W, p=p, canonical=can)


def integer_orthogonal(M: sp.Matrix) -> sp.Matrix:
    """Integer Gram-Schmidt of the columns of M (unweighted dot product)."""
    M = sp.Matrix(M)
    for i in range(1, M.shape[1]):
        prev = M[:, :i]
        a = [sp.Integer((prev[:, j].T * M[:, i])[0]) for j in range(i)]
        b = [sp.Integer((prev[:, j].T * prev[:, j])[0]) for j in range(i)]
        fr = [Fraction(int(aa), int(bb)) for aa, bb in zip(a, b)]
        den = 1
        for f in fr:
            den = den * f.denominator // np.gcd(den, f.denominator)
        col = M[:, i] * den
        for j, f in enumerate(fr):
            col = col - prev[:, j] * sp.Rational(f.numerator * den, f.denominator)
        M[:, i] = col
    return M


@dataclass
class MRTEq:
    Req: List[sp.Expr]         # equilibrium moments, symbolic in rho, J
    mat: sp.Matrix             # (Q,Q) moments = f . mat
    order: np.ndarray          # order of each moment
    U: np.ndarray
    p: Optional[np.ndarray] = None
    feq: List[sp.Expr] = field(default_factory=list)
    rho: sp.Symbol = None
    J: Sequence[sp.Symbol] = ()


def _truncate(expr: sp.Expr, J: Sequence[sp.Symbol], max_order: int) -> sp.Expr:
    """Drop monomials whose total degree in J exceeds max_order (rho excluded)."""
    expr = sp.expand(expr)
    out = 0
    for term in sp.Add.make_args(expr):
        pw = term.as_powers_dict()
        deg = sum(abs(int(pw.get(j, 0))) for j in J)
        if deg <= max_order:
            out += term
    return out


def mrt_eq(U, rho=None, J=None, sigma2=sp.Rational(1, 3), order=2, orthogonal=True,
           mat: Optional[sp.Matrix] = None) -> MRTEq:
    U = _u_matrix(U)
    D = U.shape[1]
    rho = rho if rho is not None else sp.Symbol("rho")
    if J is None:
        J = sp.symbols("Jx Jy Jz")[:D]
    W = poly_matrix(U)
    Q = U.shape[0]
    H = []
    for k in range(Q):
        h = rho
        for d in range(D):
            if W.p[k, d] == 1:
                h = h * J[d] / rho
            elif W.p[k, d] == 2:
                h = h * (J[d] ** 2 / rho ** 2 + sigma2)
        H.append(_truncate(sp.expand(h), J, order))
    ret = MRTEq(Req=H, mat=W.mat, order=W.order.copy(), U=U, p=W.p, rho=rho, J=J)
    Minv_raw = W.mat.inv()
    if mat is not None:
        M = sp.Matrix(mat)
        T = Minv_raw * M
        ords = []
        for k in range(Q):
            nz = [i for i in range(Q) if abs(float(T[i, k])) > 1e-10]
            ords.append(max(int(W.order[i]) for i in nz))
        ret.order = np.array(ords)
        ret.Req = [sp.expand(e) for e in (sp.Matrix([H]) * T)]
        ret.mat = M
        ret.p = None
    elif orthogonal:
        M = integer_orthogonal(W.mat)
        T = Minv_raw * M
        ret.Req = [sp.expand(e) for e in (sp.Matrix([H]) * T)]
        ret.mat = M
        ret.p = None
    Minv = ret.mat.inv()
    ret.feq = [sp.expand(e) for e in (sp.Matrix([ret.Req]) * Minv)]
    return ret


def mrt_eq_mat(U, mat, rho=None, J=None, sigma2=sp.Rational(1, 3), order=2,
               correction: Optional[Sequence[sp.Expr]] = None) -> MRTEq:
    """MRT_eq(U, rho, J, sigma2, order, mat=attr(U,"MAT"), correction=...) of the
    reference (src/lib/feq.R:38-82): raw product-form equilibrium moments, the optional
    ``correction`` added to the raw moments of polynomial order > 3 (canonical order),
    then expressed in the given moment matrix ``mat`` (mat[i, k] = moment k at direction
    i); ``order`` of every mat moment is the highest raw order it involves."""
    raw = mrt_eq(U, rho=rho, J=J, sigma2=sigma2, order=order, orthogonal=False)
    H = list(raw.Req)
    if correction is not None:
        hi = [k for k in range(len(H)) if int(raw.order[k]) > 3]
        if len(hi) != len(correction):
            raise ValueError("correction of wrong length in mrt_eq_mat")
        for k, c in zip(hi, correction):
            H[k] = sp.expand(H[k] + c)
    M = sp.Matrix(mat)
    T = raw.mat.inv() * M
    Q = M.shape[0]
    ords = []
    for k in range(Q):
        nz = [i for i in range(Q) if abs(float(T[i, k])) > 1e-10]
        ords.append(max(int(raw.order[i]) for i in nz))
    Req = [sp.expand(e) for e in (sp.Matrix([H]) * T)]
    feq = [sp.expand(e) for e in (sp.Matrix([Req]) * M.inv())]
    return MRTEq(Req=Req, mat=M, order=np.array(ords), U=raw.U, p=None, feq=feq, rho=raw.rho, J=raw.J)


def weights_from_eq(eq: MRTEq) -> List[sp.Rational]:
    """Lattice weights = feq at rho=1, J=0."""
    subs = {eq.rho: 1}
    subs.update({j: 0 for j in eq.J})
    return [sp.nsimplify(e.subs(subs)) for e in eq.feq]


# --- d3q19 (d'Humieres MRT matrix; reference src/lib/d3q19.R:1-21) -------------------
D3Q19_MRTMAT_ROWS = [
    [1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1],
    [-30, -11, -11, -11, -11, -11, -11, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8],
    [12, -4, -4, -4, -4, -4, -4, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1],
    [0, 1, -1, 0, 0, 0, 0, 1, -1, 1, -1, 1, -1, 1, -1, 0, 0, 0, 0],
    [0, -4, 4, 0, 0, 0, 0, 1, -1, 1, -1, 1, -1, 1, -1, 0, 0, 0, 0],
    [0, 0, 0, 1, -1, 0, 0, 1, 1, -1, -1, 0, 0, 0, 0, 1, -1, 1, -1],
    [0, 0, 0, -4, 4, 0, 0, 1, 1, -1, -1, 0, 0, 0, 0, 1, -1, 1, -1],
    [0, 0, 0, 0, 0, 1, -1, 0, 0, 0, 0, 1, 1, -1, -1, 1, 1, -1, -1],
    [0, 0, 0, 0, 0, -4, 4, 0, 0, 0, 0, 1, 1, -1, -1, 1, 1, -1, -1],
    [0, 2, 2, -1, -1, -1, -1, 1, 1, 1, 1, 1, 1, 1, 1, -2, -2, -2, -2],
    [0, -4, -4, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, -2, -2, -2, -2],
    [0, 0, 0, 1, 1, -1, -1, 1, 1, 1, 1, -1, -1, -1, -1, 0, 0, 0, 0],
    [0, 0, 0, -2, -2, 2, 2, 1, 1, 1, 1, -1, -1, -1, -1, 0, 0, 0, 0],
    [0, 0, 0, 0, 0, 0, 0, 1, -1, -1, 1, 0, 0, 0, 0, 0, 0, 0, 0],
    [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, -1, -1, 1],
    [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, -1, -1, 1, 0, 0, 0, 0],
    [0, 0, 0, 0, 0, 0, 0, 1, -1, 1, -1, -1, 1, -1, 1, 0, 0, 0, 0],
    [0, 0, 0, 0, 0, 0, 0, -1, -1, 1, 1, 0, 0, 0, 0, 1, -1, 1, -1],
    [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, -1, -1, -1, -1, 1, 1],
]


def d3q19_mrtmat() -> sp.Matrix:
    """MRTMAT with R's column-major fill: the rows listed above are its *columns*,
    i.e. MRTMAT[i, k] = value of moment k at direction i."""
    return sp.Matrix(D3Q19_MRTMAT_ROWS).T


def d3q19_velocities() -> np.ndarray:
    M = np.array(D3Q19_MRTMAT_ROWS, dtype=int).T  # (19 dirs, 19 moments)
    return M[:, [3, 5, 7]]


@dataclass
class D3Q19MRT:
    MAT: sp.Matrix
    Req: List[sp.Expr]
    U: np.ndarray
    selR: List[int]


def d3q19_mrt(rho=None, J=None) -> D3Q19MRT:
    rho = rho if rho is not None else sp.Symbol("rho")
    J = J if J is not None else sp.symbols("Jx Jy Jz")
    MAT = d3q19_mrtmat()
    U = d3q19_velocities()
    p = np.where(U < 0, 2, U)
    W = sp.zeros(19, 19)
    for k in range(19):
        for i in range(19):
            v = 1
            for d in range(3):
                v *= int(U[i, d]) ** int(p[k, d])
            W[i, k] = v
    sigma = sp.Symbol("sigma")
    H = []
    for k in range(19):
        h = rho
        for d in range(3):
            if p[k, d] == 1:
                h = h * J[d] / rho
            elif p[k, d] == 2:
                h = h * (J[d] ** 2 / rho ** 2 + sigma)
        H.append(h)
    feq = sp.Matrix([H]) * W.inv()
    Req = (feq.subs(sigma, sp.Rational(1, 3))) * MAT
    Req = [_truncate(sp.expand(sp.together(e)), J, 2) for e in Req]
    selR = [k for k in range(19) if k not in (0, 3, 5, 7)]
    return D3Q19MRT(MAT=MAT, Req=Req, U=U, selR=selR)
