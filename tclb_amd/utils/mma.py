"""Method of Moving Asymptotes (Svanberg 1987; the globally convergent variant's
conservative inner loop, as used by NLopt's NLOPT_LD_MMA) for bound-constrained
problems with up to a few inequality constraints.

    minimize f0(x)  s.t.  f_i(x) <= 0,  lo <= x <= hi

Each outer iteration builds the separable convex MMA approximation around x_k (moving
asymptotes L, U; Svanberg's standard heuristics) and solves it exactly through its dual:
for multipliers lam >= 0 the primal minimiser is closed-form per variable, and the
concave dual is maximised by coordinate bisection (one constraint: a 1-D root find).
The approximation is made conservative (rho_i raised until the approximation of every
function at the new point bounds the true value from above, Svanberg 2002 CCSA), so the
objective decreases monotonically for feasible iterates.  Used by the Optimize handler
(reference acOptimize: NLopt MMA is its default method).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

Fn = Callable[[np.ndarray], Tuple[float, np.ndarray]]


@dataclass
class MMAResult:
    x: np.ndarray
    f: float
    evaluations: int
    message: str
    history: List[float] = field(default_factory=list)


def _sub_x(lam, p0, q0, P, Q, low, upp, alpha, beta):
    """closed-form minimiser of sum (p/(U-x) + q/(x-L)) with p = p0 + lam.P, q = q0 + lam.Q"""
    p = p0 + (lam @ P if len(lam) else 0.0)
    q = q0 + (lam @ Q if len(lam) else 0.0)
    sp, sq = np.sqrt(p), np.sqrt(q)
    x = (sp * low + sq * upp) / (sp + sq + 1e-300)
    return np.clip(x, alpha, beta)


def _solve_sub(p0, q0, P, Q, b, low, upp, alpha, beta, c=1000.0, d=1.0):
    """dual solution of the MMA subproblem with artificial variables y_i (cost c y + d y^2/2)"""
    m = P.shape[0]
    lam = np.zeros(m)
    if m == 0:
        return _sub_x(lam, p0, q0, P, Q, low, upp, alpha, beta)

    def grad(l):
        x = _sub_x(l, p0, q0, P, Q, low, upp, alpha, beta)
        y = np.maximum(0.0, (l - c) / d)
        g = P @ (1.0 / (upp - x)) + Q @ (1.0 / (x - low)) - y - b
        return g, x
    for _ in range(60):                      # coordinate bisection on the concave dual
        for i in range(m):
            g, _ = grad(lam)
            if g[i] <= 0 and lam[i] == 0:
                continue
            lo_, hi_ = 0.0, max(1.0, 2 * lam[i])
            li = lam.copy()
            li[i] = hi_
            while grad(li)[0][i] > 0 and hi_ < 1e12:
                hi_ *= 4
                li[i] = hi_
            for _ in range(80):
                li[i] = 0.5 * (lo_ + hi_)
                if grad(li)[0][i] > 0:
                    lo_ = li[i]
                else:
                    hi_ = li[i]
            lam[i] = 0.5 * (lo_ + hi_)
        if m == 1:
            break
    return grad(lam)[1]


def mma_minimize(f0: Fn, x0: Sequence[float], lo: Sequence[float], hi: Sequence[float],
                 constraints: Sequence[Fn] = (), maxeval: int = 100, ftol_rel: float = 0.0,
                 ftol_abs: float = 0.0, xtol_abs: float = 0.0, stopval: Optional[float] = None,
                 move: float = 0.5, asyinit: float = 0.5, asyincr: float = 1.2, asydecr: float = 0.7) -> MMAResult:
    lo = np.asarray(lo, dtype=float)
    hi = np.asarray(hi, dtype=float)
    x = np.clip(np.asarray(x0, dtype=float), lo, hi)
    n = x.size
    m = len(constraints)
    span = np.maximum(hi - lo, 1e-12)

    def evaluate(xx):
        f, g = f0(xx)
        cf, cg = [], []
        for c in constraints:
            v, gv = c(xx)
            cf.append(v)
            cg.append(np.asarray(gv, dtype=float))
        return float(f), np.asarray(g, dtype=float), np.array(cf), (np.array(cg) if m else np.zeros((0, n)))
    f, df, fc, dfc = evaluate(x)
    evals = 1
    hist = [f]
    xold1 = xold2 = x.copy()
    low, upp = x - asyinit * span, x + asyinit * span
    message = "maximum evaluations reached"
    k = 0
    rho0 = 1.0
    rhoc = np.ones(m)
    while evals < maxeval:
        k += 1
        if stopval is not None and f <= stopval:
            message = "stop value reached"
            break
        if k > 2:
            zz = (x - xold1) * (xold1 - xold2)
            fac = np.where(zz > 0, asyincr, np.where(zz < 0, asydecr, 1.0))
            low = x - fac * (xold1 - low)
            upp = x + fac * (upp - xold1)
            low = np.clip(low, x - 10 * span, x - 0.01 * span)
            upp = np.clip(upp, x + 0.01 * span, x + 10 * span)
        elif k > 1:
            low, upp = x - asyinit * span, x + asyinit * span
        alpha = np.maximum.reduce([low + 0.1 * (x - low), x - move * span, lo])
        beta = np.minimum.reduce([upp - 0.1 * (upp - x), x + move * span, hi])
        # CCSA: keep a decaying memory of the curvature needed last time
        rho0 = max(0.1 * rho0, 1e-5)
        rhoc = np.maximum(0.1 * rhoc, 1e-5)
        xprev_try = None
        while True:                                           # conservative inner loop
            ux2, xl2 = (upp - x) ** 2, (x - low) ** 2
            p0 = ux2 * (np.maximum(df, 0) * 1.001 + 0.001 * np.maximum(-df, 0) + rho0 / span)
            q0 = xl2 * (0.001 * np.maximum(df, 0) + 1.001 * np.maximum(-df, 0) + rho0 / span)
            P = ux2 * (np.maximum(dfc, 0) * 1.001 + 0.001 * np.maximum(-dfc, 0) + rhoc[:, None] / span)
            Q = xl2 * (0.001 * np.maximum(dfc, 0) + 1.001 * np.maximum(-dfc, 0) + rhoc[:, None] / span)
            r0 = f - np.sum(p0 / (upp - x) + q0 / (x - low))
            rc = fc - (P @ (1 / (upp - x)) + Q @ (1 / (x - low)))
            xn = _solve_sub(p0, q0, P, Q, -rc, low, upp, alpha, beta)
            if xprev_try is not None and np.array_equal(xn, xprev_try):
                break       # the approximation no longer moves the point (bound-limited)
            xprev_try = xn
            fn, dfn, fcn, dfcn = evaluate(xn)
            evals += 1
            appr0 = r0 + np.sum(p0 / (upp - xn) + q0 / (xn - low))
            apprc = rc + P @ (1 / (upp - xn)) + Q @ (1 / (xn - low))
            tol0 = 1e-13 * max(1.0, abs(f))
            ok0 = fn <= appr0 + tol0
            okc = np.all(fcn <= apprc + 1e-13 * np.maximum(1.0, np.abs(fc))) if m else True
            if (ok0 and okc) or evals >= maxeval:
                break
            # not conservative: raise the curvature of the failing approximations
            w = np.sum((upp - low) * (xn - x) ** 2 / ((upp - xn) * (xn - low) * span))
            if not ok0:
                rho0 = min(1.1 * (rho0 + (fn - appr0) / max(w, 1e-300)), 10 * rho0)
            if m:
                bad = fcn > apprc
                rhoc = np.where(bad, np.minimum(1.1 * (rhoc + (fcn - apprc) / max(w, 1e-300)), 10 * rhoc), rhoc)
        xold2, xold1 = xold1, x
        dfx = np.max(np.abs(xn - x))
        fold = f
        x, f, df, fc, dfc = xn, fn, dfn, fcn, dfcn
        hist.append(f)
        if ftol_abs and abs(f - fold) < ftol_abs:
            message = "absolute objective tolerance reached"
            break
        if ftol_rel and abs(f - fold) < ftol_rel * abs(f):
            message = "relative objective tolerance reached"
            break
        if xtol_abs and dfx < xtol_abs:
            message = "parameter tolerance reached"
            break
    return MMAResult(x=x, f=f, evaluations=evals, message=message, history=hist)
