"""Cumulant <-> raw-moment relations on the D3Q27 (or D2Q9) moment set, derived with sympy.

For the 3^D moments with per-axis exponent <= 2 the cumulants of the normalised
distribution are kappa = a!b!c! [s^a t^b u^c] log M(s,t,u), M the moment generating
polynomial with mu_abc = m_abc / m_000.  Both directions are generated as CSE'd
straight-line C++ (the reference hand-expands the same recursions in
models/flow/d3q27_cumulant/Dynamics.c.Rt:236-330,417-445).
"""
from __future__ import annotations

import itertools
import math
from typing import Dict, List, Tuple

import sympy as sp

from .cprint import assign_block

Key = Tuple[int, ...]


def _mul(a: Dict[Key, sp.Expr], b: Dict[Key, sp.Expr], cap: int) -> Dict[Key, sp.Expr]:
    out: Dict[Key, sp.Expr] = {}
    for ka, va in a.items():
        for kb, vb in b.items():
            k = tuple(x + y for x, y in zip(ka, kb))
            if max(k) > cap:
                continue
            out[k] = out.get(k, 0) + va * vb
    return out


def _series(X: Dict[Key, sp.Expr], coefs: List[sp.Expr], cap: int, D: int) -> Dict[Key, sp.Expr]:
    """sum_n coefs[n] X^n, truncated to per-variable degree <= cap"""
    zero = tuple([0] * D)
    res: Dict[Key, sp.Expr] = {zero: coefs[0]} if coefs[0] != 0 else {}
    P = {zero: sp.Integer(1)}
    for n in range(1, len(coefs)):
        P = _mul(P, X, cap)
        for k, v in P.items():
            res[k] = res.get(k, 0) + coefs[n] * v
    return res


def keys(D: int) -> List[Key]:
    return [k for k in itertools.product(range(3), repeat=D)]


def index(k: Key) -> int:
    """storage index: a + 3 b + 9 c"""
    return sum(v * 3 ** i for i, v in enumerate(k))


def raw_to_cumulant(D: int = 3):
    mu = {k: sp.Symbol("mu_" + "".join(map(str, k))) for k in keys(D)}
    zero = tuple([0] * D)
    X = {k: mu[k] / math.prod(math.factorial(v) for v in k) for k in keys(D) if k != zero}
    nmax = 2 * D
    coefs = [sp.Integer(0)] + [sp.Rational((-1) ** (n + 1), n) for n in range(1, nmax + 1)]
    K = _series(X, coefs, 2, D)
    kap = {k: sp.expand(K.get(k, 0) * math.prod(math.factorial(v) for v in k)) for k in keys(D)}
    return mu, kap


def cumulant_to_raw(D: int = 3, drop_order_above: int = 99):
    ka = {k: sp.Symbol("k_" + "".join(map(str, k))) for k in keys(D)}
    zero = tuple([0] * D)
    X = {k: ka[k] / math.prod(math.factorial(v) for v in k) for k in keys(D)
         if k != zero and sum(k) <= drop_order_above}
    nmax = 2 * D
    coefs = [sp.Integer(1)] + [sp.Rational(1, math.factorial(n)) for n in range(1, nmax + 1)]
    M = _series(X, coefs, 2, D)
    mu = {k: sp.expand(M.get(k, 0) * math.prod(math.factorial(v) for v in k)) for k in keys(D)}
    return ka, mu


def cumulant_block(prefix: str = "cum", D: int = 3, drop_order_above: int = 3) -> str:
    """C++: <prefix>_raw2cum(const R* m, R* c) (c[0] = rho) and
    <prefix>_cum2raw(const R* c, R* m) (cumulants of total order > drop_order_above
    treated as zero, as the reference does after relaxation)."""
    ks = keys(D)
    mu, kap = raw_to_cumulant(D)
    rename = {}
    lines = [f"  // ---- {prefix}: cumulants of the normalised distribution (index a+3b+9c)"]
    # forward
    lines.append(f"  TCLB_FN static void {prefix}_raw2cum(const R* m, R* c) {{")
    lines.append("    const R irho = R(1) / m[0];")
    for k in ks:
        if k == tuple([0] * D):
            continue
        rename[mu[k]] = f"mu{index(k)}"
        lines.append(f"    const R mu{index(k)} = m[{index(k)}] * irho;")
    tgt = [f"c[{index(k)}]" for k in ks if k != tuple([0] * D)]
    ex = [kap[k] for k in ks if k != tuple([0] * D)]
    lines.append(assign_block(tgt, ex, rename=rename, indent="    ", tmp_prefix="a_"))
    lines.append("    c[0] = m[0];")
    lines.append("  }")
    # inverse
    ka, mu2 = cumulant_to_raw(D, drop_order_above)
    rename2 = {ka[k]: f"c[{index(k)}]" for k in ks}
    lines.append(f"  TCLB_FN static void {prefix}_cum2raw(const R* c, R* m) {{")
    tgt = [f"m[{index(k)}]" for k in ks if k != tuple([0] * D)]
    ex = [sp.expand(mu2[k] * sp.Symbol("RHO")) for k in ks if k != tuple([0] * D)]
    rename2[sp.Symbol("RHO")] = "c[0]"
    lines.append(assign_block(tgt, ex, rename=rename2, indent="    ", tmp_prefix="b_"))
    lines.append("    m[0] = c[0];")
    lines.append("  }")
    return "\n".join(lines)
