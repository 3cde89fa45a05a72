"""Codegen blocks: sympy-derived member functions injected into a model's Node struct.

Each generator returns C++ source text (member functions of the generated
``Node<R,S,GLOB>`` struct).  They replace the inline ``<?R C(...) ?>`` blocks of the
reference's Dynamics.c.Rt templates (e.g. models/flow/d3q27/Dynamics.c.Rt:166-244,
models/flow/d2q9/Dynamics.c.Rt:1-40) with build-time generated, CSE'd straight-line
code, and — for tensor-product raw-moment bases (D2Q9, D3Q27) — a factorised
axis-by-axis moment transform (O(Q·D) instead of O(Q^2) flops), which matters on
gfx950 where the d3q27 fp64 collide-stream must stay HBM-bound.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import sympy as sp

from .cprint import RPrinter, assign_block, cexpr
from .symbolic import MRTEq


def _fmt_coef(v) -> str:
    return cexpr(sp.nsimplify(v))


def dense_transform(fname: str, mat: sp.Matrix, nin: int, nout: int, comment: str = "") -> str:
    """out[k] = sum_i in[i] * mat[i, k]  (straight-line, zero terms skipped)."""
    lines = [f"  // {comment}" if comment else "",
             f"  TCLB_FN static void {fname}(const R* in, R* out) {{"]
    for k in range(nout):
        terms = []
        for i in range(nin):
            c = mat[i, k]
            if c == 0:
                continue
            if c == 1:
                terms.append(f"in[{i}]")
            elif c == -1:
                terms.append(f"-in[{i}]")
            else:
                terms.append(f"{_fmt_coef(c)}*in[{i}]")
        expr = " + ".join(terms) if terms else "R(0)"
        expr = expr.replace("+ -", "- ")
        lines.append(f"    out[{k}] = {expr};")
    lines.append("  }")
    return "\n".join(l for l in lines if l != "")


def tensor_raw_transform(fname: str, U: np.ndarray, p: np.ndarray, inverse: bool = False) -> str:
    """Factorised raw-moment transform for full tensor-product lattices.

    Forward: m_k = sum_i f_i prod_d c_{i,d}^{p_{k,d}}   (p in {0,1,2}; 0^0 = 1)
    Per axis, the 1-D transform on a (f_-, f_0, f_+) triple is
        p0 = f_- + f_0 + f_+,  p1 = f_+ - f_-,  p2 = f_+ + f_-
    and its inverse
        f_0 = p0 - p2,  f_+ = (p2 + p1)/2,  f_- = (p2 - p1)/2.
    """
    U = np.asarray(U, dtype=int)
    p = np.asarray(p, dtype=int)
    Q, D = U.shape
    if Q != 3 ** D:
        raise ValueError("tensor_raw_transform needs a full 3^D lattice")
    dir_index = {tuple(int(v) for v in U[i]): i for i in range(Q)}
    mom_index = {tuple(int(v) for v in p[k]): k for k in range(Q)}
    lines = [f"  TCLB_FN static void {fname}(const R* in, R* out) {{"]
    # state keyed by a D-tuple where axes < a hold exponents and axes >= a hold velocities
    cur: Dict[tuple, str] = {}
    if not inverse:
        for key, i in dir_index.items():
            cur[key] = f"in[{i}]"
    else:
        for key, k in mom_index.items():
            cur[key] = f"in[{k}]"
    tmp = 0
    axes = list(range(D)) if not inverse else list(range(D))[::-1]
    for a in axes:
        nxt: Dict[tuple, str] = {}
        groups: Dict[tuple, Dict[int, str]] = {}
        for key, v in cur.items():
            rest = key[:a] + key[a + 1:]
            groups.setdefault(rest, {})[key[a]] = v
        for rest, g in groups.items():
            def put(val, expr):
                nonlocal tmp
                name = f"t{tmp}"; tmp += 1
                lines.append(f"    const R {name} = {expr};")
                nxt[rest[:a] + (val,) + rest[a:]] = name
            if not inverse:
                fm, f0, fp = g[-1], g[0], g[1]
                put(0, f"{fm} + {f0} + {fp}")
                put(1, f"{fp} - {fm}")
                put(2, f"{fp} + {fm}")
            else:
                p0, p1, p2 = g[0], g[1], g[2]
                put(0, f"{p0} - {p2}")
                put(1, f"R(0.5)*({p2} + {p1})")
                put(-1, f"R(0.5)*({p2} - {p1})")
        cur = nxt
    if not inverse:
        for key, name in cur.items():
            lines.append(f"    out[{mom_index[key]}] = {name};")
    else:
        for key, name in cur.items():
            lines.append(f"    out[{dir_index[key]}] = {name};")
    lines.append("  }")
    return "\n".join(lines)


def exprs_function(fname: str, args: Sequence[str], exprs: Sequence[sp.Expr], out: str = "out",
                   rename: Optional[dict] = None, static: bool = True) -> str:
    arglist = ", ".join(f"R {a}" for a in args)
    if arglist:
        arglist += ", "
    head = f"  TCLB_FN {'static ' if static else ''}void {fname}({arglist}R* {out}) {{"
    body = assign_block([f"{out}[{k}]" for k in range(len(exprs))], exprs, rename=rename, indent="    ")
    return "\n".join([head, body, "  }"])


def vjp_function(fname: str, args: Sequence[str], exprs: Sequence[sp.Expr]) -> str:
    """Transposed Jacobian-vector product of a block of expressions, for hand-written
    reverse sweeps (Model.set_reverse): out[j] = sum_i a[i] * d exprs[i] / d args[j].
    The reference gets these from Tapenade's reverse mode over the generated C
    (tools/makeAD); here they are differentiated symbolically at build time."""
    syms = [sp.Symbol(a) for a in args]
    a = [sp.Symbol(f"adj_{i}") for i in range(len(exprs))]
    outs = [sp.expand(sum(a[i] * sp.diff(sp.sympify(e), s) for i, e in enumerate(exprs))) for s in syms]
    rename = {a[i]: f"a[{i}]" for i in range(len(exprs))}
    arglist = ", ".join(f"R {x}" for x in args)
    head = f"  TCLB_FN static void {fname}({arglist}, const R* a, R* out) {{"
    body = assign_block([f"out[{k}]" for k in range(len(syms))], outs, rename=rename, indent="    ",
                        tmp_prefix="v_")
    return "\n".join([head, body, "  }"])


def feq_block(fname: str, U, order: int = 2) -> str:
    """Equilibrium of a velocity set U in the reference's raw-moment (product-form,
    J-truncated) construction, MRT_eq(U, rho, J)$feq (src/lib/feq.R:38-82):
    ``fname(rho, Jx, Jy[, Jz], out)``."""
    from .symbolic import mrt_eq
    U = np.asarray(U, dtype=int)
    eq = mrt_eq(U, orthogonal=False, order=order)
    return exprs_function(fname, ["rho"] + [str(j) for j in eq.J], eq.feq)


def mrt_block(prefix: str, eq: MRTEq, tensor: bool = False) -> str:
    """Moment transform, equilibrium moments and inverse transform of an MRTEq."""
    Q = eq.mat.shape[0]
    D = eq.U.shape[1]
    parts = [f"  // ---- {prefix}: moment basis of {Q} moments (orders {list(map(int, eq.order))})"]
    orders = ", ".join(str(int(o)) for o in eq.order)
    parts.append(f"  TCLB_FN static constexpr int {prefix}_order(int k) {{ constexpr int o[{Q}] = {{{orders}}}; return o[k]; }}")
    parts.append(f"  static constexpr int {prefix}_Q = {Q};")
    if eq.p is not None:
        diag = ", ".join("1" if (int(o) == 2 and 2 in list(eq.p[k])) else "0" for k, o in enumerate(eq.order))
        parts.append(f"  TCLB_FN static constexpr bool {prefix}_is_diag2(int k) {{ constexpr int o[{Q}] = {{{diag}}}; return o[k] != 0; }}")
    if tensor and eq.p is not None:
        parts.append(tensor_raw_transform(f"{prefix}_moments", eq.U, eq.p, inverse=False))
        parts.append(tensor_raw_transform(f"{prefix}_inverse", eq.U, eq.p, inverse=True))
    else:
        parts.append(dense_transform(f"{prefix}_moments", eq.mat, Q, Q, "moments = f . M"))
        parts.append(dense_transform(f"{prefix}_inverse", eq.mat.inv(), Q, Q, "f = moments . M^-1"))
    Js = [str(j) for j in eq.J]
    parts.append(exprs_function(f"{prefix}_req", ["rho"] + Js, eq.Req))
    parts.append(exprs_function(f"{prefix}_feq", ["rho"] + Js, eq.feq))
    return "\n".join(parts)
