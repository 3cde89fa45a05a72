"""Print sympy expressions as precision-generic C++ (every literal is ``R(...)``).

The reference prints its polyAlgebra expressions with ``C()`` (src/conf.R, polyAlgebra
ToC); here every numeric literal is wrapped in the compute type ``R`` so that one
emitted body compiles to pure-f32 or pure-f64 code on gfx950 (no silent f64
promotion in float builds)."""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

import sympy as sp
from sympy.printing.c import C99CodePrinter


class RPrinter(C99CodePrinter):
    def __init__(self, rename: Dict[sp.Symbol, str] | None = None):
        super().__init__({"strict": False})
        self._rename = {k: v for k, v in (rename or {}).items()}

    def _lit(self, v) -> str:
        if isinstance(v, sp.Integer):
            return f"R({int(v)})"
        f = float(v)
        r = repr(f)
        if "e" not in r and "." not in r and "inf" not in r and "nan" not in r:
            r += ".0"
        return f"R({r})"

    def _print_Integer(self, expr):
        return self._lit(expr)

    def _print_Rational(self, expr):
        if expr.q == 1:
            return self._lit(sp.Integer(expr.p))
        return self._lit(expr)

    def _print_Float(self, expr):
        return self._lit(expr)

    def _print_Half(self, expr):
        return "R(0.5)"

    def _print_One(self, expr):
        return "R(1)"

    def _print_Zero(self, expr):
        return "R(0)"

    def _print_NegativeOne(self, expr):
        return "R(-1)"

    def _print_Symbol(self, expr):
        if expr in self._rename:
            return self._rename[expr]
        return super()._print_Symbol(expr)

    def _print_Pow(self, expr):
        b, e = expr.as_base_exp()
        if e.is_Integer:
            n = int(e)
            bs = self.parenthesize(b, 100)
            if n == 1:
                return bs
            if n == -1:
                return f"(R(1)/{bs})"
            if 1 < n <= 4:
                return "(" + "*".join([bs] * n) + ")"
            if -4 <= n < -1:
                return "(R(1)/(" + "*".join([bs] * (-n)) + "))"
        if e == sp.Rational(1, 2):
            return f"sqrt({self._print(b)})"
        return f"pow({self._print(b)}, {self._print(e)})"


def cexpr(expr, rename=None) -> str:
    return RPrinter(rename)._print(sp.sympify(expr))


def assign_block(targets: Sequence[str], exprs: Sequence[sp.Expr], rename=None, indent="    ",
                 cse: bool = True, decl_targets: bool = False, tmp_prefix="t_") -> str:
    """Emit `target = expr;` lines (with common-subexpression temporaries)."""
    exprs = [sp.sympify(e) for e in exprs]
    lines: List[str] = []
    if cse:
        syms = sp.numbered_symbols(tmp_prefix)
        repl, red = sp.cse(exprs, symbols=syms, optimizations="basic")
    else:
        repl, red = [], exprs
    pr = RPrinter(rename)
    for s, e in repl:
        lines.append(f"{indent}const R {s} = {pr._print(e)};")
    for t, e in zip(targets, red):
        d = "R " if decl_targets else ""
        lines.append(f"{indent}{d}{t} = {pr._print(e)};")
    return "\n".join(lines)
