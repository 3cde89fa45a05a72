"""Model option formulas (the reference's ``OPT=`` lines in each ``conf.mk``).

The reference reads ``OPT`` as an R model formula (src/models.R:41-66): every term of
the expanded formula is one compiled variant whose name is the model name followed by
the options present, in order of first appearance in the formula; the intercept (the
plain model) is a variant unless the formula has ``-1``; and every variant containing
``autosym`` also exists with ``autosym2``.  This module implements that expansion
without R:

    >>> [v.name for v in expand("d2q9", "bc*autosym")]
    ['d2q9_bc', 'd2q9_autosym', 'd2q9_bc_autosym', 'd2q9', 'd2q9_autosym2', 'd2q9_bc_autosym2']

Grammar (R formula semantics): ``a + b`` union of terms, ``a:b`` interaction,
``a*b = a + b + a:b`` (distributing over parenthesised sums), ``- t`` removes a term,
``-1`` / ``+0`` removes the intercept.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, FrozenSet, List, Set, Tuple

Term = FrozenSet[str]


class FormulaError(ValueError):
    pass


def _tokens(s: str) -> List[str]:
    toks = re.findall(r"[A-Za-z_][A-Za-z0-9_.]*|\d+|[()+*:\-]", s)
    if "".join(toks) != re.sub(r"\s+", "", s):
        raise FormulaError(f"bad option formula: {s!r}")
    return toks


class _Parser:
    """recursive descent; returns (ordered terms, intercept flag, variable order)"""

    def __init__(self, s: str):
        self.t = _tokens(s)
        self.i = 0
        self.vars: List[str] = []

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def take(self, tok=None):
        v = self.peek()
        if tok is not None and v != tok:
            raise FormulaError(f"expected {tok!r} at token {self.i} in {' '.join(self.t)}")
        self.i += 1
        return v

    # expr := ['-'] prod (('+'|'-') prod)*
    def expr(self) -> Tuple[List[Term], bool]:
        terms: List[Term] = []
        icpt = True
        sign = "+"
        if self.peek() == "-":
            self.take()
            sign = "-"
        while True:
            ts, num = self.prod()
            if num is not None:
                if (sign == "-" and num == 1) or (sign == "+" and num == 0):
                    icpt = False
                elif sign == "-" and num == 0:
                    icpt = True
            elif sign == "+":
                for t in ts:
                    if t not in terms:
                        terms.append(t)
            else:
                terms = [t for t in terms if t not in ts]
            if self.peek() in ("+", "-"):
                sign = self.take()
            else:
                return terms, icpt

    # prod := inter ('*' inter)*
    def prod(self):
        ts, num = self.inter()
        while self.peek() == "*":
            self.take()
            us, _ = self.inter()
            ts = _ordered(ts + us + [a | b for a in ts for b in us])
            num = None
        return ts, num

    # inter := atom (':' atom)*
    def inter(self):
        ts, num = self.atom()
        while self.peek() == ":":
            self.take()
            us, _ = self.atom()
            ts = _ordered([a | b for a in ts for b in us])
            num = None
        return ts, num

    def atom(self):
        v = self.take()
        if v == "(":
            ts, icpt = self.expr()
            self.take(")")
            return ts, None
        if v is None or not (v[0].isalpha() or v[0] == "_" or v.isdigit()):
            raise FormulaError(f"unexpected token {v!r}")
        if v.isdigit():
            return [], int(v)
        if v not in self.vars:
            self.vars.append(v)
        return [frozenset([v])], None


def _ordered(ts: List[Term]) -> List[Term]:
    out: List[Term] = []
    for t in ts:
        if t not in out:
            out.append(t)
    return out


@dataclass
class Variant:
    name: str
    options: Dict[str, int] = field(default_factory=dict)   # option -> level (autosym: 1 or 2)


def parse(formula: str) -> Tuple[List[Term], bool, List[str]]:
    p = _Parser(formula)
    terms, icpt = p.expr()
    if p.peek() is not None:
        raise FormulaError(f"trailing tokens in {formula!r}")
    # R's terms(): ordered by degree, then by appearance
    terms = sorted(terms, key=lambda t: len(t))
    return terms, icpt, p.vars


def expand(model: str, formula: str) -> List[Variant]:
    """all variants of ``model`` for an OPT formula, named like src/models.R:60-66"""
    if not formula.strip():
        return [Variant(model, {})]
    terms, icpt, order = parse(formula)
    rows: List[Dict[str, int]] = [{v: 1 for v in t} for t in terms]
    if icpt:
        rows.append({})
    if "autosym" in order:
        rows += [{**r, "autosym": 2} for r in rows if r.get("autosym")]
    out = []
    for r in rows:
        parts = [model] + [v + (str(r[v]) if r[v] > 1 else "") for v in order if r.get(v)]
        out.append(Variant("_".join(parts), r))
    return out


def variant_options(model: str, formula: str, name: str) -> Dict[str, int]:
    """options of a variant name, or KeyError"""
    for v in expand(model, formula):
        if v.name == name:
            return v.options
    raise KeyError(name)


def all_option_names(formula: str) -> Set[str]:
    return set(parse(formula)[2]) if formula.strip() else set()
