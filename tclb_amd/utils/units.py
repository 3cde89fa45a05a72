"""Physical units and gauge solving.

Same semantics as the reference's UnitVal/UnitEnv (reference: src/unit.h:17-218,
src/unit.cpp:63-279): 9 base units (m, s, kg, K, x, y, z, A, t), derived units
(N, Pa, J, W, V, C), prefixes (nm..km, ns..ms, h, g, mg), angles (d), percent (%),
``An``; values like ``"0.01m/s"``, ``"1.5e-3kg/m3"``, sums like ``"1m+2cm"``; a set of
gauge equations (``<Units><Param name= value= gauge=/>``) is solved by Gaussian
elimination of the log-scales so that every quantity can be converted to lattice
units (``alt``)."""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

BASE = ["m", "s", "kg", "K", "x", "y", "z", "A", "t"]
NU = len(BASE)


class UnitError(ValueError):
    pass


@dataclass
class UnitVal:
    val: float = 0.0
    uni: np.ndarray = field(default_factory=lambda: np.zeros(NU))

    @staticmethod
    def base(k: int) -> "UnitVal":
        u = np.zeros(NU)
        u[k] = 1
        return UnitVal(1.0, u)

    def __mul__(self, o: "UnitVal") -> "UnitVal":
        o = _uv(o)
        return UnitVal(self.val * o.val, self.uni + o.uni)

    def __truediv__(self, o: "UnitVal") -> "UnitVal":
        o = _uv(o)
        return UnitVal(self.val / o.val, self.uni - o.uni)

    def __add__(self, o: "UnitVal") -> "UnitVal":
        o = _uv(o)
        if not np.array_equal(self.uni, o.uni):
            raise UnitError("Different units in addition")
        return UnitVal(self.val + o.val, self.uni.copy())

    def pow(self, p: float) -> "UnitVal":
        return UnitVal(self.val ** p, self.uni * p)

    def same_unit(self, o: "UnitVal") -> bool:
        return np.array_equal(self.uni, o.uni)

    def __str__(self):
        s = f"{self.val:g}"
        num = "".join(f"{BASE[i]}{_fmt(self.uni[i])}" for i in range(NU) if self.uni[i] > 0)
        den = "".join(f"{BASE[i]}{_fmt(-self.uni[i])}" for i in range(NU) if self.uni[i] < 0)
        return s + num + ("/" + den if den else "")


def _fmt(p):
    return "" if p == 1 else f"{p:g}"


def _uv(v) -> UnitVal:
    if isinstance(v, UnitVal):
        return v
    return UnitVal(float(v), np.zeros(NU))


_NUMCHARS = set("+-0123456789.eE")


class UnitEnv:
    def __init__(self):
        self.scale = np.ones(NU)
        self.units: Dict[str, UnitVal] = {}
        for i, n in enumerate(BASE):
            self.units[n] = UnitVal.base(i)
        self.units["N"] = self.read_text("1kgm/s2")
        self.units["Pa"] = self.read_text("1N/m2")
        self.units["J"] = self.read_text("1Nm")
        self.units["W"] = self.read_text("1J/s")
        self.units["V"] = self.read_text("1kgm2/t3/A")
        self.units["C"] = self.read_text("1tA")
        for n, v in [("nm", "1e-9m"), ("um", "1e-6m"), ("mm", "1e-3m"), ("cm", "1e-2m"), ("km", "1e+3m"),
                     ("h", "3600s"), ("ns", "1e-9s"), ("us", "1e-6s"), ("ms", "1e-3s"), ("g", "1e-3kg"),
                     ("mg", "1e-6kg")]:
            self.units[n] = self.read_text(v)
        self.units["d"] = _uv(math.atan(1.0) * 4.0 / 180.0)
        self.units["%"] = _uv(0.01)
        self.units["An"] = _uv(6.022e23)
        self.gauge: Dict[str, UnitVal] = {}

    # -- parsing (reference readUnitOne/readUnitAlpha/readUnit/readText) --------------
    def _one(self, s: str) -> UnitVal:
        return self.units.get(s, _uv(0.0))

    def _alpha(self, s: str, p: float) -> UnitVal:
        r1 = self._one(s[:1])
        if len(s) < 2:
            return r1.pow(p)
        r1 = r1 * self._alpha(s[1:], p) if r1.val != 0 else _uv(0.0)
        r2 = self._one(s[:2])
        if r2.val != 0:
            r2 = r2 * self._alpha(s[2:], p) if len(s) > 2 else r2.pow(p)
        if r1.val == 0:
            return r2 if r2.val != 0 else _uv(0.0)
        if r2.val == 0:
            return r1
        if s[0] == "m":  # "mm": milli-metre wins over metre*metre (reference warns)
            return r2
        raise UnitError(f"Ambiguous unit: \"{s}\"")

    def read_unit(self, s: str) -> UnitVal:
        ret = _uv(1.0)
        i, w, n = 0, 1, len(s)
        while i < n:
            j = i
            while i < n and s[i].isalpha():
                i += 1
            k = i
            while i < n and (s[i].isdigit() or s[i] == "."):
                i += 1
            l = i
            p = float(s[k:l]) if l > k else 1.0
            last = self._alpha(s[j:k], p) if k > j else _uv(1.0)
            if j < k and last.val == 0:
                raise UnitError(f"Unknown unit \"{s[j:k]}\" in \"{s}\"")
            ret = ret * last if w > 0 else ret / last
            j = i
            while i < n and not s[i].isalnum():
                i += 1
            if i - j > 1:
                raise UnitError(f"Too many non-alpha-numeric characters in units: \"{s[j:i]}\"")
            if i - j == 1:
                if s[j] == "/":
                    w = -1
                elif s[j] == "%":
                    ret = ret * self.units["%"]
                else:
                    raise UnitError(f"Only \"/\" allowed in units: \"{s[j]}\"")
            if i == j and i < n and not s[i].isalnum():
                i += 1
        return ret

    def read_text(self, s: str) -> UnitVal:
        s = s.strip()
        i = 0
        while i < len(s) and s[i] in _NUMCHARS:
            # an 'e' not followed by a digit/sign is the start of a unit word
            if s[i] in "eE" and (i + 1 >= len(s) or s[i + 1] not in "+-0123456789"):
                break
            i += 1
        unit = s[i:]
        ret = self.read_unit(unit) if unit else _uv(1.0)
        if i > 0:
            ret = ret * _uv(float(s[:i]))
        return ret

    # -- conversion --------------------------------------------------------------
    def alt_val(self, v: UnitVal) -> float:
        return float(v.val * np.prod(self.scale ** v.uni))

    def si(self, s: str) -> float:
        return self.read_text(s).val

    def alt(self, s, default: Optional[float] = None) -> float:
        """value in lattice units; accepts sums ``a+b-c`` of unit-bearing terms."""
        if s is None or (isinstance(s, str) and s.strip() == ""):
            if default is None:
                raise UnitError("empty value")
            return float(default)
        if isinstance(s, (int, float)):
            return float(s)
        s = s.strip()
        ret = 0.0
        i = 0
        j = 0
        n = len(s)
        while True:
            c = s[j] if j < n else "\0"
            if c in "+-\0":
                if j > i:
                    ret += self.alt_val(self.read_text(s[i:j]))
                i = j
                if c == "\0":
                    break
            elif c in "eE" and j + 1 < n and s[j + 1] in "+-":
                j += 1
            j += 1
        return ret

    def unit_scale(self, unit: str) -> float:
        """lattice value of 1 [unit] (used to scale outputs back to SI: divide)."""
        if not unit or unit == "1":
            return 1.0
        return self.alt_val(self.read_text("1" + unit if unit[0].isalpha() or unit[0] == "%" else unit))

    # -- gauge ---------------------------------------------------------------------
    def set_unit(self, name: str, v: UnitVal, v2: float = 1.0):
        self.gauge[name] = v / _uv(v2)

    def make_gauge(self):
        M = np.zeros((NU, NU))
        b = np.zeros(NU)
        i = 0
        for name in sorted(self.gauge):
            v = self.gauge[name]
            M[:, i] = v.uni
            b[i] = math.log(v.val)
            i += 1
        for j in range(NU):
            if not np.any(M[j, :i] != 0):
                if i >= NU:
                    raise UnitError("Gauge variables over-constructed")
                M[j, i] = 1
                b[i] = 0
                i += 1
        if i < NU:
            raise UnitError("Gauge variables under-constructed")
        # reference solves Mat^T-indexed system: sum_j uni_j(i) x_j = b_i
        x = np.linalg.solve(M.T, b)
        self.scale = np.exp(-x)

    def describe(self) -> str:
        return "\n".join(f"1 {BASE[j]} = {self.scale[j]:g} units" for j in range(NU))
