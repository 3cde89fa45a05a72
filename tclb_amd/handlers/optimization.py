"""Adjoint and optimisation handlers (reference: src/Handlers/acUSAdjoint.cpp,
acSAdjoint.cpp, acOptimize.cpp.Rt, acFDTest.cpp, acObjective.cpp, acThreshold*.cpp,
acOptSolve, InternalTopology.cpp, conFieldParameter.cpp, OptimalControl.cpp,
GenericOptimizer.cpp).

Gradients come from the AD adjoint (tclb_amd.adjoint) — available for every model, not
only Tapenade-processed ones.  Design parameters follow the reference's PAR_GET / PAR_SET /
PAR_GRAD / PAR_LOWER / PAR_UPPER protocol; the optimiser is SciPy (L-BFGS-B / SLSQP) in
place of NLopt, maximising the Objective like the reference's nlopt_set_max_objective.
"""
from __future__ import annotations

import math
from typing import List

import numpy as np
import torch

from ..utils.log import log
from .base import (HANDLER_DESIGN, Action, Design, GenericAction, HandlerError, register)

PAR_GET, PAR_SET, PAR_GRAD, PAR_UPPER, PAR_LOWER = range(5)
PAR_X, PAR_Y, PAR_Z, PAR_T = 6, 7, 8, 9          # parameter coordinates (reference vHandler.h:19-22)


def _designs(solver) -> List[Design]:
    return [h for h in solver.hands if h.kind & HANDLER_DESIGN]


def _get_all(solver, kind):
    out = []
    for d in _designs(solver):
        n = d.number_of_parameters()
        buf = np.zeros(n)
        d.parameters(kind, buf)
        out.append(buf)
    return np.concatenate(out) if out else np.zeros(0)


def _set_all(solver, x):
    k = 0
    for d in _designs(solver):
        n = d.number_of_parameters()
        d.parameters(PAR_SET, np.asarray(x[k:k + n], dtype=np.float64))
        k += n


# ----------------------------------------------------------------------------- adjoint
@register("Adjoint")
class AdjointAction(GenericAction):
    """<Adjoint type="unsteady|steady"> children </Adjoint>.  Unsteady: the children run
    the primal (callbacks included); the recorded window is then re-run with checkpoints
    and swept backwards.  Steady: after the children, a fixed-point adjoint of
    ``Iterations`` steps at the final primal state.  The objective of the window and the
    adjoint state are left on the solver for designs/optimisers."""

    def init(self):
        super().init()
        from ..adjoint import Adjoint
        s = self.solver
        lat = s.lattice
        typ = self.node.get("type")
        if typ is None:
            typ = "steady" if self.node.get("Iterations") is not None else "unsteady"
        settings = [d.setting for d in _designs(s) if getattr(d, "setting", None) and d.setting in lat.gsettings]
        zonal = [d.setting for d in _designs(s) if getattr(d, "setting", None) and d.setting in lat.zsettings]
        state0 = lat.snaps[lat.cur].clone()
        it0 = lat.iter
        s_it0 = s.iter
        self.execute_internal()
        self.unstack()
        steps = s.iter - s_it0
        ad = Adjoint(lat, settings=settings, zonal=zonal)
        if typ == "unsteady":
            if steps <= 0:
                raise HandlerError("No iterations done inside of Unsteady Adjoint! Nothing to do")
            lat.snaps[lat.cur].copy_(state0)
            lat.iter = it0
            ad.unsteady(steps)
            s.objective = ad.J
        else:
            n = int(self.solver.units.alt(self.node.get("Iterations", "100")))
            ad.steady(n)
            s.objective = lat.globals.get("Objective", 0.0)
        s.adjoint = ad
        log.notice(f"Adjoint ({typ}): objective {s.objective:.10g}")
        return 0


# ----------------------------------------------------------------------------- designs
def _design_mask(solver):
    lat = solver.lattice
    m = lat.model
    mask = m.group_masks.get("DESIGNSPACE")
    fl = lat.get_flags()
    if not mask:
        return np.ones(fl.shape, dtype=bool)
    return (fl & mask) != 0


@register("InternalTopology")
class InternalTopology(Design):
    """parameter densities on DESIGNSPACE nodes, bounds [0, 1] (reference
    InternalTopology.cpp + Solver::getPar/setPar/getDPar)"""

    def init(self):
        s = self.solver
        self.fields = [f for f in s.model.fields if f.parameter and f.is_density]
        if not self.fields:
            raise HandlerError(f"model {s.model.name} has no parameter densities")
        self.mask = _design_mask(s)
        return 0

    def number_of_parameters(self):
        return int(self.mask.sum()) * len(self.fields)

    def _view(self, i):
        lat = self.solver.lattice
        nx, ny, nz = lat.shape
        return lat.snaps[lat.cur][i, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx]

    def coords(self, kind):
        """x/y/z (global node indices) or t (0) of every parameter"""
        lat = self.solver.lattice
        if kind == PAR_T:
            return np.zeros(self.number_of_parameters())
        nx, ny, nz = lat.shape
        ox, oy, oz = lat.slab.offset
        Z, Y, X = np.meshgrid(np.arange(nz) + oz, np.arange(ny) + oy, np.arange(nx) + ox, indexing="ij")
        c = {PAR_X: X, PAR_Y: Y, PAR_Z: Z}[kind][self.mask].astype(np.float64)
        return np.tile(c, len(self.fields))

    def parameters(self, kind, data):
        lat = self.solver.lattice
        n = int(self.mask.sum())
        if kind in (PAR_X, PAR_Y, PAR_Z, PAR_T):
            data[:] = self.coords(kind)
            return 0
        if kind in (PAR_UPPER, PAR_LOWER):
            data[:] = 1.0 if kind == PAR_UPPER else 0.0
            return 0
        for k, f in enumerate(self.fields):
            i = lat.model.field_index(f.name)
            if kind == PAR_GET:
                data[k * n:(k + 1) * n] = self._view(i).numpy()[self.mask]
            elif kind == PAR_SET:
                v = self._view(i)
                a = v.numpy().copy()
                a[self.mask] = data[k * n:(k + 1) * n]
                import torch
                v.copy_(torch.from_numpy(a))
                lat.exchange()
            elif kind == PAR_GRAD:
                ad = getattr(self.solver, "adjoint", None)
                if ad is None:
                    raise HandlerError("no adjoint gradient available (run <Adjoint> first)")
                data[k * n:(k + 1) * n] = ad.field_gradient(f.name)[self.mask]
        return 0


@register("FieldParameter")
class FieldParameter(InternalTopology):
    """one named field on DESIGNSPACE nodes, bounds from lower/upper attributes
    (reference conFieldParameter.cpp)"""

    def init(self):
        s = self.solver
        name = self.node.get("field")
        if name is None:
            raise HandlerError("FieldParameter needs field=")
        self.fields = [s.model.field(name)]
        self.mask = _design_mask(s)
        self.lower = float(self.node.get("lower", "0"))
        self.upper = float(self.node.get("upper", "1"))
        return 0

    def parameters(self, kind, data):
        if kind == PAR_UPPER:
            data[:] = self.upper
            return 0
        if kind == PAR_LOWER:
            data[:] = self.lower
            return 0
        return super().parameters(kind, data)


@register("Extrude")
class Extrude(Design):
    """<Extrude direction="x|y|z|t" theta= margin=> child design: the child's parameters
    are grouped into lines along ``direction`` (equal other coordinates); one parameter
    per line is the position v of a smooth front, child value = 1/(1 + exp(-(c - v)/theta))
    (reference conExtrude.cpp: sorted lines, Fun/FunD, GET/UPPER/LOWER front search)."""

    def init(self):
        kids = [c for c in self.node if isinstance(c.tag, str)]
        if len(kids) != 1:
            raise HandlerError("Extrude needs exactly one child design")
        from .base import make_handler
        self.child = make_handler(kids[0], self.solver)
        if self.child is None or not (self.child.kind & HANDLER_DESIGN):
            raise HandlerError("Extrude needs a child of design type")
        d = self.node.get("direction")
        if d not in ("x", "y", "z", "t"):
            raise HandlerError(f"Extrude needs proper direction - \"{d}\" given")
        self.dir = "xyzt".index(d)
        self.theta = self.solver.units.alt(self.node.get("theta", "1"))
        self.margin = self.solver.units.alt(self.node.get("margin", "1"))
        self.setting = getattr(self.child, "setting", None)
        self.zone = getattr(self.child, "zone", None)
        n2 = self.child.number_of_parameters()
        C = np.zeros((4, n2))
        for i, k in enumerate((PAR_X, PAR_Y, PAR_Z, PAR_T)):
            self.child.parameters(k, C[i])
        self.C = C
        others = [i for i in range(4) if i != self.dir]
        keys = [tuple(C[others, j]) for j in range(n2)]
        pos = C[self.dir] if self.theta > 0 else -C[self.dir]
        self.idx = sorted(range(n2), key=lambda j: (keys[j], pos[j]))
        self.line = np.zeros(n2, dtype=int)          # line number of every child parameter
        k = 0
        for a, j in enumerate(self.idx):
            self.line[j] = k
            if a + 1 < n2 and keys[self.idx[a + 1]] != keys[j]:
                k += 1
        self.n = k + 1 if n2 else 0
        self.par = np.zeros(self.n)
        return 0

    def number_of_parameters(self):
        return self.n

    def _fun(self, x, v):
        e = np.exp((x - v) / self.theta)
        return e / (e + 1)

    def _fund(self, x, v):
        e = np.exp((x - v) / self.theta)
        return -(e / (e + 1) / (e + 1)) / self.theta

    def parameters(self, kind, data):
        c = self.C[self.dir]
        if kind == PAR_SET:
            self.par = np.asarray(data, dtype=np.float64).copy()
            self.child.parameters(PAR_SET, self._fun(c, self.par[self.line]))
        elif kind == PAR_GRAD:
            g2 = np.zeros(c.size)
            self.child.parameters(PAR_GRAD, g2)
            data[:] = np.bincount(self.line, weights=self._fund(c, self.par[self.line]) * g2, minlength=self.n)
        else:   # GET / UPPER / LOWER: per line, the first position past the front / the extremes
            vals = np.zeros(c.size)
            if kind == PAR_GET:
                self.child.parameters(PAR_GET, vals)
            out = np.zeros(self.n)
            st = True
            k = 0
            for a, j in enumerate(self.idx):
                if kind == PAR_UPPER and out[k] < c[j]:
                    st = True
                if kind == PAR_LOWER and out[k] > c[j]:
                    st = True
                if kind == PAR_GET and vals[j] < 0.5:
                    st = True
                if st:
                    out[k] = c[j]
                    st = False
                if a + 1 < len(self.idx) and self.line[self.idx[a + 1]] != k:
                    k += 1
                    st = True
            off = abs(self.margin * self.theta)
            data[:] = out + off if kind == PAR_UPPER else out - off
        return 0


@register("OptimalControl", "ControlParameter")
class OptimalControl(Design):
    """a (zonal) setting as design parameter, what="Setting" or "Setting-Zone".  When the
    zonal setting carries a time series (set by <Control>), every entry of the series is a
    parameter and its gradient comes per time index from the adjoint (reference
    OptimalControl.cpp: zSet.get/set/get_grad of length zSet.getLen); otherwise the
    setting value itself is the single parameter (conControlParameter.cpp)."""

    def init(self):
        what = self.node.get("what") or self.node.get("name")
        if not what:
            raise HandlerError("OptimalControl needs what=")
        self.setting, _, zone = what.partition("-")
        self.zone = zone or None
        lat = self.solver.lattice
        if self.setting not in lat.gsettings and self.setting not in lat.zsettings:
            raise HandlerError(f"unknown setting {self.setting}")
        self.lower = self.solver.units.alt(self.node.get("lower", "-1e30"))
        self.upper = self.solver.units.alt(self.node.get("upper", "1e30"))
        return 0

    def _series(self):
        lat = self.solver.lattice
        if self.setting in lat.zsettings:
            return lat.zone_series(self.setting, self.zone)
        return None

    def number_of_parameters(self):
        v = self._series()
        return 1 if v is None else len(v)

    def parameters(self, kind, data):
        lat = self.solver.lattice
        v = self._series()
        if kind == PAR_GET:
            data[:] = lat.get_setting(self.setting, zone=self.zone) if v is None else v
        elif kind == PAR_SET:
            if v is None:
                lat.set_setting(self.setting, float(data[0]), zone=self.zone)
            else:
                lat.set_zone_series(self.setting, np.asarray(data, dtype=np.float64), zone=self.zone)
        elif kind == PAR_GRAD:
            ad = self.solver.adjoint
            data[:] = ad.setting_gradient(self.setting, self.zone) if v is None else \
                ad.series_gradient(self.setting, self.zone)
        elif kind == PAR_UPPER:
            data[:] = self.upper
        elif kind == PAR_LOWER:
            data[:] = self.lower
        elif kind == PAR_T:
            data[:] = np.arange(len(data))
        elif kind in (PAR_X, PAR_Y, PAR_Z):
            data[:] = 0.0
        return 0


@register("OptimalControlSecond")
class OptimalControlSecond(OptimalControl):
    """time-series control at half resolution: parameter i sets entry 2i, odd entries are
    linearly interpolated (reference OptimalControlSecond.cpp:70-112)"""

    def number_of_parameters(self):
        return super().number_of_parameters() // 2

    def _basis(self):
        n2 = super().number_of_parameters()
        n = n2 // 2
        B = np.zeros((n2, n))
        for i in range(n):
            if 2 * i < n2:
                B[2 * i, i] = 1.0
            if 2 * i + 1 < n2:
                if i + 1 < n:
                    B[2 * i + 1, i] = B[2 * i + 1, i + 1] = 0.5
                else:
                    B[2 * i + 1, i] = 1.0
        return B

    def parameters(self, kind, data):
        n2 = super().number_of_parameters()
        if kind in (PAR_UPPER, PAR_LOWER):
            return super().parameters(kind, data)
        B = self._basis()
        full = np.zeros(n2)
        if kind == PAR_GET:
            super().parameters(PAR_GET, full)
            data[:] = full[0::2][:len(data)]
        elif kind == PAR_SET:
            super().parameters(PAR_SET, B @ np.asarray(data, dtype=np.float64))
        elif kind == PAR_GRAD:
            super().parameters(PAR_GRAD, full)
            data[:] = B.T @ full
        return 0


class _ReducedControl(Design):
    """a design re-parameterising its single child design through a linear basis B
    (child = B @ own): SET pushes B p, GRAD pulls B^T g, GET least-squares fits"""

    def init(self):
        kids = [c for c in self.node if isinstance(c.tag, str)]
        if len(kids) != 1:
            raise HandlerError(f"{self.node.tag} needs exactly one child design")
        from .base import make_handler
        self.child = make_handler(kids[0], self.solver)
        if self.child is None or not (self.child.kind & HANDLER_DESIGN):
            raise HandlerError(f"{self.node.tag} needs a child of design type")
        self.n2 = self.child.number_of_parameters()
        self.setting = getattr(self.child, "setting", None)     # for the adjoint's zonal seeds
        self.zone = getattr(self.child, "zone", None)
        self.lower = self.solver.units.alt(self.node.get("lower", "-1"))
        self.upper = self.solver.units.alt(self.node.get("upper", "1"))
        self.B = self.basis()
        return 0

    def number_of_parameters(self):
        return self.B.shape[1]

    def get(self, full):
        return np.linalg.lstsq(self.B, full, rcond=None)[0]

    def parameters(self, kind, data):
        if kind == PAR_UPPER:
            data[:] = self.upper
        elif kind == PAR_LOWER:
            data[:] = self.lower
        elif kind == PAR_SET:
            self.child.parameters(PAR_SET, self.B @ np.asarray(data, dtype=np.float64))
        else:
            full = np.zeros(self.n2)
            self.child.parameters(kind, full)
            data[:] = self.get(full) if kind == PAR_GET else self.B.T @ full
        return 0


def bspline_basis(n2: int, n: int, order: int = 3, periodic: bool = False) -> np.ndarray:
    """B-spline basis of n functions sampled at n2 control instants (reference
    src/spline.h bspline_b: clamped uniform knots, or periodic wrap)"""
    def knot(i, nn, k, cut):
        if not cut:
            return (i - k) / (nn - k)
        if i < k + 1:
            return 0.0
        if i < nn:
            return (i - k) / (nn - k)
        return 1.0

    def bmod(x, p, k, cut):
        nn = len(p)
        i = int(math.floor(x * (nn - k))) + k
        if k > nn - 1:
            k = nn - 1
        i = min(max(i, k), nn - 1)
        for j in range(k, 0, -1):
            for l in range(j):
                a = (x - knot(i - l, nn, k, cut)) / (knot(i - l + j, nn, k, cut) - knot(i - l, nn, k, cut))
                p[i - l] = a * p[i - l] + (1 - a) * p[i - l - 1]
        return p[i]

    B = np.zeros((n2, n))
    for j in range(n2):
        x = j / n2 if periodic else j / max(n2 - 1.0, 1.0)
        for w in range(n):
            nn = n + order if periodic else n
            p = [0.0] * nn
            p[min(max(w, 0), n - 1)] = 1.0
            ww = w + nn - order
            if periodic and ww < nn:
                p[ww] = 1.0
            B[j, w] = bmod(x, p, order, not periodic)
    return B


@register("BSpline")
class BSpline(_ReducedControl):
    """<BSpline nodes= order= periodic=> child control (reference BSpline.cpp)"""

    def basis(self):
        n = int(self.node.get("nodes", "10"))
        return bspline_basis(self.n2, n, int(self.node.get("order", "3")),
                             self.node.get("periodic", "false").lower() in ("1", "true", "yes"))


@register("Fourier")
class Fourier(_ReducedControl):
    """<Fourier modes=(odd)> child control: constant + cos/sin pairs over the control
    window (reference Fourier.cpp)"""

    def basis(self):
        n = int(self.node.get("modes", "10"))
        if n % 2 != 1:
            n += 1
        j = np.arange(self.n2)
        B = np.zeros((self.n2, n))
        for i in range(n):
            i0, i1 = (i + 1) >> 1, i & 1
            B[:, i] = np.sin(i0 * math.pi * 2 * j / self.n2) if i1 else np.cos(i0 * math.pi * 2 * j / self.n2)
        return B


@register("RepeatControl")
class RepeatControl(_ReducedControl):
    """<RepeatControl length= flip=> child control: a segment of ``length`` entries
    repeated over the window; with ``flip`` every other repetition is mirrored about the
    flip level (reference RepeatControl.cpp)"""

    def init(self):
        self.flip = self.node.get("flip") is not None
        return super().init()

    def basis(self):
        n = int(self.solver.units.alt(self.node.get("length", "1")))
        B = np.zeros((self.n2, n))
        for j in range(self.n2):
            odd = self.flip and ((j // n) % 2 == 1)
            B[j, j % n] = -1.0 if odd else 1.0
        return B

    def parameters(self, kind, data):
        if self.flip and kind in (PAR_SET, PAR_GET):
            lvl = self.solver.units.alt(self.node.get("flip"))
            n = self.B.shape[1]
            odd = np.array([((j // n) % 2 == 1) for j in range(self.n2)])
            if kind == PAR_SET:
                full = self.B @ np.asarray(data, dtype=np.float64) + np.where(odd, lvl, 0.0)
                self.child.parameters(PAR_SET, full)
            else:
                full = np.zeros(self.n2)
                self.child.parameters(PAR_GET, full)
                full = np.where(odd, lvl - full, full)
                data[:] = np.array([full[i::n].mean() for i in range(n)])
            return 0
        return super().parameters(kind, data)


# ----------------------------------------------------------------------------- optimisers
class _Optimizer(GenericAction):
    def _evaluate(self, x):
        s = self.solver
        lat = s.lattice
        lat.snaps[lat.cur].copy_(self.state0)
        lat.iter = self.lat_it0
        s.iter = self.it0
        _set_all(s, x)
        self.execute_internal()
        self.unstack()
        J = float(getattr(s, "objective", lat.globals.get("Objective", 0.0)))
        g = _get_all(s, PAR_GRAD)
        self.evals += 1
        self.history.append(J)
        log.notice(f"{self.node.tag} evaluation {self.evals}: objective {J:.10g}")
        return J, g

    def _prepare(self):
        s = self.solver
        lat = s.lattice
        self.evals = 0
        self.history = s.opt_history = []
        self.state0 = lat.snaps[lat.cur].clone()
        self.lat_it0 = lat.iter
        self.it0 = s.iter
        x0 = _get_all(s, PAR_GET)
        if x0.size == 0:
            raise HandlerError(f"{self.node.tag}: no design parameters defined")
        lo, hi = _get_all(s, PAR_LOWER), _get_all(s, PAR_UPPER)
        return x0, lo, hi


@register("Optimize")
class Optimize(_Optimizer):
    """maximise the Objective over the design parameters (reference acOptimize,
    src/Handlers/acOptimize.cpp.Rt:1-140, NLopt).  ``method``: MMA (default; the
    conservative moving-asymptotes method of tclb_amd.utils.mma), LBFGS (L-BFGS-B),
    COBYLA, NELDERMEAD (derivative-free, scipy), DIRECT_L (scipy ``direct``, locally
    biased) and ESCH (evolutionary; scipy differential evolution stands in for NLopt's
    ESCH).  Stopping criteria: MaxEvaluations, RelTolerance, AbsTolerance,
    XAbsTolerance, StopAtValue.  ``Material="more|less"`` adds the inequality
    constraint sum(x) >= / <= sum(x0) (tolerance 1e-3)."""

    METHODS = ("LBFGS", "MMA", "COBYLA", "NELDERMEAD", "DIRECT_L", "ESCH")

    def init(self):
        super().init()
        import scipy.optimize as so
        from ..utils.mma import mma_minimize
        n = self.node
        x0, lo, hi = self._prepare()
        x0 = np.clip(x0, lo, hi)
        method = (n.get("method") or n.get("Method") or "MMA").upper()
        if method not in self.METHODS:
            raise HandlerError(f"Unknown Method in Optimize: {method}")

        def pos(attr, conv=float):
            v = n.get(attr)
            if v is None:
                return None
            v = conv(float(v))
            if v <= 0:
                raise HandlerError(f"{attr} in Optimize have to be above 0")
            return v
        maxev = pos("MaxEvaluations", int) or 1000
        ftol_rel, ftol_abs, xtol = pos("RelTolerance"), pos("AbsTolerance"), pos("XAbsTolerance")
        stopval = float(n.get("StopAtValue")) if n.get("StopAtValue") is not None else None
        material = float(np.sum(x0))
        mat = n.get("Material")
        if mat not in (None, "more", "less"):
            raise HandlerError('Material attribute in Optimize should be "more" or "less"')
        sign = {"more": 1.0, "less": -1.0}.get(mat)
        cache = {}

        def f_neg(x):                               # NLopt maximises; minimise -J
            key = x.tobytes()
            if key not in cache:
                J, g = self._evaluate(np.asarray(x, dtype=float))
                cache.clear()
                cache[key] = (-J, -g)
            return cache[key]
        if method == "MMA":
            cons = []
            if sign is not None:   # more: material - sum(x) <= 0 ; less: sum(x) - material <= 0
                cons.append(lambda x: (sign * (material - np.sum(x)) - 1e-3, -sign * np.ones_like(x)))
            r = mma_minimize(f_neg, x0, lo, hi, constraints=cons, maxeval=maxev, ftol_rel=ftol_rel or 0.0,
                             ftol_abs=ftol_abs or 0.0, xtol_abs=xtol or 0.0,
                             stopval=None if stopval is None else -stopval)
            xbest, fbest, msg = r.x, r.f, r.message
        else:
            cons = ()
            if sign is not None:
                cons = ({"type": "ineq", "fun": lambda x: sign * (np.sum(x) - material) + 1e-3,
                         "jac": lambda x: sign * np.ones_like(x)},)
            bounds = list(zip(lo, hi))
            fun = lambda x: f_neg(x)[0]   # noqa: E731
            if method == "LBFGS":
                res = so.minimize(f_neg, x0, jac=True, method="L-BFGS-B" if not cons else "SLSQP", bounds=bounds,
                                  constraints=cons, tol=ftol_rel,
                                  options={"maxiter": maxev, **({} if cons else {"maxfun": maxev})})
            elif method == "COBYLA":
                bc = [{"type": "ineq", "fun": (lambda x, i=i: x[i] - lo[i])} for i in range(x0.size)] + \
                     [{"type": "ineq", "fun": (lambda x, i=i: hi[i] - x[i])} for i in range(x0.size)]
                res = so.minimize(fun, x0, method="COBYLA", constraints=list(cons) + bc,
                                  options={"maxiter": maxev, **({"tol": xtol} if xtol else {})})
            elif method == "NELDERMEAD":
                res = so.minimize(fun, x0, method="Nelder-Mead", bounds=bounds,
                                  options={"maxfev": maxev, **({"xatol": xtol} if xtol else {}),
                                           **({"fatol": ftol_abs} if ftol_abs else {})})
            elif method == "DIRECT_L":
                res = so.direct(fun, bounds, maxfun=maxev, locally_biased=True)
            else:  # ESCH
                res = so.differential_evolution(fun, bounds, maxiter=max(1, maxev // (15 * x0.size)), polish=False,
                                                seed=0, constraints=() if not cons else
                                                so.LinearConstraint(sign * np.ones((1, x0.size)),
                                                                    sign * material - 1e-3, np.inf))
            xbest, fbest, msg = np.asarray(res.x), float(res.fun), str(getattr(res, "message", ""))
        self.solver.lattice.snaps[self.solver.lattice.cur].copy_(self.state0)
        _set_all(self.solver, xbest)
        self.solver.optimum = (-fbest, xbest)
        log.notice(f"Optimize [{method}] finished after {self.evals} evaluations: objective {-fbest:.10g} ({msg})")
        return 0


@register("FDTest")
class FDTest(_Optimizer):
    """finite-difference check of the adjoint gradient (reference acFDTest): prints and
    stores (parameter, adjoint, finite difference) rows; order 2/4/6 central differences"""

    def init(self):
        super().init()
        x0, _, _ = self._prepare()
        order = max(2, min(6, int(self.node.get("order", "2"))))
        order += order % 2
        h = float(self.node.get("h", "1e-6"))
        sel = self.node.get("parameters")
        idx = list(range(x0.size))
        if sel:
            a, _, b = sel.partition(":")
            idx = list(range(int(a or 0), int(b) + 1 if b else x0.size)) if ":" in sel else [int(sel)]
        J0, g0 = self._evaluate(x0)
        coef = {2: [(1, 0.5)], 4: [(1, 2 / 3), (2, -1 / 12)], 6: [(1, 0.75), (2, -0.15), (3, 1 / 60)]}[order]
        rows = []
        for i in idx:
            d = 0.0
            for k, c in coef:
                xp, xm = x0.copy(), x0.copy()
                xp[i] += k * h
                xm[i] -= k * h
                d += c * (self._evaluate(xp)[0] - self._evaluate(xm)[0]) / h
            rows.append((i, float(g0[i]), d))
            log.notice(f"FDTest parameter {i}: adjoint {g0[i]:.10g}  finite difference {d:.10g}")
        self.solver.fdtest = rows
        self._evaluate(x0)
        return 0


@register("OptSolve")
class OptSolve(GenericAction):
    """one-shot optimisation loop (reference acOptSolve, src/Handlers/acOptSolve.cpp:5-40):
    a Solve whose iterations are ITER_OPT iterations — primal step, one steady-adjoint
    step, then the design update p += Descent * dJ/dp on DesignSpace nodes (clamped to
    [0, 1]) — until Iterations, with the callbacks of the enclosing level firing as in
    <Solve>.  The adjoint state is carried from iteration to iteration."""

    def init(self):
        super().init()
        from ..adjoint import Adjoint
        from ..solver import ITER_OPT
        s = self.solver
        lat = s.lattice
        old = s.iter_type
        self.execute_internal()
        s.opt_adjoint = Adjoint(lat)
        s.opt_state = torch.zeros_like(lat.snaps[lat.cur])
        s.iter_type = old | ITER_OPT
        try:
            self.solve_loop()
        finally:
            s.iter_type = old
        self.unstack()
        return 0


@register("Threshold", "ThresholdNow")
class Threshold(Action):
    """topology thresholding of the design parameters: p <- (p > level), level from the
    ``Level`` attribute or the Threshold setting (reference acThreshold/acThresholdNow)"""

    def init(self):
        super().init()
        s = self.solver
        lvl = self.node.get("Level")
        level = float(lvl) if lvl is not None else s.lattice.get_setting("Threshold")
        x = _get_all(s, PAR_GET)
        lo, hi = _get_all(s, PAR_LOWER), _get_all(s, PAR_UPPER)
        _set_all(s, np.where(x > level, hi, lo))
        log.notice(f"Threshold at {level}: {int((x > level).sum())} of {x.size} parameters set to upper bound")
        return 0


@register("Objective")
class Objective(Action):
    """<Objective G1="w1" EfficiencyX="w2"/>: every global is an objective of itself, and a
    model may define objective functions of the globals (reference AddObjective, the
    OF_<name> functions of src/Lists.cpp.Rt:18-40).  Objective = sum w_k F_k(globals);
    the <G>InObj weights (zone 0) are set to sum w_k dF_k/dG (reference acObjective)."""

    def init(self):
        super().init()
        s = self.solver
        lat = s.lattice
        m = s.model
        gnames = [g.name for g in m.globals_]
        vals = {g: lat.globals.get(g, 0.0) for g in gnames}
        obj = 0.0
        inobj = {g: 0.0 for g in gnames}
        funcs = [(g, None) for g in gnames if g != "Objective"] + list(getattr(m, "objectives", {}).items())
        for name, expr in funcs:
            w = self.node.get(name)
            if w is None:
                continue
            w = float(w)
            if expr is None:
                obj += w * vals[name]
                inobj[name] += w
            else:
                import sympy as sp
                syms = {g: sp.Symbol(g) for g in gnames}
                e = sp.sympify(expr, locals=syms)
                sub = {syms[g]: vals[g] for g in gnames}
                obj += w * float(e.subs(sub))
                for g in gnames:
                    d = sp.diff(e, syms[g])
                    if d != 0:
                        inobj[g] += w * float(d.subs(sub))
        for g, v in inobj.items():
            if f"{g}InObj" in lat.zsettings:
                lat.set_setting(f"{g}InObj", v)
        lat.globals["Objective"] = obj
        s.objective = obj
        return 0
