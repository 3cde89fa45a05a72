"""The ``Solver`` object seen by embedded code (<RunPython>, <RunR python="true">).

Reference: the R object model of src/Handlers/cbRunR.cpp:67-516 (Settings, Fields,
Parameters, Quantities, Globals, Actions, Geometry, Info) and its Python face through
reticulate (:687-760: ``Solver.Geometry.X``, ``for name, arr in Solver.Quantities``,
factors handed to Python as 0-based integer codes).  Here the objects are plain Python
classes over the lattice; arrays are NumPy with the reference's R/reticulate axis order
``(nx, ny, nz)`` (vector quantities ``(3, nx, ny, nz)``), covering this rank's region.

* ``Solver.Settings.nu`` / ``Solver.Settings.nu = 0.1``; a zonal setting returns a
  ``ZoneSetting`` (``.DefaultZone``, ``.Inlet = v``, ``dict(...)``).
* ``Solver.Fields.<field>``: stored field values, assignable (the halo is refreshed).
* ``Solver.Quantities.<Q>`` (lattice units) / ``Solver.Quantities["<Q>.si"]``;
  iterating yields ``(name, array)`` for every quantity and its ``.si`` form.
* ``Solver.Globals.<G>``, ``Solver.Globals["<G>.si"]``, ``Solver.Globals.Iteration``.
* ``Solver.Actions.<A>()`` runs an action.
* ``Solver.Geometry``: ``dx dy dz size dim X Y Z`` (cell centres in metres, as the
  reference) and every node-type group (``BOUNDARY``, ``COLLISION``, ...,
  ``SETTINGZONE``) as 0-based codes (0 = None), assignable with codes or names;
  ``Solver.Geometry.levels("BOUNDARY")`` lists the names of the codes.
* ``Solver.Parameters.Values/Lower/Upper/Gradient/X/Y/Z/T`` over the case's design
  elements (``Values`` assignable).
* ``Solver.Info.OutputPath``.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch


class EmbedError(RuntimeError):
    pass


def _xyz(a: np.ndarray) -> np.ndarray:
    """(nz, ny, nx[, ...]) -> (nx, ny, nz) — the R array order of the reference"""
    return np.ascontiguousarray(np.transpose(a, (2, 1, 0)))


def _zyx(a, shape) -> np.ndarray:
    a = np.asarray(a)
    nx, ny, nz = shape
    if a.size != nx * ny * nz:
        raise EmbedError(f"wrong size {a.size} of the assigned array (region {nx}x{ny}x{nz})")
    return np.ascontiguousarray(np.transpose(a.reshape(nx, ny, nz), (2, 1, 0)))


class _Obj:
    """attribute access + ``[name]`` + ``dir()`` + iteration over (name, value)"""
    _names: List[str] = []

    def _get(self, name):
        raise AttributeError(name)

    def _set(self, name, value):
        raise EmbedError(f"{type(self).__name__}: cannot set {name}")

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return self._get(name)

    def __setattr__(self, name, value):
        if name.startswith("_"):
            object.__setattr__(self, name, value)
        else:
            self._set(name, value)

    def __getitem__(self, name):
        return self._get(name)

    def __setitem__(self, name, value):
        self._set(name, value)

    def __dir__(self):
        return list(self._list())

    def _list(self) -> List[str]:
        return []

    def __iter__(self):
        for n in self._list():
            yield n, self._get(n)

    def __repr__(self):
        return f"<{type(self).__name__}: {', '.join(self._list())}>"


class ZoneSetting(_Obj):
    def __init__(self, solver, name):
        object.__setattr__(self, "_s", solver)
        object.__setattr__(self, "_n", name)

    def _list(self):
        return list(self._s.lattice.zone_names)

    def _get(self, zone):
        if zone not in self._s.lattice.zone_names:
            raise AttributeError(f"no zone {zone}")
        return self._s.lattice.get_setting(self._n, zone)

    def _set(self, zone, value):
        self._s.lattice.set_setting(self._n, float(np.asarray(value).reshape(-1)[0]), zone=zone)


class Settings(_Obj):
    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _list(self):
        return [s.name for s in self._s.model.settings]

    def _get(self, name):
        st = self._s.model.setting(name)
        if st is None:
            raise AttributeError(f"unknown setting {name}")
        if st.zonal:
            return ZoneSetting(self._s, name)
        return self._s.lattice.get_setting(name)

    def _set(self, name, value):
        st = self._s.model.setting(name)
        if st is None:
            raise EmbedError(f"unknown setting {name}")
        if st.zonal:       # reference rSettings: "ZoneSetting not supported in rSetting"
            raise EmbedError(f"zonal setting {name}: assign through Solver.Settings.{name}.<zone>")
        self._s.lattice.set_setting(name, float(np.asarray(value).reshape(-1)[0]))


class Fields(_Obj):
    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _list(self):
        return [f.name for f in self._s.model.fields]

    def _index(self, name):
        m = self._s.model
        for i, f in enumerate(m.fields):
            if name in (f.name, f.nicename):
                return i
        raise AttributeError(f"unknown field {name}")

    def _get(self, name):
        lat = self._s.lattice
        i = self._index(name)
        return _xyz(lat.fields_interior(torch.float64)[i].cpu().numpy())

    def _set(self, name, value):
        lat = self._s.lattice
        i = self._index(name)
        cur = lat.fields_interior(torch.float64).clone()
        cur[i] = torch.from_numpy(_zyx(value, lat.shape).astype(np.float64)).to(cur.device)
        lat.set_fields_interior(cur)


class Quantities(_Obj):
    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _list(self):
        out = []
        for q in self._s.model.quantities:
            if not q.adjoint:
                out += [q.name, q.name + ".si"]
        return out

    def _get(self, name):
        s = self._s
        si = name.endswith(".si")
        qn = name[:-3] if si else name
        q = next((q for q in s.model.quantities if q.name == qn), None)
        if q is None:
            raise AttributeError(f"unknown quantity {name}")
        scale = 1.0 / s.units.unit_scale(q.unit) if si else 1.0
        a = s.lattice.quantity(qn, scale=scale).detach().cpu().numpy().astype(np.float64)
        if q.vector:
            return np.ascontiguousarray(np.transpose(a, (0, 3, 2, 1)))
        return _xyz(a[0])


class Globals(_Obj):
    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _list(self):
        out = ["Iteration"]
        for g in self._s.model.globals_:
            out += [g.name, g.name + ".si"]
        return out

    def _get(self, name):
        s = self._s
        if name == "Iteration":
            return s.iter
        si = name.endswith(".si")
        gn = name[:-3] if si else name
        g = next((g for g in s.model.globals_ if g.name == gn), None)
        if g is None:
            raise AttributeError(f"unknown global {name}")
        v = s.lattice.globals.get(gn, 0.0)
        return v / s.units.unit_scale(g.unit) if si else v


class Actions(_Obj):
    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _list(self):
        return [a.name for a in self._s.model.actions]

    def _get(self, name):
        s = self._s
        if s.model.action(name) is None:
            raise AttributeError(f"unknown action {name}")

        def run():
            from ..solver import ITER_GLOBS, ITER_LASTGLOB
            s.lattice.run_action(name, glob=bool(s.iter_type & (ITER_GLOBS | ITER_LASTGLOB)))
        run.__name__ = name
        return run


class Geometry(_Obj):
    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _groups(self) -> List[str]:
        m = self._s.model
        return sorted(g for g in m.group_masks if g not in ("ALL", "NONE"))

    def _list(self):
        return ["dx", "dy", "dz", "X", "Y", "Z", "size", "dim"] + self._groups()

    def levels(self, group: str) -> List[str]:
        """names of the codes of a node-type group (code 0 = None), or the zone names"""
        m = self._s.model
        if group == "SETTINGZONE":
            zn = self._s.lattice.zone_names
            out = [""] * (max(zn.values()) + 1)
            for k, v in zn.items():
                out[v] = k
            return out
        if group not in m.group_masks:
            raise EmbedError(f"Geometry component not found: {group}")
        mask, shift = m.group_masks[group], m.group_shift.get(group, 0)
        out = ["None"] + [""] * (mask >> shift)          # unused codes: "" (as the reference)
        for nt in m.node_types:
            if nt.group == group:
                k = nt.value >> shift
                if k < len(out):
                    out[k] = nt.name
        return out

    def _get(self, name):
        s = self._s
        lat = s.lattice
        nx, ny, nz = lat.shape
        ox, oy, oz = lat.slab.offset
        if name in ("dx", "dy", "dz"):
            return int({"dx": ox, "dy": oy, "dz": oz}[name])
        if name == "size":
            return nx * ny * nz
        if name == "dim":
            return np.array([nx, ny, nz])
        if name in ("X", "Y", "Z"):
            unit = 1.0 / s.units.alt("1m")
            n, o = {"X": (nx, ox), "Y": (ny, oy), "Z": (nz, oz)}[name]
            v = (np.arange(n) + o + 0.5) * unit
            shape = [1, 1, 1]
            shape["XYZ".index(name)] = n
            return np.broadcast_to(v.reshape(shape), (nx, ny, nz)).copy()
        m = s.model
        if name not in m.group_masks or name in ("ALL", "NONE"):
            raise AttributeError(f"Geometry component not found: {name}")
        mask, shift = m.group_masks[name], m.group_shift.get(name, 0)
        fl = lat.get_flags().astype(np.int64)
        return _xyz(((fl & mask) >> shift).astype(np.int32))

    def _set(self, name, value):
        s = self._s
        lat = s.lattice
        m = s.model
        if name not in m.group_masks or name in ("ALL", "NONE"):
            raise EmbedError(f"Geometry component not found: {name}")
        mask, shift = m.group_masks[name], m.group_shift.get(name, 0)
        v = np.asarray(value)
        if v.dtype.kind in "USO":          # names -> codes
            lv = {}
            for i, n in enumerate(self.levels(name)):
                lv.setdefault(n, i)
            bad = set(np.unique(v).tolist()) - set(lv)
            if bad:
                raise EmbedError(f"unknown {name} level(s): {sorted(bad)}")
            v = np.vectorize(lv.__getitem__, otypes=[np.int64])(v)
        codes = _zyx(v, lat.shape).astype(np.int64)
        if codes.min() < 0 or codes.max() > (mask >> shift):
            raise EmbedError(f"{name} codes out of range 0..{mask >> shift}")
        fl = lat.get_flags().astype(np.int64)
        fl = (fl & ~mask) | (codes << shift)
        full = lat.flags.cpu().numpy().astype(np.int64) & ((1 << m.flag_bits) - 1)
        nx, ny, nz = lat.shape
        full[lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx] = fl
        lat.set_flags(full[:, :, :nx])
        if lat.g:
            _refresh_flag_ghosts(lat)


def _refresh_flag_ghosts(lat):
    """ghost planes of the flags follow their owners (neighbour ranks or the periodic
    image): the flags go through the halo exchange as a one-field snapshot"""
    buf = (lat.flags.to(torch.int64) & ((1 << lat.model.flag_bits) - 1)).to(torch.float64).unsqueeze(0)
    saved = lat.halo_sets
    lat.halo_sets = {a: ([0], [0]) for a in saved}
    try:
        lat._halo_finish(lat._halo_start(buf, None))
    finally:
        lat.halo_sets = saved
    v = buf[0].to(torch.int64)
    if lat.model.flag_bits == 16:
        v = torch.where(v >= 1 << 15, v - (1 << 16), v)
    else:
        v = torch.where(v >= 1 << 31, v - (1 << 32), v)
    lat.flags.copy_(v.to(lat.flags.dtype))
    lat.flags_changed()


class Parameters(_Obj):
    _KIND = {"Values": 0, "Gradient": 2, "Upper": 3, "Lower": 4, "X": 6, "Y": 7, "Z": 8, "T": 9}

    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _list(self):
        return list(self._KIND)

    def _get(self, name):
        from .optimization import _get_all
        if name not in self._KIND:
            raise AttributeError(f"unknown parameter view {name}")
        return _get_all(self._s, self._KIND[name])

    def _set(self, name, value):
        from .optimization import _get_all, _set_all
        if name != "Values":
            raise EmbedError("Cannot set anything but Values")
        v = np.asarray(value, dtype=np.float64).reshape(-1)
        if v.size != _get_all(self._s, 0).size:
            raise EmbedError("Wrong number of parameters")
        _set_all(self._s, v)


class Info(_Obj):
    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)

    def _list(self):
        return ["OutputPath"]

    def _get(self, name):
        if name == "OutputPath":
            return self._s.outpath
        raise AttributeError(name)


class SolverAPI(_Obj):
    """the ``Solver`` global of embedded code"""

    def __init__(self, solver):
        object.__setattr__(self, "_s", solver)
        object.__setattr__(self, "_parts", {"Settings": Settings(solver), "Fields": Fields(solver),
                                            "Parameters": Parameters(solver), "Quantities": Quantities(solver),
                                            "Globals": Globals(solver), "Actions": Actions(solver),
                                            "Geometry": Geometry(solver), "Info": Info(solver)})

    def _list(self):
        return list(self._parts)

    def _get(self, name):
        if name not in self._parts:
            raise AttributeError(f"Solver has no {name}")
        return self._parts[name]


def namespace(solver) -> Dict:
    """the persistent namespace shared by every embedded block of one case (the
    reference keeps one interpreter for the whole run)"""
    ns = getattr(solver, "_embed_ns", None)
    if ns is None:
        ns = {"Solver": SolverAPI(solver), "np": np, "numpy": np, "__name__": "__tclb__"}
        solver._embed_ns = ns
    return ns
