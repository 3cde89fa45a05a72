"""Core XML handlers (reference: src/Handlers/*.cpp, one class per element)."""
from __future__ import annotations

import collections
import copy
import math

import torch
import os
import xml.etree.ElementTree as ET
from typing import List, Optional

import numpy as np

from ..utils.log import log
from .base import (HANDLER_CALLBACK, ITERATION_STOP, Action, Callback, Design, GenericAction, GenericContainer,
                   Handler, HandlerError, make_handler, register)


def _what(node, default="all") -> List[str]:
    return [w.strip() for w in node.get("what", default).split(",") if w.strip()]


# ---------------------------------------------------------------------------- containers
@register("CLBConfig")
class MainContainer(GenericAction):
    """reference MainContainer (src/Handlers/MainContainer.cpp:5-27)"""

    def init(self):
        super().init()
        s = self.solver
        fn = s.out_iter_file("config", ".xml")
        if s.rank == 0:
            cfg = copy.deepcopy(s.config_tree)
            run = ET.SubElement(cfg, "Run", {"model": s.model_name})
            ET.SubElement(run, "Code", {"version": "tclb_amd-0.1", "precision": s.precision,
                                        "cross": "GPU" if s.lattice.is_gpu else "CPU"})
            ET.ElementTree(cfg).write(fn)
        return self.execute_internal()

    def finish(self):
        self.unstack()
        return 0


@register("Units", "Container")
class UnitsContainer(GenericContainer):
    """<Units> params are consumed before the run (reference readUnits); <Container> groups."""

    def init(self):
        if self.node.tag == "Units":
            self.stack = 0
            return 0
        return super().init()


@register("Model")
class ModelContainer(GenericContainer):
    """reference acModel: run children (Params), then lattice Init"""

    def init(self):
        r = super().init()
        self.solver.lattice.init()
        self.solver.iter = 0
        return r


@register("EvalIf")
class IfContainer(GenericAction):
    def init(self):
        super().init()
        present, missing = self.node.get("opt_present"), self.node.get("opt_missing")
        if (present is None) == (missing is None):
            raise HandlerError("Use either opt_present or opt_missing (not both) in EvalIf")
        opt = present if present is not None else missing
        opts = self.solver.model.options
        if opt not in opts:
            raise HandlerError(f"Unknown option in EvalIf: {opt}")
        if bool(opts[opt]) == (present is not None):
            return self.execute_internal()
        return 0

    def finish(self):
        self.unstack()
        return 0


@register("Repeat")
class Repeat(GenericAction):
    def init(self):
        super().init()
        t = self.node.get("Times")
        if t is None:
            raise HandlerError("no Times parameter in Repeat")
        for _ in range(int(t)):
            self.execute_internal()
            self.unstack()
        return 0


# ---------------------------------------------------------------------------- actions
@register("Geometry")
class GeometryAction(Action):
    """reference acGeometry (src/Handlers/acGeometry.cpp:5-23)"""

    def init(self):
        super().init()
        from ..geometry.geometry import Geometry
        s = self.solver
        lat = s.lattice
        sl = lat.slab
        g = Geometry(s.model, lat.gshape, sl.lo, sl.n, sl.axis, lat.g, units=s.units, permissive=s.permissive,
                     yz=(sl.ylo, sl.ny, lat.gy, sl.zlo, sl.nz, lat.gz) if sl.axis == 3 else None)
        g.load(self.node)
        s.geometry = g
        lat.set_flags(g.flags)
        for z in g.zones:
            lat.add_zone(z)
        if g.cuts is not None:
            lat.set_cuts(g.cuts)
        if self.node.get("save"):
            g_path = self.node.get("save")
            s.write_vtk("geometry", ["flag"], None) if g_path else None
        return 0


@register("Param")
class Param(Action):
    """reference acParam (src/Handlers/acParam.cpp:5-64)"""

    def init(self):
        super().init()
        s = self.solver
        par = self.node.get("name", "")
        zone = self.node.get("zone", "")
        value = self.node.get("value")
        gauge = self.node.get("gauge")
        permissive = str(self.context_attr("permissive", "false")).lower() in ("true", "1", "yes")
        if zone and zone not in s.lattice.zone_names:
            raise HandlerError(f"Unknown zone {zone} (found while setting parameter {par})")
        if par == "":
            if gauge is not None:
                return 0
            raise HandlerError("Setting name not specified in Param element")
        st = s.model.setting(par)
        if st is None:
            if permissive:
                log.warning(f"Unknown setting {par}")
                return 0
            raise HandlerError(f"Unknown setting {par}")
        val = s.units.alt(value)
        log.output(f"Setting {par}{' in zone ' + zone if zone else ''} to {value} ({val:g})")
        s.lattice.set_setting(par, val, zone=zone or None)
        return 0


@register("Init")
class InitAction(Action):
    def init(self):
        super().init()
        self.solver.lattice.init()
        self.solver.iter = 0
        return 0


@register("Solve")
class Solve(GenericAction):
    def init(self):
        super().init()
        self.execute_internal()
        self.solve_loop()
        self.unstack()
        return 0


@register("RunAction")
class RunAction(GenericAction):
    """reference acRunAction (src/Handlers/acRunAction.cpp:5-61)"""

    def init(self):
        super().init()
        name = self.node.get("name", "")
        if not name:
            raise HandlerError("Have to specify the name of the Action in RunAction")
        if self.solver.model.action(name) is None:
            raise HandlerError(f"Unknown Action {name}")
        self.execute_internal()
        self.solve_loop(action=name)
        self.unstack()
        return 0


@register("LoadBinary", "LoadMemoryDump")
class LoadBinary(Action):
    def init(self):
        super().init()
        f = self.node.get("file") or self.node.get("filename")
        if f is None:
            raise HandlerError("No file specified in LoadBinary")
        self.solver.load_solution(f, comp=self.node.get("comp"))
        return 0


# ---------------------------------------------------------------------------- callbacks
def _region_attrs(h, total):
    x0, y0, z0, nx, ny, nz = total
    reg = [x0, y0, z0, nx, ny, nz]
    for i, a in enumerate("xyz"):
        d = h.node.get("d" + a)
        if d is not None:
            v = int(round(h.solver.units.alt(d)))
            if v < 0:
                v = total[3 + i] + v
            reg[i] = v
            reg[3 + i] = total[3 + i] - v
    for i, a in enumerate("xyz"):
        n = h.node.get("n" + a)
        if n is not None:
            v = int(round(h.solver.units.alt(n)))
            if v < 0:
                v = total[3 + i] - reg[i] + v
            reg[3 + i] = v
    # intersect with total
    for i in range(3):
        lo = max(reg[i], total[i])
        hi = min(reg[i] + reg[3 + i], total[i] + total[3 + i])
        reg[i], reg[3 + i] = lo, max(0, hi - lo)
    return tuple(reg)


@register("VTK")
class VTK(Callback):
    """reference cbVTK (src/Handlers/cbVTK.cpp:5-68)"""

    def init(self):
        super().init()
        self.name = self.node.get("name", "VTK")
        self.what = _what(self.node)
        self.reg = _region_attrs(self, self.solver.total)
        if self.reg[3] * self.reg[4] * self.reg[5] == 0:
            raise HandlerError(f'VTK "{self.name}" output has size 0')
        return 0

    def do_it(self):
        return self.solver.write_vtk(self.name, self.what, self.reg)


def _bool(v) -> bool:
    """pugixml as_bool: true for a value starting with 1, t, T, y or Y"""
    return str(v).strip()[:1] in ("1", "t", "T", "y", "Y")


@register("HDF5")
class HDF5(Callback):
    """reference cbHDF5 (src/Handlers/cbHDF5.cpp): region-cropped field output, one HDF5
    file per step (written by the native writer csrc/runtime/h5.cpp, no libhdf5) with an
    XDMF sidecar (``write_xdmf``).  As the reference: chunked datasets whose chunk dims are
    negotiated at start as the GCD of every rank's local extent along z, y and x (a chunk
    never spans two ranks; cbHDF5.cpp:98-126), deflated at level 6 unless
    ``compress="false"`` (cbHDF5.cpp:20-24); ``point_data`` writes node-centred XDMF;
    an explicit ``chunk`` is refused, as the reference refuses it.  Deviation: a chunk is
    capped at 16 MiB by splitting its z (then y) extent along divisors of the negotiated
    one, so chunks stay under the format's 4 GiB chunk-size field and compress in
    parallel.  ``format="binary"`` writes a raw binary file plus .xmf instead."""

    CHUNK_CAP = 16 << 20

    def init(self):
        super().init()
        self.name = self.node.get("name", "HDF5")
        self.what = _what(self.node)
        self.reg = _region_attrs(self, self.solver.total)
        if self.reg[3] * self.reg[4] * self.reg[5] == 0:
            raise HandlerError(f'HDF5 "{self.name}" output has size 0')
        prec = self.node.get("precision")
        calc_double = self.solver.lattice.rdtype.itemsize == 8 if self.solver.lattice else True
        self.double = calc_double if prec is None else prec == "double"
        if prec not in (None, "double", "float"):
            raise HandlerError("HDF5 precision should be double or float")
        self.deflate = _bool(self.node.get("compress", "true"))
        self.point_data = _bool(self.node.get("point_data", "false"))
        if self.node.get("chunk") is not None:
            raise HandlerError("HDF5: supplying chunk size is not yet supported (as in the reference)")
        if self.double != calc_double and self.deflate:
            log.notice("HDF5: writing a different type than the one calculated")
        self.hdf5 = self.node.get("format", "hdf5").lower() != "binary"
        self.xdmf = self.node.get("write_xdmf", "true").lower() in ("true", "1", "yes")
        self.chunk = self._negotiate_chunks() if self.hdf5 else None
        return 0

    def _negotiate_chunks(self):
        """GCD over the ranks of the local output extents (z, y, x); ranks without a part
        of the region take no part (reference cbHDF5::Init)"""
        import math
        sv = self.solver
        lat = sv.lattice
        X0, Y0, Z0, NX, NY, NZ = self.reg
        x0, y0, z0 = lat.slab.offset
        nx, ny, nz = lat.shape
        ext = (min(z0 + nz, Z0 + NZ) - max(z0, Z0), min(y0 + ny, Y0 + NY) - max(y0, Y0),
               min(x0 + nx, X0 + NX) - max(x0, X0))
        mine = ext if min(ext) > 0 else None
        every = [e for e in sv.comm.gather_objects(mine) if e is not None]
        cz, cy, cx = (math.gcd(*[e[k] for e in every]) for k in range(3))
        # cap: the largest divisors of the z (then y) extent keeping a double-vector chunk
        # within CHUNK_CAP
        per = 8 * 3
        while cz > 1 and cz * cy * cx * per > self.CHUNK_CAP:
            cz = max(d for d in range(1, cz) if cz % d == 0)
        while cy > 1 and cz * cy * cx * per > self.CHUNK_CAP:
            cy = max(d for d in range(1, cy) if cy % d == 0)
        log.output(f"Negotiated HDF5 chunks: {cz}x{cy}x{cx}[x3]")
        return (cz, cy, cx)

    def do_it(self):
        return self.solver.write_xdmf(self.name, self.what, self.reg, double=self.double, hdf5=self.hdf5,
                                      write_xdmf=self.xdmf, chunk=self.chunk, deflate=self.deflate,
                                      point_data=self.point_data)


@register("Catalyst")
class Catalyst(Callback):
    """reference cbCatalyst (ParaView in-situ).  ParaView Catalyst is not available in this
    image: the element is accepted, and every ``Iterations`` step falls back to writing a
    VTK dataset that a Catalyst script could post-process offline."""

    def init(self):
        super().init()
        log.warning("Catalyst: ParaView Catalyst not available; writing VTK output instead")
        self.reg = _region_attrs(self, self.solver.total)
        return 0

    def do_it(self):
        return self.solver.write_vtk(self.node.get("name", "Catalyst"), ["all"], self.reg)


@register("Graphics")
class Graphics(Callback):
    """colour frames (PNG) of a z slice every ``Iterations``: the headless counterpart of
    the reference's GLUT window (built with GRAPHICS, src/gpu_anim.h, which shows the
    model's Color() of the middle slice, src/LatticeContainer.inc.cpp.Rt:350-423).
    Attributes: ``name`` (file tag, default Graphics), ``z`` (slice, default middle)."""

    def init(self):
        super().init()
        self.name = self.node.get("name", "Graphics")
        z = self.node.get("z")
        self.z = None if z is None else int(round(self.solver.units.alt(z)))
        return 0

    def do_it(self):
        self.solver.write_frame(self.name, self.z)
        return 0


@register("TXT")
class TXT(Callback):
    def init(self):
        super().init()
        self.name = self.node.get("name", "TXT")
        self.what = _what(self.node)
        self.gzip = self.node.get("gzip", "false").lower() in ("true", "1")
        return 0

    def do_it(self):
        return self.solver.write_txt(self.name, self.what, gzip=self.gzip)


@register("BIN")
class BIN(Callback):
    def init(self):
        super().init()
        self.name = self.node.get("name", "BIN")
        return 0

    def do_it(self):
        return self.solver.write_bin(self.name)


@register("Log")
class Log(Callback):
    """reference cbLog: CSV log, forces ITER_LASTGLOB"""

    def init(self):
        super().init()
        from ..solver import ITER_LASTGLOB
        self.fn = self.solver.out_iter_file(self.node.get("name", "Log"), ".csv")
        self.solver.init_log(self.fn)
        self.old = self.solver.iter_type
        self.solver.iter_type |= ITER_LASTGLOB
        return 0

    def do_it(self):
        self.solver.write_log(self.fn)
        return 0

    def finish(self):
        self.solver.iter_type = self.old
        return 0


@register("Failcheck")
class Failcheck(Callback):
    """reference cbFailcheck (src/Handlers/cbFailcheck.cpp:5-93): NaN scan, LOR, last words"""

    def init(self):
        super().init()
        self.active = False
        self.what = _what(self.node)
        return 0

    def do_it(self):
        if self.active:
            return 0
        self.active = True
        s = self.solver
        fin = False
        import torch
        for q in s.model.quantities:
            if "all" in self.what or q.name in self.what:
                a = s.lattice.quantity(q.name)
                bad = 0.0 if bool(torch.isfinite(a).all().item()) else 1.0
                if s.comm.allreduce_scalar(bad, "max") > 0:
                    log.notice(f"Checking {q.name} discovered NaN")
                    fin = True
                    break
        self.active = False
        if fin:
            log.notice("NaN value discovered. Executing final actions from the Failcheck element before full stop...")
            for c in list(self.node):
                h = make_handler(c, s)
                if h is not None:
                    h.do_it()
            log.notice("Stopping due to Nan value")
            return ITERATION_STOP
        return 0


@register("Stop")
class Stop(Callback):
    """reference cbStop (src/Handlers/cbStop.cpp:12-106)"""

    def init(self):
        super().init()
        from ..solver import ITER_LASTGLOB
        self.checks = []
        for g in self.solver.model.globals_:
            for kind in ("Change", "PercentChange", "Above", "Below"):
                v = self.node.get(g.name + kind)
                if v is not None:
                    self.checks.append([g.name, kind, float(v), -12341234.0])
        if not self.checks:
            raise HandlerError(f"No *Change attribute in {self.node.tag}")
        self.times = int(self.node.get("Times", "1"))
        if self.times < 1:
            raise HandlerError("Minimal number for Times attribute is 1")
        self.score = 0
        self.old = self.solver.iter_type
        self.solver.iter_type |= ITER_LASTGLOB
        return 0

    def do_it(self):
        g = self.solver.lattice.globals
        anyc = 0
        for c in self.checks:
            name, kind, lim, old = c
            v = g.get(name, 0.0)
            if kind == "Change" and abs(old - v) > lim:
                anyc += 1
            elif kind == "PercentChange" and (v == 0 or abs((old - v) / v) > lim):
                anyc += 1
            elif kind == "Above" and v < lim:
                anyc += 1
            elif kind == "Below" and v > lim:
                anyc += 1
            c[3] = v
        self.score = self.score + 1 if anyc == 0 else 0
        log.output(f"Stop criterium score: {self.score}")
        if self.score >= self.times:
            log.notice("Stop.")
            for c in self.checks:
                c[3] = -12341234.0
            self.score = 0
            return ITERATION_STOP
        return 0

    def finish(self):
        self.solver.iter_type = self.old
        return 0


@register("SaveCheckpoint")
class SaveCheckpoint(Callback):
    """reference cbSaveCheckpoint (src/Handlers/cbSaveCheckpoint.cpp:5-107)"""

    def init(self):
        super().init()
        k = self.node.get("keep")
        if k is None:
            self.keep = 1
        elif k == "all":
            self.keep = 0
        else:
            self.keep = int(k)
            if self.keep < 0:
                self.keep = 1
        self.q = collections.deque()
        return 0

    def do_it(self):
        s = self.solver
        fn = s.out_iter_collective_file("checkpoint", "")
        rf = s.out_iter_collective_file("restart", ".xml")
        path = s.save_solution(fn)
        if s.rank == 0:
            self.write_restart(path, rf)
        if self.keep:
            self.q.append((path, rf))
            while len(self.q) > self.keep:
                p, r = self.q.popleft()
                if s.rank == 0:
                    for f in (p, p + ".json", r):
                        if os.path.exists(f):
                            os.remove(f)
        return 0

    def write_restart(self, path, rf):
        cfg = copy.deepcopy(self.solver.config_tree)
        lb = cfg.find("LoadBinary")
        if lb is None:
            solve = cfg.find("Solve")
            idx = list(cfg).index(solve) if solve is not None else len(cfg)
            lb = ET.Element("LoadBinary", {"file": path})
            cfg.insert(idx, lb)
        else:
            lb.set("file", path)
        ET.ElementTree(cfg).write(rf)


@register("SaveBinary", "SaveMemoryDump")
class SaveBinary(Callback):
    def init(self):
        super().init()
        self.name = self.node.get("filename") or self.node.get("file") or "Save"
        return 0

    def do_it(self):
        s = self.solver
        if self.node.get("filename") or self.node.get("file"):
            path = self.name
        else:
            path = s.out_iter_collective_file(self.name, "")
        s.save_solution(path)
        return 0


@register("Average")
class Average(Callback):
    """reference cbAveraging: reset averaged densities"""

    def do_it(self):
        self.solver.lattice.reset_average()
        return 0


@register("DumpSettings")
class DumpSettings(Callback):
    def do_it(self):
        s = self.solver
        if s.rank == 0:
            fn = s.out_iter_file(self.node.get("name", "Settings"), ".csv")
            with open(fn, "w") as f:
                f.write("setting,zone,value\n")
                for st in s.model.settings:
                    if st.zonal:
                        for z in s.lattice.zone_names:
                            f.write(f"{st.name},{z},{s.lattice.get_setting(st.name, z):.13e}\n")
                    else:
                        f.write(f"{st.name},,{s.lattice.get_setting(st.name):.13e}\n")
        return 0


@register("Sample")
class Sample(Callback):
    """reference cbSample + Sampler (src/Handlers/cbSample.cpp:5-60, src/Sampler.cpp:16-99):
    the quantities at the probe points are recorded EVERY iteration on the device
    (tclb_amd.sampler, reference Lattice::updateAllSamples) and written at each callback:
    one CSV row per iteration and point, columns Iteration,X,Y,Z,<quantities> (vectors
    as .x/.y/.z), SI units.  Rows of all ranks are gathered to rank 0, which writes the
    file (the reference lets every owning rank append to it).  The Iteration column is the
    iteration count after the sampled step."""

    def init(self):
        super().init()
        from ..sampler import Sampler as _Probes
        s = self.solver
        if not self.every_iter:
            raise HandlerError("Iteration value in sampler should not be zero")
        self.what = _what(self.node)
        points = []
        for p in self.node:
            if p.tag != "Point":
                raise HandlerError(f"Unknown element in Sampler: {p.tag}")
            x = int(round(s.units.alt(p.get("dx", "0"))))
            y = int(round(s.units.alt(p.get("dy", "0"))))
            z = int(round(s.units.alt(p.get("dz", "0"))))
            if all(0 <= v < n for v, n in zip((x, y, z), s.lattice.gshape)):
                points.append((x, y, z))
        self.fn = s.out_iter_file("Sampler", ".csv")
        qs = [q for q in s.model.quantities if ("all" in self.what or q.name in self.what) and not q.adjoint]
        scales = {q.name: 1.0 / s.units.unit_scale(q.unit) for q in qs}
        self.probes = _Probes(s.lattice, points, [q.name for q in qs], scales, rows=int(math.ceil(self.every_iter)))
        s.lattice.samplers.append(self.probes)
        if s.rank == 0:
            with open(self.fn, "w") as f:
                f.write(",".join(["Iteration", "X", "Y", "Z"] + self.probes.columns) + "\n")
        return 0

    def _write(self):
        s = self.solver
        rows = self.probes.flush()
        if s.comm.distributed:
            rows = [r for part in s.comm.gather_objects(rows) or [] for r in part]
        if s.rank != 0:
            return
        rows.sort(key=lambda r: (r[0], r[1]))
        with open(self.fn, "a") as f:
            for it, _, (x, y, z), v in rows:
                f.write(",".join([str(it), str(x), str(y), str(z)] + [f"{a:.13e}" for a in v]) + "\n")

    def do_it(self):
        self._write()
        return 0

    def finish(self):
        if self.probes in self.solver.lattice.samplers:
            self._write()
            self.solver.lattice.samplers.remove(self.probes)
        return super().finish()


@register("PID")
class PID(Callback):
    """reference cbPID (src/Handlers/cbPID.cpp:94-122): drive a (zonal) setting so that a
    global reaches a target."""

    def init(self):
        super().init()
        n = self.node
        s = self.solver
        self.control = n.get("control")
        self.zone = n.get("zone")
        self.what = None
        self.target = None
        for g in s.model.globals_:
            if n.get(g.name) is not None:
                self.what = g.name
                self.target = s.units.alt(n.get(g.name))
        if self.what is None or self.control is None:
            raise HandlerError("PID needs a <Global>=target attribute and control=")
        self.P = float(n.get("P", "1"))
        self.I = float(n.get("I", "0"))
        self.D = float(n.get("D", "0"))
        self.DT = float(n.get("DerivativeTime", n.get("DT", "0")))
        self.integral = 0.0
        self.prev = None
        from ..solver import ITER_LASTGLOB
        s.iter_type |= ITER_LASTGLOB
        return 0

    def do_it(self):
        s = self.solver
        v = s.lattice.globals.get(self.what, 0.0)
        err = self.target - v
        self.integral += err * self.every_iter
        der = 0.0 if self.prev is None else (err - self.prev) / max(self.every_iter, 1)
        self.prev = err
        u = self.P * (err + self.I * self.integral + self.D * der)
        s.lattice.set_setting(self.control, u, zone=self.zone)
        return 0


@register("Keep")
class Keep(Callback):
    """reference cbKeep (src/Handlers/cbKeep.cpp:45-66): objective constraint weight"""

    def init(self):
        super().init()
        n = self.node
        s = self.solver
        self.items = []
        for g in s.model.globals_:
            for kind in ("Above", "Below", "Equal"):
                v = n.get(g.name + kind)
                if v is not None:
                    self.items.append((g.name, kind, s.units.alt(v)))
        self.force = float(n.get("Force", "1"))
        return 0

    def do_it(self):
        s = self.solver
        for name, kind, thr in self.items:
            v = s.lattice.globals.get(name, 0.0)
            w = self.force * (thr - v)
            if kind == "Above" and v > thr:
                w = 0.0
            if kind == "Below" and v < thr:
                w = 0.0
            s.lattice.set_setting(name + "InObj", w)
        return 0


def _dedent(text: str) -> str:
    import textwrap
    lines = (text or "").split("\n")
    while lines and not lines[0].strip():
        lines.pop(0)
    return textwrap.dedent("\n".join(lines)).rstrip()


@register("RunPython")
class RunPython(Callback):
    """Embedded Python (reference RunR/RunPython, src/Handlers/cbRunR.cpp:687-845): the
    element text runs in one namespace shared by every embedded block of the case, with
    the reference's ``Solver`` object model (handlers/embed.py: Settings, Fields,
    Parameters, Quantities, Globals, Actions, Geometry, Info) and ``np``; the raw
    ``solver`` / ``lattice`` objects are there as well.  Without ``Iterations`` the block
    runs once where it stands, otherwise every ``Iterations``; forces globals on the
    last step (ITER_LASTGLOB) like the reference."""

    def init(self):
        super().init()
        from ..solver import ITER_LASTGLOB
        self.code = _dedent(self.node.text)
        self.tag = f"<{self.node.tag} line {getattr(self.node, 'sourceline', '?')}>"
        self._compiled = compile(self.code, self.tag, "exec") if self.code else None
        self.old = self.solver.iter_type
        self.solver.iter_type |= ITER_LASTGLOB
        return 0

    def do_it(self):
        from .embed import namespace
        s = self.solver
        if self._compiled is None:
            return 0
        log.output(f"{s.iter:8d} it Executing {self.node.tag} code")
        ns = namespace(s)
        ns.update({"solver": s, "lattice": s.lattice, "iteration": s.iter})
        try:
            exec(self._compiled, ns)
        except NameError as e:
            raise HandlerError(f"{self.node.tag}: {e} (names available: Solver, np, solver, lattice)") from e
        return 0

    def finish(self):
        self.solver.iter_type = self.old
        return super().finish()


@register("Control")
class Control(GenericAction):
    """reference conControl (src/Handlers/conControl.cpp:1-257): time-dependent zonal
    settings over a control window of ``Iterations`` steps.

    ``<CSV file= [Time="expr"]>`` reads a table (unit-aware cells) into a context of
    columns sampled at every iteration of the window by piecewise-linear interpolation in
    time; ``Time`` is an expression of the columns (default: rows spread evenly over the
    window).  ``<Param name= [zone=] value="expr"/>`` (inside a CSV or directly in
    Control) sets a zonal setting to a time series.  Expressions follow the reference
    grammar: terms joined by ``+``, each ``Column*scale`` (scale with units), ``Column``
    or a constant with units after the first term, e.g. ``Sin*0.5m+1m``.
    Extension: a CSV without Param children applies every column named like a zonal
    (or ``<setting>-<zone>``) setting directly; global settings named so are set every
    iteration."""

    kind = HANDLER_CALLBACK

    def _expr(self, ctx, expr: str, scale: float) -> np.ndarray:
        s = self.solver
        n = len(next(iter(ctx.values()))) if ctx else 1
        out = np.zeros(n)
        for i, term in enumerate(expr.split("+")):
            parts = term.split("*")
            name = parts[0].strip()
            if name in ctx:
                if len(parts) > 2:
                    raise HandlerError(f"too many '*' in Control expression {expr!r}")
                k = s.units.alt(parts[1]) if len(parts) == 2 else 1.0
                out = out + np.asarray(ctx[name]) * k * scale
            else:
                if i == 0:
                    raise HandlerError(f"variable {name} not found in Control context "
                                       "(syntax: [Variable]*[scale with unit])")
                if len(parts) > 1:
                    raise HandlerError(f"too many '*' in Control expression {expr!r}")
                out = out + s.units.alt(name) * scale
        return out

    def _param(self, node, ctx):
        s = self.solver
        name, zone, value = node.get("name"), node.get("zone"), node.get("value")
        if value is None:
            raise HandlerError("Setting value not specified in Param element")
        if not name:
            raise HandlerError("Setting name not specified in Param element")
        st = s.model.setting(name)
        if st is None or not st.zonal:
            raise HandlerError(f"Unknown (zonal) setting {name} in Control")
        if zone and zone not in s.lattice.zone_names:
            raise HandlerError(f"Unknown zone {zone} (found while setting parameter {name})")
        vals = self._expr(ctx, value, 1.0) if ctx else np.full(self.length, self._expr({}, value, 1.0)[0])
        if len(vals) == 1:
            vals = np.full(self.length, vals[0])
        s.lattice.set_zone_series(name, vals, zone=zone or None)

    def _csv(self, node):
        import csv
        s = self.solver
        fn = node.get("file")
        if fn is None:
            raise HandlerError("No file attribute in CSV in xml config")
        with open(fn) as f:
            rows = [r for r in csv.reader(f) if r]
        if not rows:
            raise HandlerError(f"Empty file CSV {fn}")
        names = [h.strip().strip('"') for h in rows[0]]
        data = {n: [] for n in names}
        for r in rows[1:]:
            if len(r) != len(names):
                raise HandlerError(f"row length does not match the header in CSV file {fn}")
            for n, v in zip(names, r):
                data[n].append(s.units.alt(v.strip()))
        nrow = len(rows) - 1
        if nrow < 2:
            raise HandlerError("Not enough records in CSV file")
        data = {k: np.asarray(v) for k, v in data.items()}
        data["_index"] = np.arange(nrow, dtype=float)
        if node.get("Time") is None:
            t = self._expr(data, "_index", self.length / nrow)
        else:
            t = self._expr(data, node.get("Time"), 1.0)
        it = np.arange(self.length, dtype=float)
        ctx = {n: np.interp(it, t, data[n]) for n in names}
        params = [c for c in node if c.tag == "Param"]
        for c in node:
            if c.tag != "Param":
                raise HandlerError(f"Only Param allowed in CSV in Control (found {c.tag})")
        if params:
            for c in params:
                self._param(c, ctx)
        else:   # extension: columns named like settings
            for col in names:
                name, _, zone = col.partition("-")
                st = s.model.setting(name)
                if st is None or col == node.get("Time"):
                    continue
                if st.zonal:
                    s.lattice.set_zone_series(name, ctx[col], zone=zone or None)
                else:
                    self.series.append((name, ctx[col]))
        self.context.update(ctx)

    def init(self):
        super().init()
        s = self.solver
        self.series = []
        self.context = {}
        self.length = int(round(s.units.alt(self.node.get("Iterations", "0")) or 0))
        if self.length <= 0:
            raise HandlerError("Zero (or less) iterations in Control element in config")
        for c in self.node:
            if c.tag == "CSV":
                self._csv(c)
            elif c.tag == "Param":
                self._param(c, self.context)
            else:
                raise HandlerError(f"Element {c.tag} not allowed in Control element in config")
        self.every_iter = 1.0 if self.series else 0.0
        return 0

    def do_it(self):
        s = self.solver
        for name, v in self.series:
            s.lattice.set_setting(name, float(v[s.iter % len(v)]))
        return 0


@register("SyntheticTurbulence")
class SyntheticTurbulenceAction(Action):
    """reference acSyntheticTurbulence (src/Handlers/acSyntheticTurbulence.cpp)"""

    def _wn(self, name, default=None):
        n = self.node
        s = self.solver
        val = default
        if n.get(name + "WaveLength") is not None:
            val = 1.0 / s.units.alt(n.get(name + "WaveLength"))
        if n.get(name + "WaveNumber") is not None:
            val = s.units.alt(n.get(name + "WaveNumber"))
        if n.get(name + "WaveFrequency") is not None:
            val = s.units.alt(n.get(name + "WaveFrequency")) * 8 * math.atan(1.0)
        return val

    def init(self):
        super().init()
        from ..utils.turbulence import SyntheticTurbulence
        s = self.solver
        nmodes = int(self.node.get("Modes", "100"))
        spec = self.node.get("Spectrum", "Von Karman")
        st = SyntheticTurbulence(seed=int(self.node.get("Seed", "0")))
        if spec == "Von Karman":
            main = self._wn("Main")
            diff = self._wn("Diffusion")
            if main is None or diff is None:
                raise HandlerError("Must provide MainWaveNumber and DiffusionWaveNumber for Von Karman spectrum")
            mx = self._wn("Shortest", 8 * math.atan(1) / 4)
            mn = self._wn("Longest", main / 2)
            st.set_von_karman(nmodes, main, diff, mn, mx, comm=s.comm)
        elif spec == "One Wave":
            st.set_one_wave(self._wn("Main"), comm=s.comm)
        else:
            raise HandlerError(f"Unknown spectrum {spec}")
        tw = self._wn("Time")       # reference setTimeScale (acSyntheticTurbulence.cpp:103-109)
        if tw is None:
            log.notice("TimeWaveNumber not provided for synthetic turbulence")
        else:
            st.time_wn = tw
        s.lattice.set_turbulence(st.modes, st.time_wn)
        s.turbulence = st
        return 0


@register("RemoteForceInterface")
class RemoteForceInterface(Action):
    """reference acRemoteForceInterface (src/Handlers/acRemoteForceInterface.cpp): connects
    the lattice to a particle integrator.  integrator="SIMPLEPART" (or BUILTIN): the
    built-in in-process integrator, configured from the <SimplePart> child as in the
    reference.  Any other integrator runs as another program and couples over the socket
    RFI bridge (particles/rfi.py): the lattice listens on ``address`` (default
    127.0.0.1:0 = any free port) and ``spawn`` (optional) starts the integrator with
    ``{address}`` replaced, e.g.
    ``spawn="python tools/rfi_simplepart.py --address {address} --config parts.json"``.
    The reference launches its integrators MPMD-style (mpirun -np 1 tclb : -np 1 lammps)."""

    def init(self):
        super().init()
        from ..particles import SimplePart
        s = self.solver
        integ = (self.node.get("integrator") or "").upper()
        if integ not in ("SIMPLEPART", "BUILTIN"):
            return self._remote()
        sp = SimplePart()
        u = s.units
        off = [u.alt(s.config_tree.find("Geometry").get("p" + a, "0")) for a in "xyz"]
        cfg = self.node.find("SimplePart")
        lm, ls, lkg = u.alt("1m"), u.alt("1s"), u.alt("1kg")
        if cfg is not None:
            for a, d in (("ax", 0), ("ay", 1), ("az", 2)):
                if cfg.get(a) is not None:
                    sp.acc[d] = float(cfg.get(a)) * lm / ls ** 2
            for c in cfg:
                if c.tag == "Particle":
                    x = [float(c.get(a, "0")) * lm - off[i] for i, a in enumerate("xyz")]
                    v = [float(c.get("v" + a, "0")) * lm / ls for a in "xyz"]
                    w = [float(c.get("omega" + a, "0")) / ls for a in "xyz"]
                    r = float(c.get("r")) * lm
                    mass = float(c.get("m")) * lkg if c.get("m") else None
                    if c.get("log", "n").lower() in ("y", "yes", "true", "1"):
                        sp.logged.append(sp.n)
                    sp.add(x, r, v, w, mass)
                elif c.tag == "Periodic":
                    for i, a in enumerate("xyz"):
                        if c.get(a) is not None:
                            sp.periodic[i] = True
                            sp.period[i] = float(c.get(a)) * lm
                elif c.tag == "Log":
                    sp.log_every = int(c.get("Iterations", "1"))
                    sp.log_rotation = c.get("rotation", "false").lower() in ("true", "1")
                    sp.log_path = c.get("name") or (s.outpath + "_SP_Log.csv")
        for c in self.node:
            if c.tag == "Particle":   # shorthand: particles directly under the element (lattice units)
                sp.add([float(c.get(a, "0")) for a in "xyz"], float(c.get("r")),
                       [float(c.get("v" + a, "0")) for a in "xyz"], fixed=c.get("fixed", "false") == "true")
        s.lattice.particles = sp
        s.particles = sp
        log.output(f"RemoteForceInterface: {sp.n} particle(s) with built-in SIMPLEPART integrator")
        return 0

    def _remote(self):
        import os
        import shlex
        import subprocess
        from ..particles.rfi import RemoteParticles
        s = self.solver
        lat = s.lattice
        u = s.units
        units = {"m": u.alt("1m"), "s": u.alt("1s"), "kg": u.alt("1kg")}
        rp = RemoteParticles(self.node.get("address", "127.0.0.1:0"), comm=lat.comm, units=units,
                             box=list(lat.gshape), timeout=float(self.node.get("timeout", "120")))
        # negotiated variables and statistics (reference acRemoteForceInterface.cpp:26-82):
        # "output", the element's single child as "content", every other attribute as a
        # number in lattice units
        rp.set_var("output", s.outpath)
        kids = list(self.node)
        if len(kids) > 1:
            raise ValueError("only a single element/CDATA allowed inside <RemoteForceInterface>")
        content = None
        if kids:
            import xml.etree.ElementTree as ET
            content = ET.tostring(kids[0], encoding="unicode").strip()
        elif (self.node.text or "").strip():
            content = self.node.text.strip()
        if content is not None:
            rp.set_var("content", content)
        stats, prefix, every = False, s.outpath + "_RFI", 200
        own = ("integrator", "address", "spawn", "timeout", "use_box", "omega", "torque")
        for k, v in self.node.attrib.items():
            if k == "stats":
                stats = v.lower() in ("1", "true", "yes", "y")
            elif k == "stats_iter":
                every, stats = int(round(u.alt(v))), True
            elif k == "stats_prefix":
                prefix, stats = v, True
            elif k not in own:
                rp.set_var(k, "%.15g" % u.alt(v))
        if stats:
            log.output(f"Asking for stats on RFI ({prefix} every {every} it)")
            rp.enable_stats(prefix, every)
        proc = None
        cmd = self.node.get("spawn")
        if cmd and lat.comm.rank == 0:
            cwd = os.path.dirname(os.path.abspath(s.conffile)) if getattr(s, "conffile", None) else None
            proc = subprocess.Popen(shlex.split(cmd.replace("{address}", rp.address)), cwd=cwd)
        log.output(f"RemoteForceInterface: waiting for integrator '{self.node.get('integrator')}' on {rp.address}")
        rp.accept()
        lat.particles = rp
        s.particles = rp

        def stop():
            rp.close()
            if proc is not None:
                proc.wait(timeout=60)
        s.at_exit = getattr(s, "at_exit", []) + [stop]
        return 0


@register("Andersen")
class Andersen(GenericAction):
    """Anderson acceleration of a fixed-point iteration over the whole lattice state
    (reference acAndersen.cpp:45-125, "Option B"): each of ``Times`` rounds runs the
    children once from x to G(x), orthogonalises the newest residual e = G(x) - x against
    the previous ``Directions`` ones (Gram-Schmidt, the same on the states) and restarts
    from the least-squares combination of the stored states.  State vectors stay on the
    device (torch); dot products are all-reduced over ranks."""

    def init(self):
        super().init()
        s = self.solver
        lat = s.lattice
        if self.node.get("Directions") is None:
            raise HandlerError("no Directions parameter in Andersen")
        dirs = int(self.node.get("Directions"))
        times = int(self.node.get("Times", str(dirs)))
        eps = float(self.node.get("Eps", "0"))

        def skal(a, b):
            return lat.comm.allreduce_scalar(float(torch.dot(a.reshape(-1), b.reshape(-1))), "sum")

        X, E, P = [], [], []
        d = 0
        self.residuals = []
        for _ in range(times):
            x0 = lat.fields_interior().clone()
            self.execute_internal()
            self.unstack()
            e0 = lat.fields_interior().clone() - x0
            r = skal(e0, e0)
            self.residuals.append(r)
            log.notice(f"Residual in Andersen: {r:g}")
            if not math.isfinite(r) or r < eps:
                break
            X.insert(0, x0); E.insert(0, e0); P.insert(0, 1.0)
            del X[dirs:], E[dirs:], P[dirs:]
            d = min(d + 1, dirs)
            for j in range(1, d):
                a = skal(E[0], E[j])
                E[0] -= a * E[j]
                X[0] -= a * X[j]
                P[0] -= a * P[j]
            a = math.sqrt(skal(E[0], E[0]))
            E[0] /= a
            X[0] /= a
            P[0] /= a
            psum = sum(p * p for p in P[:d])
            nx = sum(X[i] * (P[i] / psum) for i in range(d))
            lat.set_fields_interior(nx)
            self.execute_internal()
            self.unstack()
        return 0


@register("RunR")
class RunR(Callback):
    """reference cbRunR (src/Handlers/cbRunR.cpp:806-872) embeds an R interpreter.  There
    is no R runtime in this framework: ``python="true"`` runs the element text as
    RunPython does; anything else stops the case with an explicit error instead of
    silently skipping the user's code."""

    def init(self):
        super().init()
        if self.node.get("python", "false").lower() not in ("true", "1", "yes"):
            raise HandlerError("RunR: no embedded R interpreter in tclb_amd; "
                               "use <RunPython> (or RunR python=\"true\") with the equivalent Python code")
        return RunPython.init(self)

    def do_it(self):
        return RunPython.do_it(self)

    def finish(self):
        return RunPython.finish(self)


@register("ESYSParticle")
class ESYSParticle(Action):
    """reference acESYSParticle spawns the ESYS-Particle DEM code over MPMD.  External
    DEM codes are not part of this build: particle coupling uses the in-process
    integrator of <RemoteForceInterface integrator="SIMPLEPART">."""

    def init(self):
        super().init()
        raise HandlerError("ESYSParticle: external ESYS-Particle coupling is not available; "
                           "use <RemoteForceInterface integrator=\"SIMPLEPART\">")
