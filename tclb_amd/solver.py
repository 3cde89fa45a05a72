"""Solver facade: case set-up, output naming, logs, handler stack.

Re-design of the reference's Solver + main() (reference: src/Solver.h.Rt:60-187,
src/Solver.cpp.Rt, src/main.cpp:173-425).  The whole run happens inside the root
handler's init (CLBConfig), exactly as in the reference (src/main.cpp:404-410).
"""
from __future__ import annotations

import copy
import json
import os
import time
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .geometry.geometry import Geometry
from .lattice import Lattice
from .models import registry
from .parallel.comm import Comm, LoopbackComm, init_distributed_from_env
from .utils.log import log
from .utils.units import UnitEnv, UnitVal

ITER_NORM = 0x00
ITER_GLOBS = 0x01
ITER_LASTGLOB = 0x02
ITER_OPT = 0x10          # combined primal + steady adjoint + descent (reference ITER_OPT)
ITERATION_STOP = 1


class SolverError(RuntimeError):
    pass


class Solver:
    def __init__(self, model: str, config: ET.Element, conffile: str = "case.xml", device: Optional[str] = None,
                 precision: str = "double", comm: Optional[Comm] = None, block=(0, 0)):
        self.model_name = model
        self.model = registry.get(model)
        from .utils.xpath import rewrite_deprecated_params
        n = rewrite_deprecated_params(config)
        if n:
            log.warning(f"{n} deprecated Params elements found. Changing them to Param")
        self.config_tree = config
        self.conffile = conffile
        self.comm = comm or LoopbackComm()
        self.rank = self.comm.rank
        self.size = self.comm.size
        self.precision = precision
        self.block = block
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        if device == "cuda":
            # one GPU per rank of a node (reference main.cpp:318-350): more ranks than GPUs
            # is refused unless the case sets oversubscribe_gpu="true"
            local = int(os.environ.get("LOCAL_RANK", "0"))
            count = max(1, torch.cuda.device_count())
            if local >= count:
                if config.get("oversubscribe_gpu", "false").lower() not in ("true", "1", "yes"):
                    raise SolverError("Oversubscribing GPUs. This is not a good idea, but if you want to do it, "
                                      'add oversubscribe_gpu="true" to the config file')
                log.warning("Oversubscribing GPUs.")
            self.device = torch.device("cuda", local % count)
        else:
            self.device = torch.device(device)
        self.units = UnitEnv()
        self.iter = 0
        self.steps = 1
        self.iter_type = ITER_NORM
        self.opt_iter = 0
        self.hands: List = []
        self.lattice: Optional[Lattice] = None
        self.geometry: Optional[Geometry] = None
        self.outpath = ""
        self.permissive = (config.get("permissive", "false").lower() in ("true", "1", "yes"))
        self.start_time = time.time()
        self.log_scales: Dict[str, float] = {}
        self.set_output(config.get("output", ""))
        self._meter_t = time.time()
        self._meter_it = 0

    # ------------------------------------------------------------------ setup
    def read_units(self):
        """reference readUnits (src/main.cpp:31-63) + Solver::setUnit (src/Solver.cpp.Rt:90-103)"""
        u = self.config_tree.find("Units")
        if u is None:
            return
        for i, p in enumerate(u.findall("Param")):
            if p.get("value") is None or p.get("gauge") is None:
                raise SolverError("Units Param needs value and gauge")
            name = p.get("name", f"unnamed{i + 1}")
            self.units.set_unit(name, self.units.read_text(p.get("value")) / self.units.read_text(p.get("gauge")), 1.0)
        self.units.make_gauge()

    def set_size(self):
        g = self.config_tree.find("Geometry")
        if g is None:
            raise SolverError("no Geometry element")
        nx = int(round(self.units.alt(g.get("nx", "1"), 1)))
        ny = int(round(self.units.alt(g.get("ny", "1"), 1)))
        nz = int(round(self.units.alt(g.get("nz", "1"), 1)))
        log.notice(f"Mesh size in config file: {nx}x{ny}x{nz}")
        self.lattice = Lattice(self.model, (nx, ny, nz), device=self.device, precision=self.precision,
                               comm=self.comm, block=self.block)
        self.total = (0, 0, 0, nx, ny, nz)

    def set_output(self, out: str):
        base = os.path.splitext(os.path.basename(self.conffile))[0]
        self.outpath = f"{out}{base}"

    def out_iter_file(self, name: str, suffix: str) -> str:
        p = f"{self.outpath}_{name}_P{self.rank:02d}_{self.iter:08d}{suffix}"
        os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        return p

    def out_global_file(self, name: str, suffix: str) -> str:
        p = f"{self.outpath}_{name}_P{self.rank:02d}{suffix}"
        os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        return p

    def out_iter_collective_file(self, name: str, suffix: str) -> str:
        p = f"{self.outpath}_{name}_{self.iter:08d}{suffix}"
        os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        return p

    # ------------------------------------------------------------------ running
    def run(self):
        from .handlers.base import make_handler
        self.read_units()
        self.set_size()
        try:
            root = make_handler(self.config_tree, self)
            if root is None:
                raise SolverError("root handler failed")
            root.finish()
        finally:
            # end-of-run hooks (e.g. the RFI death protocol towards a remote integrator)
            for fn in reversed(getattr(self, "at_exit", [])):
                fn()
        return 0

    def iterate(self, steps: int, action: Optional[str] = None):
        """one Solve segment (reference Lattice::Iterate with iter_type)"""
        lat = self.lattice
        glob = bool(self.iter_type & (ITER_LASTGLOB | ITER_GLOBS))
        if self.iter_type & ITER_OPT:
            for k in range(steps):
                # the primal step writes the other snapshot and leaves its input intact:
                # after it, snaps[1 - cur] is the pre-step state the adjoint linearises at
                lat.iterate(1, glob_last=glob and k == steps - 1, action=action or "Iteration")
                self._opt_iteration(action or "Iteration", lat.snaps[1 - lat.cur])
            self.iter += steps
            self._speed_meter(steps)
            return
        if action is None:
            lat.iterate(steps, glob_last=glob)
        else:
            lat.iterate(steps, glob_last=glob, action=action)
        self.iter += steps
        self._speed_meter(steps)

    def _opt_iteration(self, action: str, pre_state):
        """the Optimize part of one ITER_OPT iteration (reference Lattice::<Action>_Opt,
        src/Lattice.cu.Rt:624-636 and the Opt() node function, src/cuda.cu.Rt:241-253):
        one steady-adjoint step linearised at the pre-step primal state (the reference's
        Iteration_Adj(tab0, ...) after Iteration(tab0 -> tab1)), then on DesignSpace nodes
        every parameter density of the new state moves by Descent x its adjoint, clamped
        to [0, 1]"""
        lat = self.lattice
        ad = self.opt_adjoint
        self.opt_state = ad.steady_step(self.opt_state, action, state=pre_state)
        descent = lat.get_setting("Descent") if self.model.setting("Descent") is not None else 0.0
        pf = ad.param_fields()
        if not pf or descent == 0.0:
            return
        m = self.model
        mask = m.group_masks.get("DESIGNSPACE")
        nx, ny, nz = lat.shape
        sl = (slice(lat.gz, lat.gz + nz), slice(lat.gy, lat.gy + ny), slice(0, nx))
        fl = lat.flags[sl].to(torch.int64) & 0xFFFFFFFF
        ds = m.node_type("DesignSpace")
        sel = ((fl & mask) == ds.value) if (mask and ds is not None) else torch.ones_like(fl, dtype=torch.bool)
        cur = lat.snaps[lat.cur]
        for i in pf:
            p = cur[i][sl]
            upd = (p + self.opt_state[i][sl] * descent).clamp_(0.0, 1.0)
            p.copy_(torch.where(sel, upd, p))

    def _speed_meter(self, steps: int):
        """reference MainCallback (src/main.cpp:68-157): MLBUps / GB/s"""
        self._meter_it += steps
        now = time.time()
        dt = now - self._meter_t
        if dt > 1.0:
            if self.lattice.is_gpu:
                torch.cuda.synchronize()
                now = time.time()
                dt = now - self._meter_t
            mlups = self.lattice.nodes * self._meter_it / dt / 1e6
            es = self.lattice.snaps[0].element_size()
            gbs = mlups * (2 * self.lattice.nf * es + self.lattice.flags.element_size()) / 1e3
            log.output(f"{self.iter:8d} it {mlups:8.1f} MLBUps {gbs:7.2f} GB/s")
            self._meter_t = now
            self._meter_it = 0

    # ------------------------------------------------------------------ outputs
    def quantity_si(self, name: str) -> np.ndarray:
        q = next(q for q in self.model.quantities if q.name == name)
        v = self.units.unit_scale(q.unit)
        return self.lattice.quantity(name, scale=1.0 / v).cpu().numpy()

    def output_fields(self, what: Optional[Sequence[str]]):
        """(name, array (nz,ny,nx) or (3,nz,ny,nx), ncomp) of the selected flag groups and
        quantities (SI units) on this rank's slab (reference vtkWriteLattice selection)"""
        lat = self.lattice
        allq = what is None or "all" in what
        fields = []
        flags = lat.get_flags()
        if what is not None and "flag" in what:
            fields.append(("flag", flags.astype(np.uint16 if self.model.flag_bits == 16 else np.uint32), 1))
        for gname in sorted(self.model.group_masks):
            if gname in ("ALL", "NONE"):
                continue
            if (allq and gname != "SETTINGZONE" and gname in {n.group for n in self.model.node_types}) or \
                    (what is not None and gname in what):
                mask = self.model.group_masks[gname]
                shift = self.model.group_shift.get(gname, 0)
                fields.append((gname, ((flags & mask) >> shift).astype(np.uint8), 1))
        for q in self.model.quantities:
            if allq or (what is not None and q.name in what):
                a = self.quantity_si(q.name)
                if q.vector:
                    fields.append((q.name, a, 3))
                else:
                    fields.append((q.name, a[0], 1))
        return fields

    def write_frame(self, name: str = "Graphics", z: Optional[int] = None) -> str:
        """colour frame of a z slice as PNG (io/render.py; the headless counterpart of the
        reference's GLUT window): <out>_<name>_<iter>.png, written by the root rank"""
        from .io import render
        fn = self.out_iter_collective_file(name, ".png")
        if self.rank == 0:
            log.output(f"{self.iter:8d} it writing frame {fn}")
        render.write_png(self.lattice, fn, z)
        return fn

    def write_vtk(self, name: str, what: Optional[Sequence[str]], region=None):
        from .io import vtk
        lat = self.lattice
        fn = self.out_iter_file(name, ".vti")
        log.output(f"{self.iter:8d} it writing vtk {fn}")
        fields = self.output_fields(what)
        sx, sy, sz = lat.slab.offset
        nx, ny, nz = lat.shape
        reg = (sx, sy, sz, nx, ny, nz)
        region = region or self.total
        sub = _crop(fields, reg, region)
        spacing = 1.0 / self.units.alt("1m") if self.units.alt("1m") != 0 else 1.0
        if sub is not None:
            lreg, lfields = sub
            vtk.write_vti(fn, region, lreg, lfields, spacing=spacing)
        regs = self.comm.gather_objects(sub[0] if sub is not None else None)
        names = self.comm.gather_objects(os.path.basename(fn) if sub is not None else None)
        if self.rank == 0:
            pieces = [(r, n) for r, n in zip(regs, names) if r is not None]
            meta = [(nme, vtk._VTK_T[np.asarray(a).dtype], nc) for nme, a, nc in fields]
            vtk.write_pvti(fn[:-4] + ".pvti", region, pieces, meta, spacing=spacing)
        return 0

    def write_xdmf(self, name: str, what: Optional[Sequence[str]], region=None, double: bool = True,
                   hdf5: bool = True, write_xdmf: bool = True, chunk: Optional[Tuple[int, int, int]] = None,
                   deflate: bool = True, point_data: bool = False):
        """HDF5 callback output (reference hdf5WriteLattice + XDMF, src/hdf5Lattice.cpp:26-339):
        one HDF5 file per step with a dataset per flag group (uint8) and per selected
        quantity (vectors (nz, ny, nx, 3)) over the output region, written by the native
        writer (csrc/runtime/h5.cpp), and an XDMF sidecar (point_data: node-centred, as the
        reference's HDF5_WRITE_POINT).  chunk (z, y, x): chunked datasets, deflated at level
        6 unless deflate=False (the reference's default) — every rank compresses its own
        chunks, rank 0 lays out the metadata and chunk indexes from the gathered chunk
        sizes, every rank writes its chunks at the addresses it is handed.  chunk=None:
        contiguous datasets, every rank pwrite()s its slab rows.  hdf5=False writes the
        same blocks as one raw binary file instead."""
        from .io import xdmf
        lat = self.lattice
        fields = self.output_fields(what)
        region = region or self.total
        sx, sy, sz = lat.slab.offset
        nx, ny, nz = lat.shape
        sub = _crop(fields, (sx, sy, sz, nx, ny, nz), region)
        # one collective file per step, as the reference's outIterCollectiveFile(nm, ".h5")
        base = self.out_iter_collective_file(name, "")
        spacing = 1.0 / self.units.alt("1m") if self.units.alt("1m") != 0 else 1.0
        dt = np.float64 if double else np.float32
        meta = [(n, (np.dtype(dt) if np.asarray(a).dtype.kind == "f" else np.asarray(a).dtype), nc)
                for n, a, nc in fields]
        layout = xdmf.layout(region, meta)
        data = base + (".h5" if hdf5 else ".bin")
        X0, Y0, Z0, rnx, rny, rnz = region
        if hdf5 and chunk is not None:
            self._write_h5_chunked(data, region, sub, meta, chunk, 6 if deflate else -1)
        elif hdf5:
            # dataset data blocks at the offsets the native writer chose (rank 0)
            from .ops.host import h5_create
            shapes = [(n, dt, (rnz, rny, rnx) + ((nc,) if nc > 1 else ())) for n, dt, nc, _ in layout]
            offs = None
            if self.rank == 0:
                log.output(f"{self.iter:8d} it writing hdf5 {data}")
                os.makedirs(os.path.dirname(data) or ".", exist_ok=True)
                offs = h5_create(data, shapes)
            offs = self.comm.bcast_object(offs)
            layout = [(n, dt, nc, o) for (n, dt, nc, _), o in zip(layout, offs)]
        elif self.rank == 0:
            log.output(f"{self.iter:8d} it writing xdmf {base}.xmf")
            xdmf.create(data, layout)
        if not (hdf5 and chunk is not None):
            self.comm.barrier()
            if sub is not None:
                lreg, lfields = sub
                xdmf.write_piece(data, region, lreg, [(n, np.asarray(a).astype(t, copy=False), nc)
                                                    for (n, a, nc), (_, t, _) in zip(lfields, meta)], layout)
        self.comm.barrier()
        if self.rank == 0 and (write_xdmf or not hdf5):
            xdmf.write_xmf(base + ".xmf", os.path.basename(data), region, layout, spacing,
                           time=self.iter * self.units.alt("1s") if self.units.alt("1s") else self.iter, hdf5=hdf5,
                           point_data=point_data)
        return 0

    def _write_h5_chunked(self, data: str, region, sub, meta, chunk, level: int):
        """chunked (and deflated) HDF5 datasets: each rank packs the chunks of its block,
        rank 0 writes the metadata from the gathered chunk lists, each rank writes its
        chunks (one run per dataset) at the addresses rank 0 hands out"""
        from .ops.host import h5_chunk_pack, h5_create_chunked
        X0, Y0, Z0, rnx, rny, rnz = region
        blobs, info = [], None
        if sub is not None:
            (x0, y0, z0, _, _, _), lfields = sub
            info = []
            for (n, a, nc), (_, t, _) in zip(lfields, meta):
                a = np.asarray(a)
                if nc > 1:
                    a = np.moveaxis(a, 0, -1)                # (nz, ny, nx, nc)
                a = np.ascontiguousarray(a.astype(np.dtype(t).newbyteorder("<"), copy=False))
                cd = tuple(chunk) + ((nc,) if nc > 1 else ())
                blob, sizes = h5_chunk_pack(a, cd, level)
                grid = [a.shape[k] // cd[k] for k in range(a.ndim)]
                o0 = (z0 - Z0, y0 - Y0, x0 - X0, 0)
                offs = [tuple(o0[k] + idx[k] * cd[k] for k in range(a.ndim))
                        for idx in np.ndindex(*grid)]
                blobs.append(blob)
                info.append((offs, [int(v) for v in sizes]))
        every = self.comm.gather_objects(info)
        addrs = None
        if self.rank == 0:
            log.output(f"{self.iter:8d} it writing hdf5 {data}")
            os.makedirs(os.path.dirname(data) or ".", exist_ok=True)
            shapes, cdims, chunks = [], [], []
            for i, (n, t, nc) in enumerate(meta):
                shapes.append((n, t, (rnz, rny, rnx) + ((nc,) if nc > 1 else ())))
                cdims.append(tuple(chunk) + ((nc,) if nc > 1 else ()))
                chunks.append([(o, s) for r in every if r is not None for o, s in zip(*r[i])])
            flat = h5_create_chunked(data, shapes, cdims, level, chunks)
            # the address of each rank's first chunk per dataset (its chunks are one run)
            addrs, k = [], [0] * len(meta)
            for r in every:
                if r is None:
                    addrs.append(None)
                    continue
                row = []
                for i in range(len(meta)):
                    row.append(flat[i][k[i]] if r[i][0] else 0)
                    k[i] += len(r[i][0])
                addrs.append(row)
        mine = self.comm.scatter_objects(addrs) if self.comm.size > 1 else addrs[0]
        self.comm.barrier()
        if sub is not None:
            fd = os.open(data, os.O_WRONLY)
            try:
                for blob, at in zip(blobs, mine):
                    if blob.size:
                        os.pwrite(fd, blob.tobytes(), at)
            finally:
                os.close(fd)

    def write_txt(self, name: str, what: Optional[Sequence[str]], gzip: bool = False):
        prefix = self.out_iter_file(name, "")
        for q in self.model.quantities:
            if what is None or "all" in what or q.name in what:
                a = self.quantity_si(q.name)
                fn = f"{prefix}_{q.name}.txt"
                arr = a.reshape(a.shape[0], -1).T
                if gzip:
                    import gzip as gz
                    with gz.open(fn + ".gz", "wt") as f:
                        np.savetxt(f, arr)
                else:
                    np.savetxt(fn, arr)
        return 0

    def write_bin(self, name: str):
        """raw dump of every stored field (reference binWriteLattice, src/vtkLattice.cpp:56-80)"""
        prefix = self.out_iter_file(name, "")
        f = self.lattice.fields_interior().cpu().numpy()
        for i, fl in enumerate(self.model.fields):
            f[i].tofile(f"{prefix}_{fl.nicename}.bin")
        return 0

    # ---- CSV log (reference Solver::initLog/writeLog, src/Solver.cpp.Rt:120-206)
    def _log_columns(self):
        lat = self.lattice
        cols = []
        for s in self.model.global_settings:
            cols.append((s.name, lambda s=s: lat.get_setting(s.name), s.unit))
        for s in self.model.zonal_settings:
            for z in sorted(lat.zone_names):
                cols.append((f"{s.name}-{z}", lambda s=s, z=z: lat.get_setting(s.name, z), s.unit))
        for g in self.model.globals_:
            cols.append((g.name, lambda g=g: lat.globals.get(g.name, 0.0), g.unit))
        return cols

    def init_log(self, fn: str):
        if self.rank != 0:
            return
        cols = self._log_columns()
        hdr = ['"Iteration"', '"Time_si"', '"Walltime"', '"Optimization"']
        for n, _, _ in cols:
            hdr += [f'"{n}"', f'"{n}_si"']
        hdr += ['"dx_si"', '"dt_si"', '"dm_si"']
        with open(fn, "w") as f:
            f.write(",".join(hdr) + "\n")

    def write_log(self, fn: str):
        if self.rank != 0:
            return
        dt = 1.0 / self.units.alt("1s")
        row = [f"{self.iter}", f"{dt * self.iter:.13e}", f"{time.time() - self.start_time:.13e}", f"{self.opt_iter}"]
        for n, get, unit in self._log_columns():
            v = get()
            sc = 1.0 / self.units.unit_scale(unit)
            row += [f"{v:.13e}", f"{v * sc:.13e}"]
        row += [f"{1.0 / self.units.alt('1m'):.13e}", f"{dt:.13e}", f"{1.0 / self.units.alt('1kg'):.13e}"]
        with open(fn, "a") as f:
            f.write(", ".join(row) + "\n")

    # ---- checkpoints (portable: global-index layout, any rank count)
    def save_solution(self, prefix: str) -> str:
        from .io.checkpoint import save_state
        return save_state(self, prefix)

    def load_solution(self, path: str, comp: Optional[str] = None):
        from .io.checkpoint import load_state
        load_state(self, path, comp=comp)


def _crop(fields, reg, region):
    """crop local arrays (covering reg) to the output region; returns (lreg, fields)"""
    x0, y0, z0, nx, ny, nz = reg
    X0, Y0, Z0, NX, NY, NZ = region
    a0, a1 = max(x0, X0), min(x0 + nx, X0 + NX)
    b0, b1 = max(y0, Y0), min(y0 + ny, Y0 + NY)
    c0, c1 = max(z0, Z0), min(z0 + nz, Z0 + NZ)
    if a1 <= a0 or b1 <= b0 or c1 <= c0:
        return None
    out = []
    for name, a, nc in fields:
        if nc > 1:
            out.append((name, a[:, c0 - z0:c1 - z0, b0 - y0:b1 - y0, a0 - x0:a1 - x0], nc))
        else:
            out.append((name, a[c0 - z0:c1 - z0, b0 - y0:b1 - y0, a0 - x0:a1 - x0], nc))
    return (a0, b0, c0, a1 - a0, b1 - b0, c1 - c0), out
