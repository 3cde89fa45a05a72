"""Lattice runtime: snapshots, settings, zones, stages/actions, halos, globals.

MI355X-native re-design of the reference's ``Lattice`` (reference: src/Lattice.h.Rt:39-191,
src/Lattice.cu.Rt).  Differences by design:

* A snapshot is ONE device tensor ``[nfields][nz+2g][ny][px]`` (SoA, x fastest, x
  pitch padded to 64 elements = 512 B rows in fp64) with contiguous ghost planes on
  the decomposed axis, instead of 27 margin blocks per snapshot.
* Settings live in a small device array read through the scalar cache (no
  ``__constant__`` re-upload per launch, cf. CopyToConst src/LatticeContainer.inc.cpp.Rt:294).
* A stage is one kernel over a box; with >1 rank the box is split into border planes
  and interior so that the halo exchange (RCCL P2P over xGMI) overlaps the interior
  kernel (reference: RunBorder -> MPIStream_A -> RunInterior -> MPIStream_B,
  src/Lattice.cu.Rt:466-533).
* Globals: device fp64 accumulators, all-reduced (SUM then MAX) across ranks
  (reference: MPI_Reduce to rank 0, src/Lattice.cu.Rt:1279-1315).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .models import registry
from .models.dsl import Model
from .ops import abi
from .parallel.comm import Comm, LoopbackComm
from .parallel.decomp import Slab, decompose
from .parallel.native import NativeLoop, native_dist_enabled
from .utils import trace

_FLAGS_GEN = iter(range(1, 2 ** 31 - 1))      # process-unique node-type identities

_SAFE_MATH = {k: getattr(math, k) for k in ("sqrt", "exp", "log", "sin", "cos", "tan", "atan", "atan2", "pi",
                                              "pow", "fabs", "floor", "ceil", "tanh", "sinh", "cosh", "acos", "asin")}
_SAFE_MATH["abs"] = abs
_SAFE_MATH["min"] = min
_SAFE_MATH["max"] = max


def eval_expr(expr: str, env: Dict[str, float]) -> float:
    return float(eval(expr, {"__builtins__": {}}, {**_SAFE_MATH, **env}))


FIXED_POINT_SWEEPS = 100   # reference: for (int fix=0; fix<100; fix++), src/Lattice.cu.Rt:484


def _runs(idx: Sequence[int]) -> List[Tuple[int, int]]:
    """contiguous runs [a, b) of a sorted index list"""
    out = []
    for i in sorted(idx):
        if out and out[-1][1] == i:
            out[-1][1] = i + 1
        else:
            out.append([i, i + 1])
    return [(a, b) for a, b in out]


class Lattice:
    def __init__(self, model, shape: Tuple[int, int, int], device: Optional[torch.device] = None,
                 precision: str = "double", comm: Optional[Comm] = None, block: Tuple[int, int] = (0, 0),
                 overlap: Optional[bool] = None, variant: Optional[str] = None, ghosts: Optional[bool] = None,
                 native_loop: Optional[bool] = None, grid: Optional[Tuple[int, int]] = None):
        self.model: Model = registry.get(model) if isinstance(model, str) else model.finalize()
        m = self.model
        self.comm = comm or LoopbackComm()
        gnx, gny, gnz = (list(shape) + [1, 1])[:3]
        if m.dims == 2 and gnz != 1:
            raise ValueError(f"2-D model {m.name} needs nz=1")
        self.gshape = (gnx, gny, gnz)
        hx, hy, hz = m.halo()
        # 1-D slab, or a Y x Z grid (grid=(py, pz), env TCLB_GRID="py,pz", or automatic
        # when the slab axis is too thin for the rank count; parallel/decomp.py)
        if grid is None and os.environ.get("TCLB_GRID"):
            grid = tuple(int(v) for v in os.environ["TCLB_GRID"].split(","))
        self.slab: Slab = decompose(gnx, gny, gnz, self.comm.rank, self.comm.size, halo=max(1, hz if gnz > 1 else hy),
                                    grid=grid, halo_y=max(1, hy))
        ax = self.slab.axis
        # ghost planes on the decomposed axis only when ranks exchange halos; a single
        # rank wraps periodically inside the kernel (Addr::off) and copies nothing
        self.ghosts = (self.comm.distributed or ax == 3) if ghosts is None else bool(ghosts)
        self.g = max(1, hz if ax == 2 else hy) if self.ghosts else 0
        nx, ny, nz = self.slab.local_shape
        self.shape = (nx, ny, nz)
        self.gy = self.g if ax == 1 else 0
        self.gz = self.g if ax == 2 else 0
        if ax == 3:                       # ghosts on both split axes
            self.gy, self.gz = max(1, hy), max(1, hz)
            self.g = max(self.gy, self.gz)
        if ax == 2 and hy > ny:
            raise ValueError("y stencil larger than domain")
        self.px = ((nx + 63) // 64) * 64 if nx >= 64 else ((nx + 7) // 8) * 8
        # optional extra x pitch (elements, a multiple of 64, env TCLB_X_PAD): moves the
        # rows of power-of-two lattices off a common HBM channel stride; 0 = none
        xpad = int(os.environ.get("TCLB_X_PAD", "0"))
        if xpad and nx >= 64:
            self.px += (xpad + 63) // 64 * 64
        self.NY = ny + 2 * self.gy
        self.NZ = nz + 2 * self.gz
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.is_gpu = self.device.type == "cuda"
        if precision not in abi.PRECISIONS:
            raise ValueError(f"unknown precision {precision!r}: one of {', '.join(abi.PRECISIONS)}")
        self.precision = precision
        self.prec, self.storage_shift = abi.PRECISIONS[precision]
        self.sdtype = {0: torch.float64, 1: torch.float32, 2: torch.float32, 3: torch.float16}[self.prec]
        self.rdtype = torch.float64 if self.prec in (0, 2) else torch.float32
        # per-field storage shift (f - w_i) of the *-shift modes, as a (nf,1,1,1) tensor
        self._shift_t = None
        if self.storage_shift:
            from .emit.emitter import field_shifts
            self._shift_t = torch.tensor(field_shifts(m), dtype=torch.float64, device=self.device).view(-1, 1, 1, 1)
        nf = len(m.fields)
        self.nf = nf
        plane = self.NZ * self.NY * self.px
        # optional padding between field planes (elements, env TCLB_FIELD_PAD): staggers
        # the 2 x nf concurrent HBM streams across channels; 0 = dense
        self.field_pad = int(os.environ.get("TCLB_FIELD_PAD", "0"))
        self.fs = plane + self.field_pad
        if self.fs >= 2 ** 31:
            raise ValueError("local field exceeds 2^31 elements; use more ranks")
        self.placement = None
        self.snaps = self._alloc_snapshots()
        self.cur = 0
        fdt = torch.int16 if m.flag_bits == 16 else torch.int32
        self.flags = torch.zeros((self.NZ, self.NY, self.px), dtype=fdt, device=self.device)
        # identity of the node types, process-unique and renewed by every change
        # (flags_changed): keys caches of the node types (the adjoint's dual flags, the GPU
        # executor's class tile lists of split stages, Launch.flags_gen)
        self.flags_version = next(_FLAGS_GEN)
        self._kept_cache: Dict[str, List[int]] = {}
        self._fields_gen = 0              # bumped by set_fields_interior (setting-derived kept fields)
        self._fill_state = None
        self._iterating = False
        # settings
        self.gsettings = [s.name for s in m.global_settings]
        self.zsettings = [s.name for s in m.zonal_settings]
        self.svals = np.zeros(max(1, len(self.gsettings)), dtype=np.float64)
        self.zone_names: Dict[str, int] = {"DefaultZone": 0}
        self.zvals = np.zeros((max(1, len(self.zsettings)), 1), dtype=np.float64)
        # time derivatives of the zonal settings (reference ZoneSettings _DT tables), set by
        # time-dependent controls; uploaded after the values: zonal[(NZS + i) * nzones + z]
        self.zdt = np.zeros_like(self.zvals)
        # time series of zonal settings (reference ZoneSettings with len > 1):
        # (setting index, zone index) -> values; entry (iter % len) is active in an iteration
        self.zseries: Dict[tuple, np.ndarray] = {}
        self._settings_dirty = True
        self._glob_flags = 0
        self.settings_t = torch.zeros(self.svals.shape, dtype=torch.float64, device=self.device)
        self.zonal_t = torch.zeros(self.zvals.size, dtype=torch.float64, device=self.device)
        # globals accumulator: GSLOTS slots of gstride(NG) doubles (core.hpp TCLB_GSLOTS);
        # the GPU blocks add into slot (block % GSLOTS), the CPU executor into slot 0
        self._gstride = abi.gstride(max(1, len(m.globals_)))
        self.globals_t = torch.zeros(abi.GSLOTS * self._gstride, dtype=torch.float64, device=self.device)
        self.globals: Dict[str, float] = {g.name: 0.0 for g in m.globals_}
        self.iter = 0
        self.block = block
        self.overlap = self.comm.distributed if overlap is None else overlap
        self._halo_stream = None          # side stream of the Y x Z grid's two-phase halo
        # overlapped steps pack their outgoing halo inside the border kernels (Launch.mbase);
        # TCLB_HALO_MIRROR=0 keeps the separate pack kernels (A/B)
        self.halo_mirror = os.environ.get("TCLB_HALO_MIRROR", "1") != "0"
        kind = "hip" if self.is_gpu else "cpu"
        self.lib = abi.load(m.name, kind, variant=variant)
        # halo field sets per split axis: fields read from below (stencil min < 0) /
        # above (max > 0) along that axis
        self.halo_sets = {a: ([i for i, f in enumerate(m.fields) if f.stencil[a][0] < 0],
                              [i for i, f in enumerate(m.fields) if f.stencil[a][1] > 0])
                          for a in ((1, 2) if ax == 3 else (ax,))}
        self.halo_lo, self.halo_hi = self.halo_sets[2 if ax == 3 else ax]
        self._halo_bufs = {}
        self._dist = None                 # NativeLoop of the native action loop (parallel/native.py)
        # native multi-step loop (ops.abi ModelLib.iterate) for halo-free lattices
        self.native_loop = (os.environ.get("TCLB_NATIVE_LOOP", "1") != "0") if native_loop is None else native_loop
        for s in m.settings:
            self.set_setting(s.name, s.default, _init=True)
        # GPU block -> tile windows (executor_hip.hpp tile_id): log2 of the number of
        # contiguous tile ranges the work-groups are dealt over; env TCLB_TILE_SPLIT
        self.tile_split = self._default_tile_split()
        self._L = self._base_launch()
        self.callbacks = []
        self.samplers = []        # tclb_amd.sampler.Sampler: probes recorded every iteration
        self.turb_t = None
        self.turb_time_wn = 0.0
        self.cuts = None
        self.particles = None     # ParticleSystem with pre_stage/post_stage/step hooks
        self.average_start = 0
        # the native loop of a multi-rank lattice is created with the lattice, so its
        # collective set-up (the RCCL communicator) happens at the same point on every rank
        if (self.comm.distributed and self.native_loop and native_dist_enabled() and self.lib.has_iterate
                and NativeLoop.supported(self)):
            self._dist = NativeLoop(self)

    def _default_tile_split(self) -> int:
        """4 windows (k = 2) for 3-D single-stage models of up to 32 fields (d3q27 fp64
        512^3 +2-4 %, d3q27_cumulant / d3q19 256^3 +2-10 %); the linear order elsewhere
        (multi-stage, LDS-tile and CHT models measured equal or slower, profiles/README.md
        r05e)"""
        env = os.environ.get("TCLB_TILE_SPLIT")
        if env is not None and env != "":
            return max(0, min(15, int(env)))
        m = self.model
        act = m.action("Iteration")
        if self.is_gpu and m.dims == 3 and act is not None and len(act.stages) == 1 and len(m.fields) <= 32:
            return 2
        return 0

    def set_tile_split(self, k: int):
        """log2 of the tile windows of the GPU kernels (0: linear block order)"""
        self.tile_split = max(0, min(15, int(k)))
        self._L.tile_split = self.tile_split

    def _alloc_snapshots(self) -> List[torch.Tensor]:
        """the A/B pair.  On a GPU, for large snapshots, placement-aware: where a 29 GB
        snapshot lands in HBM moves the streaming speed of the kernel that writes (or reads)
        it by up to ~20 % (tools/direction_probe.py, tools/placement_probe.py: the same
        d3q27 fp64 512^3 collide ran 9.5-11.8 ms per dispatch from one allocation to the
        next), so K candidates (TCLB_PLACE_CANDIDATES, default 4, as many as fit) are
        allocated at once, each timed by a streaming read and write of its field planes
        (ops.device.snap_probe_ms), and the two fastest kept.  TCLB_PLACE=0: no probing;
        TCLB_PLACE_MIN_GB: smallest snapshot probed (default 2)."""
        if not self.is_gpu or os.environ.get("TCLB_PLACE", "1") == "0":
            return [self.new_snapshot() for _ in range(2)]
        es = torch.tensor([], dtype=self.sdtype).element_size()
        nbytes = self.nf * self.fs * es
        if nbytes < float(os.environ.get("TCLB_PLACE_MIN_GB", "2")) * 2 ** 30:
            return [self.new_snapshot() for _ in range(2)]
        free, _ = torch.cuda.mem_get_info(self.device)
        k = min(int(os.environ.get("TCLB_PLACE_CANDIDATES", "4")), int(0.9 * free // nbytes))
        if k < 3:
            return [self.new_snapshot() for _ in range(2)]
        from .ops.device import snap_probe_ms
        cands = [self.new_snapshot() for _ in range(k)]
        times = [snap_probe_ms(c, self.nf, self.fs) for c in cands]
        order = sorted(range(k), key=lambda i: times[i][0] + times[i][1])
        keep = sorted(order[:2])
        self.placement = {"candidates": k, "read_write_ms": [[round(r, 4), round(w, 4)] for r, w in times],
                          "kept": keep}
        snaps = [cands[i] for i in keep]
        del cands
        torch.cuda.empty_cache()
        return snaps

    def new_snapshot(self, uninit: bool = False) -> torch.Tensor:
        """a zeroed snapshot buffer with the layout of snaps[0/1] ([nf][NZ][NY][px], field
        stride fs): the A/B pair, and states kept by the adjoint's checkpointing.
        uninit: no zero fill, for a buffer the next step overwrites in full (every field
        of every interior node); padding columns and ghost planes are then undefined"""
        alloc = torch.empty if uninit else torch.zeros
        return (alloc(self.nf * self.fs, dtype=self.sdtype, device=self.device)
                .as_strided((self.nf, self.NZ, self.NY, self.px), (self.fs, self.NY * self.px, self.px, 1)))

    def writes_all_fields(self, action: str = "Iteration") -> bool:
        """every field is saved by some stage of `action` (its output snapshot holds no
        value from before the step)"""
        m = self.model
        saved = set()
        for sname in m.action(action).stages:
            saved.update(self._saved_fields(m.stage(sname)))
        return len(saved) == self.nf

    # ------------------------------------------------------------------ launch
    def _base_launch(self) -> abi.Launch:
        L = abi.Launch()
        nx, ny, nz = self.shape
        L.sy = self.px
        L.sz = self.px * self.NY
        L.fs = self.fs
        L.nx, L.ny, L.nz, L.px = nx, ny, nz, self.px
        L.gy, L.gz = self.gy, self.gz
        ox, oy, oz = self.slab.offset
        L.x0, L.y0, L.z0 = ox, oy, oz
        L.gnx, L.gny, L.gnz = self.gshape
        L.xlo, L.xhi, L.ylo, L.yhi, L.zlo, L.zhi = 0, nx, 0, ny, 0, nz
        L.block_x, L.block_y = self.block
        L.flags = self.flags.data_ptr()
        L.flags_gen = self.flags_version
        L.storage_shift = 1 if self.storage_shift else 0
        L.tile_split = self.tile_split
        return L

    def _sync_settings(self):
        if self._settings_dirty:
            self.settings_t = torch.as_tensor(self.svals, dtype=torch.float64).to(self.device)
            z = np.concatenate([self.zvals.reshape(-1), self.zdt.reshape(-1)])
            self.zonal_t = torch.as_tensor(z, dtype=torch.float64).to(self.device)
            self._settings_dirty = False
            # no objective weight anywhere: the kernels skip the weighted Objective sum
            obj = [i for i, n in enumerate(self.zsettings) if n.endswith("InObj")]
            self._glob_flags = 4 if not np.any(self.zvals[obj]) else 0     # TCLB_GLOB_NOOBJ
        L = self._L
        L.settings = self.settings_t.data_ptr()
        L.zonal = self.zonal_t.data_ptr()
        L.nzones = self.zvals.shape[1]
        L.globals_ = self.globals_t.data_ptr()
        L.flags = self.flags.data_ptr()
        L.flags_gen = self.flags_version
        if self.turb_t is not None:
            L.ext[0] = self.turb_t.data_ptr()
            L.next[0] = self.turb_t.shape[0]
            L.time_shift = self.turb_time_wn
        if self.cuts is not None:
            L.ext[1] = self.cuts.data_ptr()
            L.next[1] = self.cuts.numel()

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream if self.is_gpu else 0

    def _launch_stage(self, stage: int, src: torch.Tensor, dst: torch.Tensor, glob: bool,
                      axis_range: Optional[Tuple[int, int]] = None,
                      box: Optional[Tuple[int, int, int, int]] = None):
        L = self._L
        L.in_ = src.data_ptr()
        L.out = dst.data_ptr()
        L.stage = stage
        L.glob = (1 | self._glob_flags) if glob else 0
        L.iter = self.iter
        L.reserved1 = self.iter - self.average_start + 1
        L.stream = self._stream()
        nx, ny, nz = self.shape
        L.ylo, L.yhi, L.zlo, L.zhi = 0, ny, 0, nz
        if axis_range is not None:
            if self.slab.axis == 2:
                L.zlo, L.zhi = axis_range
            else:
                L.ylo, L.yhi = axis_range
        if box is not None:               # (ylo, yhi, zlo, zhi) of the Y x Z grid split
            L.ylo, L.yhi, L.zlo, L.zhi = box
        self.lib.run(L, self.prec)
        if trace.SYNC:
            trace.after_launch(self, f"{self.model.name} stage {stage}")

    # ------------------------------------------------------------------ halos
    def _axis_planes(self, buf: torch.Tensor, a: int, b: int, axis: Optional[int] = None) -> torch.Tensor:
        """view of planes [a, b) in ghost-inclusive coordinates along a split axis
        (default: the slab axis; 1 = y rows, 2 = z planes)"""
        axis = self.slab.axis if axis is None else axis
        return buf[:, a:b] if axis == 2 else buf[:, :, a:b]

    def _field_index_t(self, fields: List[int]) -> torch.Tensor:
        key = tuple(fields)
        t = self._halo_bufs.get(key)
        if t is None:
            t = self._halo_bufs[key] = torch.tensor(fields, dtype=torch.long, device=self.device)
        return t

    def _pack(self, buf: torch.Tensor, fields: List[int], a: int, b: int, axis: Optional[int] = None) -> torch.Tensor:
        """the halo planes of `fields` as one contiguous message: one strided copy for a
        contiguous run of fields, else one gather kernel (index_select)"""
        planes = self._axis_planes(buf, a, b, axis)
        runs = _runs(fields)
        if len(runs) == 1:
            return planes[runs[0][0]:runs[0][1]].contiguous()
        return planes.index_select(0, self._field_index_t(fields))

    def _unpack(self, buf: torch.Tensor, fields: List[int], a: int, b: int, data: torch.Tensor,
                axis: Optional[int] = None):
        planes = self._axis_planes(buf, a, b, axis)
        runs = _runs(fields)
        if len(runs) == 1:
            planes[runs[0][0]:runs[0][1]].copy_(data)
        else:
            planes.index_copy_(0, self._field_index_t(fields), data)      # one scatter kernel

    def _halo_start(self, buf: torch.Tensor, fields: Optional[Sequence[int]] = None):
        if self.g == 0:
            return None
        if self.slab.axis == 3:
            # Y x Z grid: z planes first, then y rows over the whole z extent (ghosts
            # included), which also fills the edge ghosts; no overlap split
            for a in (2, 1):
                self._halo_finish(self._halo_axis_start(buf, fields, a))
            return None
        return self._halo_axis_start(buf, fields, self.slab.axis)

    def _halo_axis_start(self, buf: torch.Tensor, fields: Optional[Sequence[int]], axis: int):
        g = self.gz if axis == 2 else self.gy
        n = self.shape[2] if axis == 2 else self.shape[1]
        lo_set, hi_set = self.halo_sets[axis]
        lo = [i for i in lo_set if fields is None or i in fields]
        hi = [i for i in hi_set if fields is None or i in fields]
        if not self.comm.distributed:
            # loopback: periodic wrap = plane copies inside this snapshot
            for r0, r1 in _runs(lo):
                self._axis_planes(buf, 0, g, axis)[r0:r1].copy_(self._axis_planes(buf, n, n + g, axis)[r0:r1])
            for r0, r1 in _runs(hi):
                self._axis_planes(buf, n + g, n + 2 * g, axis)[r0:r1].copy_(self._axis_planes(buf, g, 2 * g, axis)[r0:r1])
            return None
        if trace.ENABLED:
            trace.push("halo")
        send_up = self._pack(buf, lo, n, n + g, axis) if lo else None        # my top planes -> next's lower ghost
        send_down = self._pack(buf, hi, g, 2 * g, axis) if hi else None      # my bottom planes -> prev's upper ghost
        recv_below = torch.empty_like(send_up) if lo else None
        recv_above = torch.empty_like(send_down) if hi else None
        nbr = self.slab.neighbours(axis) if self.slab.axis == 3 else None
        h = self.comm.start_halo(send_up, send_down, recv_below, recv_above, nbr=nbr)
        return (h, buf, lo, hi, recv_below, recv_above, send_up, send_down, axis)

    def _halo_finish(self, st):
        if st is None:
            return
        h, buf, lo, hi, rb, ra, su, sd, axis = st
        self.comm.wait_halo(h)
        g = self.gz if axis == 2 else self.gy
        n = self.shape[2] if axis == 2 else self.shape[1]
        if lo:
            self._unpack(buf, lo, 0, g, rb, axis)
        if hi:
            self._unpack(buf, hi, n + g, n + 2 * g, ra, axis)
        if trace.ENABLED:
            trace.pop()

    def _mirror_buffer(self, fields: List[int], axis: int, side: str) -> torch.Tensor:
        """persistent packed halo buffer [len(fields)][g planes] of one side, laid out as
        _pack's output (zeroed once, so the x pitch padding stays finite).  The side is
        part of the key: with a symmetric stencil the lo and hi field lists are equal,
        and one shared buffer would carry the top planes in both directions."""
        key = ("mirror", axis, side, tuple(fields))
        t = self._halo_bufs.get(key)
        if t is None:
            g = self.gz if axis == 2 else self.gy
            shape = (len(fields), g, self.NY, self.px) if axis == 2 else (len(fields), self.NZ, g, self.px)
            t = self._halo_bufs[key] = torch.zeros(shape, dtype=self.sdtype, device=self.device)
        return t

    def _launch_mirrored(self, stage: int, src, dst, glob: bool, rng: Tuple[int, int], fields: List[int],
                         target: torch.Tensor, axis: int):
        """launch over border planes rng whose stores of `fields` also land in the packed
        buffer `target` (Launch.mbase, core.hpp mirror_store): the border kernel packs the
        outgoing halo itself"""
        L = self._L
        key = ("slots", tuple(fields))
        table = self._halo_bufs.get(key)
        if table is None:
            vals = [-1] * abi.MIRROR_FIELDS
            for k, f in enumerate(fields):
                vals[f] = k
            table = self._halo_bufs[key] = (ctypes.c_byte * abi.MIRROR_FIELDS)(*vals)
        L.mslot = table
        L.mbase = target.data_ptr()
        L.mfs = target.stride(0)
        if axis == 2:
            L.msy, L.msz, L.moy, L.moz = self.px, self.NY * self.px, self.gy, -rng[0]
        else:
            L.msy, L.msz, L.moy, L.moz = self.px, target.shape[2] * self.px, -rng[0], self.gz
        try:
            self._launch_stage(stage, src, dst, glob, rng)
        finally:
            L.mbase = None

    def _border_mirrored(self, stage: int, src, dst, glob: bool, fields: List[int]):
        """overlapped slab step, border part: the two border launches write their halo
        planes straight into the send buffers (no pack kernels), then the exchange starts.
        Reference: RunBorder + MPIStream_A (src/Lattice.cu.Rt:466-533), which packs the
        margin blocks on the device in separate copy kernels."""
        axis = self.slab.axis
        g = self.gz if axis == 2 else self.gy
        n = self.shape[2] if axis == 2 else self.shape[1]
        lo_set, hi_set = self.halo_sets[axis]
        fs = set(fields)
        lo = [i for i in lo_set if i in fs]        # read from below: my top planes go up
        hi = [i for i in hi_set if i in fs]        # read from above: my bottom planes go down
        send_down = self._mirror_buffer(hi, axis, "down") if hi else None
        send_up = self._mirror_buffer(lo, axis, "up") if lo else None
        if hi:
            self._launch_mirrored(stage, src, dst, glob, (0, g), hi, send_down, axis)
        else:
            self._launch_stage(stage, src, dst, glob, (0, g))
        if lo:
            self._launch_mirrored(stage, src, dst, glob, (n - g, n), lo, send_up, axis)
        else:
            self._launch_stage(stage, src, dst, glob, (n - g, n))
        if trace.ENABLED:
            trace.push("halo")
        if isinstance(self.comm, LoopbackComm):
            # this rank is its own neighbour: the send buffers are the received halos
            return (None, dst, lo, hi, send_up, send_down, send_up, send_down, axis)
        recv_below = torch.empty_like(send_up) if lo else None
        recv_above = torch.empty_like(send_down) if hi else None
        h = self.comm.start_halo(send_up, send_down, recv_below, recv_above)
        return (h, dst, lo, hi, recv_below, recv_above, send_up, send_down, axis)

    def _grid_overlapped(self, stage: int, src, dst, glob: bool, fields: List[int]):
        """overlapped step of the Y x Z process grid: the four border slabs (z planes over
        all y, then y rows over the inner z), then the two-phase halo (z planes, then y
        rows over the ghost-inclusive z extent, which fills the edge ghosts) on a side
        stream while the interior kernel runs.  Reference: RunBorder -> MPIStream_A ->
        RunInterior -> MPIStream_B (src/Lattice.cu.Rt:466-533) over MPIDivision's grid."""
        nx, ny, nz = self.shape
        gy, gz = self.gy, self.gz
        for box in ((0, ny, 0, gz), (0, ny, nz - gz, nz), (0, gy, gz, nz - gz), (ny - gy, ny, gz, nz - gz)):
            self._launch_stage(stage, src, dst, glob, box=box)
        if trace.ENABLED:
            trace.push("halo")
        done = None
        if self.is_gpu:
            # the halo packs/unpacks go on a side stream ordered after the border kernels,
            # so the y phase (which waits for the z phase) never queues behind the interior
            cur = torch.cuda.current_stream(self.device)
            if self._halo_stream is None:
                self._halo_stream = torch.cuda.Stream(self.device)
            hs = self._halo_stream
            hs.wait_stream(cur)
            with torch.cuda.stream(hs):
                for a in (2, 1):
                    self._halo_finish(self._halo_axis_start(dst, fields, a))
            done = torch.cuda.Event()
            done.record(hs)
        else:
            hz = self._halo_axis_start(dst, fields, 2)
        self._launch_stage(stage, src, dst, glob, box=(gy, ny - gy, gz, nz - gz))
        if self.is_gpu:
            torch.cuda.current_stream(self.device).wait_event(done)
        else:
            self._halo_finish(hz)
            self._halo_finish(self._halo_axis_start(dst, fields, 1))
        if trace.ENABLED:
            trace.pop()

    def reverse_halo(self, a: torch.Tensor):
        """adjoint of the halo exchange: contributions accumulated in the ghost planes of
        an adjoint snapshot `a` are added to the planes of their owner (the neighbour
        rank, or the periodic image on one rank) and the ghosts are cleared.  Phases in
        the reverse order of the forward exchange (Y x Z grid: y rows over the
        ghost-inclusive z extent, then z planes), so edge ghosts reach the diagonal
        owner.  Reference: Iteration_Adj's reversed margin exchange and the atomic
        adjoint push into the margins (src/Lattice.cu.Rt:542-613,
        src/LatticeAccess.inc.cpp.Rt:349-361)."""
        if self.g == 0:
            return
        axes = (1, 2) if self.slab.axis == 3 else (self.slab.axis,)
        for axis in axes:
            g = self.gz if axis == 2 else self.gy
            n = self.shape[2] if axis == 2 else self.shape[1]
            if g == 0:
                continue
            lo_ghost = self._axis_planes(a, 0, g, axis)              # owner: prev rank, its top planes
            hi_ghost = self._axis_planes(a, n + g, n + 2 * g, axis)  # owner: next rank, its bottom planes
            top = self._axis_planes(a, n, n + g, axis)
            bottom = self._axis_planes(a, g, 2 * g, axis)
            if not self.comm.distributed:
                top += lo_ghost
                bottom += hi_ghost
            else:
                send_up = hi_ghost.contiguous()
                send_down = lo_ghost.contiguous()
                recv_below = torch.empty_like(send_up)
                recv_above = torch.empty_like(send_down)
                nbr = self.slab.neighbours(axis) if self.slab.axis == 3 else None
                h = self.comm.start_halo(send_up, send_down, recv_below, recv_above, nbr=nbr)
                self.comm.wait_halo(h)
                bottom += recv_below
                top += recv_above
            lo_ghost.zero_()
            hi_ghost.zero_()

    def exchange(self, buf: Optional[torch.Tensor] = None, fields=None):
        buf = self.snaps[self.cur] if buf is None else buf
        if self._dist is not None and self._dist.gpu and self._dist.transport == "ipc":
            # the IPC ranks' halos only travel through the native loop's transport
            self._dist.exchange_fields(buf, fields)
            return
        self._halo_finish(self._halo_start(buf, fields))

    # ------------------------------------------------------------------ actions
    def _saved_fields(self, stage) -> List[int]:
        # cached per stage: the per-step paths (halo, particles, adjoint) ask every launch
        cache = self.__dict__.setdefault("_saved_cache", {})
        key = (stage.name, tuple(stage.save_fields) if stage.save_fields is not None else None)
        r = cache.get(key)
        if r is None:
            r = cache[key] = [i for i, f in enumerate(self.model.fields) if self.model.matches(f, stage.save_fields)]
        return r

    def run_action(self, name: str, glob: bool = False, reduce: bool = True):
        """one action; with glob the globals are integrated and (reduce) all-reduced and
        copied to the host (reduce=False leaves them on the device: globals_vector())"""
        m = self.model
        act = m.action(name)
        if act is None:
            raise KeyError(f"model {m.name} has no action {name}")
        if not self._iterating:
            self._mirror_kept(name)
        self._sync_settings()
        src = self.snaps[self.cur]
        dst = self.snaps[1 - self.cur]
        if glob:
            self.globals_t.zero_()
        n = self.shape[2] if self.slab.axis == 2 else self.shape[1]
        g = self.g
        if trace.ENABLED:
            trace.push(f"action {name}")
        for k, sname in enumerate(act.stages):
            if trace.ENABLED:
                trace.push(f"stage {sname}")
            si = m.stage_index(sname)
            st = m.stage(sname)
            inp = src if k == 0 else dst
            fields = self._saved_fields(st)
            if st.particle and self.particles is not None:
                self.particles.pre_stage(self)
            if st.snapshot_reads and k > 0 and not st.fixed_point:
                # a stage that reads (through a stencil) a field it also writes: run it
                # out of place so every node sees the pre-stage values (the reference runs
                # it in place, an order-dependent race; tools/race_check.py finds these)
                scratch = self._scratch_snapshot()
                self._launch_stage(si, dst, scratch, glob)
                for r0, r1 in _runs(fields):
                    dst[r0:r1].copy_(scratch[r0:r1])
                self._halo_finish(self._halo_start(dst, fields))
            elif st.fixed_point and k > 0:
                # fixed-point stage (reference AddStage(fixedPoint=TRUE): 100 sweeps,
                # src/Lattice.cu.Rt:484).  The reference sweeps in place (input == output
                # snapshot, an order-dependent Gauss-Seidel on the GPU); here every sweep
                # reads the current snapshot and writes a scratch one whose saved fields
                # are copied back: a deterministic Jacobi iteration.
                scratch = self._scratch_snapshot()
                for _ in range(FIXED_POINT_SWEEPS):
                    self._launch_stage(si, dst, scratch, glob)
                    for r0, r1 in _runs(fields):
                        dst[r0:r1].copy_(scratch[r0:r1])
                    self._halo_finish(self._halo_start(dst, fields))
            elif self.overlap and self.slab.axis == 3:
                if self.shape[1] > 2 * self.gy and self.shape[2] > 2 * self.gz:
                    self._grid_overlapped(si, inp, dst, glob, fields)
                else:
                    self._launch_stage(si, inp, dst, glob)
                    self._halo_finish(self._halo_start(dst, fields))
            elif self.overlap and n > 2 * g:
                # a split stage's class-0 nodes store nothing, not even into the mirror
                if self.halo_mirror and not st.split:
                    hs = self._border_mirrored(si, inp, dst, glob, fields)
                else:
                    self._launch_stage(si, inp, dst, glob, (0, g))
                    self._launch_stage(si, inp, dst, glob, (n - g, n))
                    hs = self._halo_start(dst, fields)
                self._launch_stage(si, inp, dst, glob, (g, n - g))
                self._halo_finish(hs)
            else:
                self._launch_stage(si, inp, dst, glob)
                self._halo_finish(self._halo_start(dst, fields))
            if st.particle and self.particles is not None:
                self.particles.post_stage(self)
                if name != "Init":
                    self.particles.step(self)
            if trace.ENABLED:
                trace.pop()
        self.cur = 1 - self.cur
        if glob and reduce:
            self._reduce_globals()
        if trace.ENABLED:
            trace.pop()

    def _scratch_snapshot(self) -> torch.Tensor:
        if getattr(self, "_scratch", None) is None:
            self._scratch = torch.zeros(self.nf * self.fs, dtype=self.sdtype, device=self.device).as_strided(
                self.snaps[0].shape, self.snaps[0].stride())
        return self._scratch

    def globals_vector(self) -> torch.Tensor:
        """the NG globals of this rank: SUM globals summed and MAX globals max-reduced
        over the accumulator slots"""
        ng, ns = len(self.model.globals_), self.model.n_sum_globals
        slots = self.globals_t.view(abi.GSLOTS, self._gstride)[:, :ng]
        if ns == ng:
            return slots.sum(0)
        return torch.cat([slots[:, :ns].sum(0), slots[:, ns:].amax(0)])

    def _reduce_globals(self):
        with trace.span("globals"):
            g = self.comm.allreduce_globals(self.globals_vector(), self.model.n_sum_globals)
        vals = g.detach().cpu().numpy()
        for i, gl in enumerate(self.model.globals_):
            self.globals[gl.name] = float(vals[i])

    def init(self):
        """Action Init (reference: Lattice::Init -> Action_Init, src/Lattice.cu.Rt:799-821):
        through the native action loop when it takes the action (e.g. d2q9_csf's
        fixed-point wall-normal stage), else the Python step path."""
        self.iter = 0
        if self._native_path("Init") == "loop":
            self.iterate(1, glob_last=False, action="Init")
            self.iter = 0
        else:
            self.run_action("Init", glob=False)

    def _native_path(self, action: str) -> Optional[str]:
        """how `action` steps: "lib" — one call into the model library (one rank, no
        ghosts, plain stages: tclb::iterate_action); "loop" — the native action loop
        (parallel/native.py, tclb_rt/dist_loop.hpp: any rank count, slab or Y x Z grid,
        particle / out-of-place / fixed-point stages, time series, samplers); None — the
        Python step path (per-step callbacks, a particle system that talks to another
        program, TCLB_NATIVE_LOOP=0)"""
        if not (self.native_loop and self.lib.has_iterate):
            return None
        act = self.model.action(action)
        if act is None or self.callbacks:
            return None
        if self.particles is not None and not self.particles.native_ok():
            return None
        if self.comm.distributed and not native_dist_enabled():
            return None
        if not NativeLoop.supported(self):
            return None
        special = any(self.model.stage(s).fixed_point or self.model.stage(s).particle or
                      self.model.stage(s).snapshot_reads for s in act.stages)
        if (self.g == 0 and not self.comm.distributed and not self.zseries and self.particles is None
                and len(self.samplers) <= 1 and not special):
            return "lib"
        return "loop"

    def _native_ok(self, action: str) -> bool:
        return self._native_path(action) is not None

    def iterate(self, n: int, glob_last: bool = True, action: str = "Iteration", reduce: bool = True):
        """Reference Lattice::Iterate (src/Lattice.cu.Rt:900-989): globals on the last step.

        The n steps run in one native call whenever nothing needs Python between steps:
        on one rank without ghosts and with plain stages tclb::iterate_action of the model
        library (one kernel launch per stage); otherwise the native action loop of
        parallel/native.py (border launches, RCCL exchange into the ghost planes, interior
        launch; particle hooks, out-of-place and fixed-point stages, time series,
        samplers)."""
        if n <= 0:
            return
        self._mirror_kept(action)
        path = self._native_path(action)
        if path is not None:
            m = self.model
            stages = [m.stage_index(s) for s in m.action(action).stages]
            self._sync_settings()
            if self.zseries and any(self.zsettings[k[0]].endswith("InObj") for k in self.zseries):
                # an Objective weight follows a series: keep the weighted sum on
                self._glob_flags &= ~4
            if glob_last:
                self.globals_t.zero_()
            L = self._L
            nx, ny, nz = self.shape
            L.xlo, L.xhi, L.ylo, L.yhi, L.zlo, L.zhi = 0, nx, 0, ny, 0, nz
            L.in_ = self.snaps[self.cur].data_ptr()
            L.out = self.snaps[1 - self.cur].data_ptr()
            L.iter = self.iter
            L.reserved1 = self.iter - self.average_start + 1
            L.stream = self._stream()
            L.glob = self._glob_flags            # bit 0 set per step by the loop
            with trace.span(f"iterate {action} x{n}"):
                if path == "lib":
                    smp = self.samplers[0] if self.samplers else None
                    self.lib.iterate(L, self.prec, n, stages, glob_last, smp.plan_for(n) if smp else None)
                else:
                    if self._dist is None:
                        self._dist = NativeLoop(self)
                    self._dist.iterate(L, n, action, glob_last)
            if trace.SYNC:
                trace.after_launch(self, f"{self.model.name} native loop")
            if action != "Init":
                for smp in self.samplers:
                    smp.advance(n)
            if self.particles is not None:
                self.particles.after_native(self, n, action)
            self.iter += n
            if n % 2 == 1:
                self.cur = 1 - self.cur
            if self.zseries:
                # the host copy of the zonal table follows the device: entries of the last step
                self.iter -= 1
                self.apply_series()
                self.iter += 1
            if glob_last and reduce:
                if self._dist is not None:
                    self._dist.wait()
                self._reduce_globals()
            return
        self._iterating = True
        try:
            for i in range(n):
                glob = glob_last and i == n - 1
                if self.zseries:
                    self.apply_series()
                self.run_action(action, glob=glob, reduce=reduce)
                self.iter += 1
                for smp in self.samplers:
                    smp.sample_now()
                for cb in self.callbacks:
                    cb(self)
        finally:
            self._iterating = False

    def _kept_fields(self, action: str) -> List[int]:
        """indices of the fields that a stage of `action` keeps (DSL add_stage(keep=...)):
        unchanged by it and not stored, so both snapshots must hold them"""
        c = self._kept_cache.get(action)
        if c is None:
            m = self.model
            act = m.action(action)
            tags = [t for s in (act.stages if act else []) for t in (m.stage(s).keep or [])]
            c = [i for i, f in enumerate(m.fields) if tags and m.matches(f, tags)]
            self._kept_cache[action] = c
        return c

    def _mirror_kept(self, action: str):
        """copy the kept fields of `action` (whole planes, ghosts included) from the current
        snapshot into the other one: whatever wrote them last (an initialisation stage, a
        field load, a checkpoint restore) wrote one snapshot; the action's steps alternate
        between the two and never store them.  A device copy of a few fields per iterate
        call, against a read and a write of each of them per node and step."""
        idx = self._kept_fields(action)
        if not idx:
            return
        src, dst = self.snaps[self.cur], self.snaps[1 - self.cur]
        m = self.model
        sf = m.setting_fields
        fill = {}
        for i in idx:
            f = m.fields[i]
            key = f.nicename if f.nicename in sf else (f.name if f.name in sf else None)
            if key is not None:
                v = sf[key]
                fill[i] = float(self.svals[self.gsettings.index(v)]) if isinstance(v, str) else float(v)
        # setting-derived fields: filled on both snapshots (ghosts included) when their
        # values or the fields changed since the last fill — what the reference's Run
        # stores on every node in every step
        state = (tuple(sorted(fill.items())), self._fields_gen, self.snaps[0].data_ptr(), self.snaps[1].data_ptr())
        for i in idx:
            if i in fill:
                if state != self._fill_state:
                    sh = float(self._shift_t[i].reshape(-1)[0]) if self._shift_t is not None else 0.0
                    src[i].fill_(fill[i] - sh)
                    dst[i].fill_(fill[i] - sh)
            else:
                dst[i].copy_(src[i])
        self._fill_state = state

    # ------------------------------------------------------------------ settings
    def set_setting(self, name: str, value: float, zone: Optional[str] = None, _init: bool = False):
        m = self.model
        s = m.setting(name)
        if s is None:
            raise KeyError(f"model {m.name} has no setting {name}")
        value = float(value)
        if s.zonal:
            zi = self.zsettings.index(name)
            if zone is None:
                self.zvals[zi, :] = value
            else:
                self.zvals[zi, self.zone_index(zone)] = value
        else:
            self.svals[self.gsettings.index(name)] = value
        self._settings_dirty = True
        if s.derived:
            env = self.settings_dict(zone)
            env[name] = value
            for tgt, expr in s.derived.items():
                self.set_setting(tgt, eval_expr(expr, env), zone=zone)

    def set_setting_dt(self, name: str, value: float, zone: Optional[str] = None):
        """time derivative of a zonal setting (read by the dynamics as <name>_DT())"""
        zi = self.zsettings.index(name)
        if zone is None:
            self.zdt[zi, :] = float(value)
        else:
            self.zdt[zi, self.zone_index(zone)] = float(value)
        self._settings_dirty = True

    def set_zone_series(self, name: str, values, zone: Optional[str] = None):
        """time-dependent zonal setting: values[k] is active in iterations with
        iter % len(values) == k (reference ZoneSettings, ZoneIndex = Iter % len,
        src/Lattice.cu.Rt:473-477); the time derivative <name>_DT follows the series"""
        zi = self.zsettings.index(name)
        z = self.zone_index(zone or "DefaultZone")
        self.zseries[(zi, z)] = np.asarray(values, dtype=np.float64).copy()
        self.apply_series()

    def zone_series(self, name: str, zone: Optional[str] = None) -> Optional[np.ndarray]:
        zi = self.zsettings.index(name)
        return self.zseries.get((zi, self.zone_index(zone or "DefaultZone")))

    def series_index(self, key) -> int:
        return self.iter % len(self.zseries[key])

    def apply_series(self):
        """load the active entries of all zonal time series (and their slopes)"""
        for key, v in self.zseries.items():
            n = len(v)
            k = self.iter % n
            self.zvals[key] = v[k]
            if n > 1:
                lo, hi = max(k - 1, 0), min(k + 1, n - 1)
                self.zdt[key] = (v[hi] - v[lo]) / max(hi - lo, 1)
        self._settings_dirty = True

    def get_setting(self, name: str, zone: Optional[str] = None) -> float:
        s = self.model.setting(name)
        if s is None:
            raise KeyError(name)
        if s.zonal:
            return float(self.zvals[self.zsettings.index(name), self.zone_index(zone or "DefaultZone")])
        return float(self.svals[self.gsettings.index(name)])

    def settings_dict(self, zone: Optional[str] = None) -> Dict[str, float]:
        d = {n: float(self.svals[i]) for i, n in enumerate(self.gsettings)}
        zi = self.zone_index(zone) if zone is not None and zone in self.zone_names else 0
        for i, n in enumerate(self.zsettings):
            d[n] = float(self.zvals[i, zi])
        return d

    def zone_index(self, zone: str) -> int:
        if zone not in self.zone_names:
            self.add_zone(zone)
        return self.zone_names[zone]

    def add_zone(self, zone: str) -> int:
        if zone in self.zone_names:
            return self.zone_names[zone]
        zi = len(self.zone_names)
        if zi > self.model.zone_max:
            raise ValueError(f"too many zones for model {self.model.name} (max {self.model.zone_max})")
        self.zone_names[zone] = zi
        col = self.zvals[:, :1]
        self.zvals = np.concatenate([self.zvals, col], axis=1)
        self.zdt = np.concatenate([self.zdt, np.zeros_like(col)], axis=1)
        self._settings_dirty = True
        return zi

    # ------------------------------------------------------------------ flags
    def set_flags(self, flags: np.ndarray):
        """flags: (NZ, NY, nx) incl. ghost planes along the decomposed axis"""
        nx = self.shape[0]
        full = np.zeros((self.NZ, self.NY, self.px), dtype=np.uint16 if self.model.flag_bits == 16 else np.uint32)
        full[:, :, :nx] = flags
        view = full.view(np.int16 if self.model.flag_bits == 16 else np.int32)
        self.flags.copy_(torch.from_numpy(view))
        self.flags_changed()

    def flags_changed(self):
        """to be called after any write into self.flags"""
        self.flags_version = next(_FLAGS_GEN)

    def get_flags(self) -> np.ndarray:
        """interior flags (nz, ny, nx) as unsigned"""
        f = self.flags.cpu().numpy()
        f = f.view(np.uint16 if self.model.flag_bits == 16 else np.uint32)
        return self._interior(f)

    def _interior(self, a):
        nx, ny, nz = self.shape
        return a[self.gz:self.gz + nz, self.gy:self.gy + ny, :nx]

    def set_cuts(self, cuts: np.ndarray):
        """sub-voxel cuts (26, NZ, NY, nx) uint16 for interpolated bounce-back models"""
        nx = self.shape[0]
        full = np.full((26, self.NZ, self.NY, self.px), 65535, dtype=np.uint16)
        full[:, :, :, :nx] = cuts
        self.cuts = torch.from_numpy(full.view(np.int16)).to(self.device)

    def set_turbulence(self, modes: np.ndarray, time_wn: float = 0.0):
        """synthetic-turbulence modes (n, 7) -> device (Launch.ext[0]); the time wave number
        of time-correlated inflow turbulence travels in Launch.time_shift"""
        self.turb_t = torch.as_tensor(np.ascontiguousarray(modes, dtype=np.float64)).to(self.device)
        self.turb_time_wn = float(time_wn)

    def reset_average(self):
        """reset averaged fields (reference cbAveraging -> resetAverage, src/Lattice.cu.Rt:1360-1365)"""
        idx = [i for i, f in enumerate(self.model.fields) if f.average]
        for i in idx:
            self.snaps[self.cur][i].zero_()
        self.average_start = self.iter

    # ------------------------------------------------------------------ fields / quantities
    def field(self, name: str) -> torch.Tensor:
        """interior view of a stored field in the current snapshot: (nz, ny, nx)"""
        i = self.model.field_index(name)
        nx, ny, nz = self.shape
        v = self.snaps[self.cur][i, self.gz:self.gz + nz, self.gy:self.gy + ny, :nx]
        if self._shift_t is not None:        # shifted storage: a copy of the true values
            return v.to(self.rdtype) + self._shift_t[i, 0].to(self.rdtype)
        return v

    def fields_interior(self, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """all fields on the interior (nf, nz, ny, nx): a view of the storage, or for the
        *-shift precisions a copy with the storage shift added back in `dtype` (default
        the compute dtype; checkpoints ask for fp64 so that f - w round-trips exactly)"""
        nx, ny, nz = self.shape
        v = self.snaps[self.cur][:, self.gz:self.gz + nz, self.gy:self.gy + ny, :nx]
        if self._shift_t is not None:
            dt = dtype or self.rdtype
            return v.to(dt) + self._shift_t.to(dt)
        return v if dtype is None else v.to(dtype)

    def set_fields_interior(self, data: torch.Tensor):
        nx, ny, nz = self.shape
        if self._shift_t is not None:
            data = data.to(torch.float64) - self._shift_t
        self.snaps[self.cur][:, self.gz:self.gz + nz, self.gy:self.gy + ny, :nx].copy_(data)
        self._fields_gen += 1
        self.exchange()

    def quantity(self, name: str, scale: float = 1.0) -> torch.Tensor:
        """compute a quantity over the local interior: returns (ncomp, nz, ny, nx)"""
        m = self.model
        qi = next((i for i, q in enumerate(m.quantities) if q.name == name), None)
        if qi is None:
            raise KeyError(f"model {m.name} has no quantity {name}")
        q = m.quantities[qi]
        nc = 3 if q.vector else 1
        nx, ny, nz = self.shape
        if q.adjoint:
            return self._adjoint_quantity(q, nc) * scale
        out = torch.empty((nc, nz, ny, nx), dtype=self.rdtype, device=self.device)
        self._sync_settings()
        L = self._L
        L.in_ = self.snaps[self.cur].data_ptr()
        L.out = self.snaps[1 - self.cur].data_ptr()
        L.aux = out.data_ptr()
        L.quantity = qi
        L.qcomp = nx * ny * nz
        L.qscale = float(scale)
        L.qsy = nx
        L.qsz = nx * ny
        L.reserved0 = nc
        L.ylo, L.yhi, L.zlo, L.zhi = 0, ny, 0, nz
        L.iter = self.iter
        L.reserved1 = max(1, self.iter - self.average_start)
        L.stream = self._stream()
        if self.particles is not None:   # quantities may look at particles (e.g. Checks)
            self.particles.attach_for_quantity(self)
        try:
            self.lib.quantity(L, self.prec)
        finally:
            if self.particles is not None:
                self.particles.detach(self)
        L.reserved0 = 0
        return out

    def color(self, z: Optional[int] = None) -> Optional[torch.Tensor]:
        """the model's node colour pair (value l, weight w; reference ``Color()``) over the
        global z slice `z` (default: the middle one, reference LatticeContainer::Color):
        (ny, nx, 2) on this rank's rows, or None when the slice is not on this rank.
        Evaluated by the quantity kernel with quantity index -1 (the emitted ``color()``)"""
        gz = self.gshape[2] // 2 if z is None else int(z)
        if not 0 <= gz < self.gshape[2]:
            raise ValueError(f"slice z={gz} outside the lattice")
        lz = gz - self.slab.offset[2]
        nx, ny, nz = self.shape
        if not 0 <= lz < nz:
            return None
        out = torch.empty((2, ny, nx), dtype=self.rdtype, device=self.device)
        self._sync_settings()
        L = self._L
        L.in_ = self.snaps[self.cur].data_ptr()
        L.out = self.snaps[1 - self.cur].data_ptr()
        L.aux = out.data_ptr()
        L.quantity = -1
        L.qcomp = nx * ny
        L.qscale = 1.0
        L.qsy = nx
        L.qsz = nx * ny
        L.reserved0 = 2
        L.ylo, L.yhi, L.zlo, L.zhi = 0, ny, lz, lz + 1
        L.iter = self.iter
        L.reserved1 = max(1, self.iter - self.average_start)
        L.stream = self._stream()
        if self.particles is not None:
            self.particles.attach_for_quantity(self)
        try:
            self.lib.quantity(L, self.prec)
        finally:
            if self.particles is not None:
                self.particles.detach(self)
            L.reserved0 = 0
            L.zlo, L.zhi = 0, nz
        return out.permute(1, 2, 0)

    def draw_wall(self, x: int, y: int, z: Optional[int] = None, kind: str = "Wall"):
        """set one node (global coordinates; z default: the rendered middle slice) to a
        boundary type — the reference window's mouse editing (MouseMove,
        src/Solver.cpp.Rt:730-745: FlagOverwrite of NODE_Wall under the pointer)"""
        m = self.model
        nt = m.node_type(kind)
        z = self.gshape[2] // 2 if z is None else int(z)
        ox, oy, oz = self.slab.offset
        nx, ny, nz = self.shape
        lx, ly, lz = int(x) - ox, int(y) - oy, z - oz
        if not (0 <= lx < nx and 0 <= ly < ny and 0 <= lz < nz):
            return
        if nt is None:
            raise KeyError(f"model {m.name} has no node type {kind}")
        full = self.flags.cpu().numpy().view(np.uint16 if m.flag_bits == 16 else np.uint32)[:, :, :nx].copy()
        v = int(full[self.gz + lz, self.gy + ly, lx])
        full[self.gz + lz, self.gy + ly, lx] = (v & ~nt.mask) | nt.value     # its group only
        self.set_flags(full)

    def _adjoint_quantity(self, q, nc: int) -> torch.Tensor:
        """adjoint quantities (reference AddQuantity(adjoint=T)) from the adjoint state of
        the last Adjoint sweep (zeros before any): <F>B = dJ/dF, RhoB = sum of the
        adjoint populations of the first density group"""
        nx, ny, nz = self.shape
        out = torch.zeros((nc, nz, ny, nx), dtype=self.rdtype, device=self.device)
        a = getattr(self, "adjoint_state", None)
        name = q.name
        if a is None or not (name.endswith("B") or q.adjoint_of):
            return out
        a = a[:, self.gz:self.gz + nz, self.gy:self.gy + ny, :nx].to(self.device, self.rdtype)
        m = self.model
        if q.adjoint_of:
            sel = [i for i, f in enumerate(m.fields) if q.adjoint_of in (f.group, f.nicename, f.name)]
            out[0] = a[sel].sum(0)
            return out
        base = name[:-1]
        idx = [i for i, f in enumerate(m.fields) if base in (f.nicename, f.array) or base.lower() in
               (f.nicename.lower(), f.array.lower())]
        if idx:
            out[0] = a[idx[0]]
        elif base in ("Rho", "U") and m.densities:
            # RhoB / UB: zeroth / first moment of the adjoint populations of the first group
            g = m.densities[0].field.group
            dens = [d for d in m.densities if d.field.group == g]
            sel = [m.fields.index(d.field) for d in dens]
            if base == "Rho":
                out[0] = a[sel].sum(0)
            else:
                for k, attr in enumerate(("dx", "dy", "dz")[:nc]):
                    out[k] = sum(a[i] * float(getattr(d, attr)) for i, d in zip(sel, dens) if getattr(d, attr))
        return out

    # ------------------------------------------------------------------ state
    def state(self) -> torch.Tensor:
        return self.fields_interior()

    @property
    def nodes(self) -> int:
        return self.gshape[0] * self.gshape[1] * self.gshape[2]

    def memory_bytes(self) -> int:
        es = self.snaps[0].element_size()
        return 2 * self.nf * self.fs * es + self.flags.numel() * self.flags.element_size()
