"""Native action loop: the n steps of an action run in one C++ call
(csrc/include/tclb_rt/dist_loop.hpp action_loop) — stage launches with the border /
exchange / interior split, out-of-place and fixed-point stages, the particle hooks, the
zonal time series and every sampler, on one rank or many, over a slab or a Y x Z process
grid, with no Python in between.

Reference: each MPI rank runs Lattice::Iterate in C++: RunBorder -> MPIStream_A ->
RunInterior -> MPIStream_B (src/Lattice.cu.Rt:466-533,900-989), particle stages with
CopyInParticles / CopyOutParticles (:392-437), fixed-point stages (:484), the zone index of
the time series (:473-477), samplers (:1376-1389).

Transports (``TCLB_DIST_TRANSPORT`` = auto | rccl | ipc | copy):

Every stage exchanges ONE packed message per neighbour and direction (phase_a): the border
launches mirror their stores of the exchanged fields into contiguous send buffers
(core.hpp mirror_store; pack segments where no border split runs), and one copy launch
unpacks what arrived into the ghost planes (round 5 sent one message per field: 36 RCCL
operations per d3q27 stage).

* ``rccl``     — GPU: this module's own RCCL communicator (librccl dlopen'ed from torch's
  lib dir; the unique id travels through torch.distributed), one grouped ncclSend/ncclRecv
  per neighbour of the packed buffers on a high-priority comm stream, ncclAllReduce of the
  particle forces.  With one rank (LoopbackComm) the peer is the rank itself: RCCL self
  send/receive, so a single MI355X exercises the multi-GPU code.
* ``ipc``      — GPU, no collective library: every rank's staging buffer and a block of
  counters live in device memory the other ranks map (hipIpcGetMemHandle / OpenMemHandle,
  handles through torch.distributed).  A rank publishes READY when its send buffers are
  written, pulls its neighbours' buffers straight into its ghost planes (one copy kernel,
  peer reads over xGMI) after their READY, publishes DONE, and waits for the neighbours'
  DONE before the buffers are rewritten; the particle forces are summed from every rank's
  shared copy in rank order.  Waits are bounded (TCLB_IPC_TIMEOUT_S).  This is also the
  transport of several processes on ONE device (a gloo process group), which RCCL refuses:
  the multi-process path runs on a single MI355X (tests/test_gpu_ipc.py).
* ``copy``     — one rank as its own neighbour (or no neighbour at all), the plan executed
  as device-to-device copies (GPU) or memcpy (CPU).
* ``callback`` — CPU ranks (gloo): the loop calls back into Python per exchange phase and
  per particle-force all-reduce, which run as torch.distributed operations.  Same plan,
  same loop.
"""
from __future__ import annotations

import ctypes
import os
import threading
import traceback
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..ops import abi
from .comm import LoopbackComm, TorchDistComm

MAX_STAGES = 32       # dist_loop.hpp DIST_MAX_STAGES
TAG_HI = 1 << 12      # tag offset of the fields read from above
TAG_Y = 1 << 13       # tag offset of the grid's y phase
FIXED_POINT_SWEEPS = 100


class HaloOp(ctypes.Structure):
    _fields_ = [("off", ctypes.c_longlong), ("bytes", ctypes.c_longlong), ("kind", ctypes.c_int),
                ("peer", ctypes.c_int), ("tag", ctypes.c_int), ("buf", ctypes.c_int)]


class PackOp(ctypes.Structure):
    _fields_ = [("boff", ctypes.c_longlong), ("field0", ctypes.c_int), ("nfield", ctypes.c_int),
                ("y0", ctypes.c_int), ("ny", ctypes.c_int), ("z0", ctypes.c_int), ("nz", ctypes.c_int),
                ("unpack", ctypes.c_int), ("reserved", ctypes.c_int)]


class SegOp(ctypes.Structure):
    _fields_ = [("dst", ctypes.c_longlong), ("src", ctypes.c_longlong), ("bytes", ctypes.c_longlong),
                ("dir", ctypes.c_int), ("peer", ctypes.c_int)]


class MirrorSpec(ctypes.Structure):
    _fields_ = [("boff", ctypes.c_longlong), ("mfs", ctypes.c_longlong), ("msy", ctypes.c_longlong),
                ("msz", ctypes.c_longlong), ("moy", ctypes.c_int), ("moz", ctypes.c_int),
                ("slot", ctypes.c_byte * abi.MIRROR_FIELDS)]


class StagePlan(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ("stage", "mode", "sweeps", "particle", "op0", "nops", "opb0", "nopsb",
                                            "pk0", "npk", "run0", "nruns", "seg0", "npack", "nunpack", "mir_lo",
                                            "mir_hi", "yseg0", "nyseg", "mirror", "reserved")]


class SeriesEntry(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ("idx", "dtidx", "len", "off")]


class PartPlan(ctypes.Structure):
    _fields_ = [("P", ctypes.c_void_p), ("acc", ctypes.c_void_p), ("m", ctypes.c_void_p), ("free_", ctypes.c_void_p),
                ("n", ctypes.c_int), ("container", ctypes.c_int), ("grid", ctypes.c_void_p),
                ("grid_n", ctypes.c_longlong), ("gdim", ctypes.c_int * 3), ("cell", ctypes.c_int),
                ("ncell", ctypes.c_int), ("nl", ctypes.c_int), ("mscale", ctypes.c_double),
                ("tmp", ctypes.c_void_p), ("tmp_bytes", ctypes.c_longlong), ("a", ctypes.c_double * 3),
                ("period", ctypes.c_double * 3), ("periodic", ctypes.c_int), ("integrate", ctypes.c_int),
                ("allreduce", ctypes.c_int), ("nslots", ctypes.c_int), ("accbuf", ctypes.c_void_p),
                ("accs", ctypes.c_void_p)]


class LoopPlan(ctypes.Structure):
    _fields_ = [("axis", ctypes.c_int), ("n", ctypes.c_int), ("g", ctypes.c_int),
                ("ny", ctypes.c_int), ("nz", ctypes.c_int), ("gy", ctypes.c_int), ("gz", ctypes.c_int),
                ("overlap", ctypes.c_int), ("nstages", ctypes.c_int), ("st", StagePlan * MAX_STAGES),
                ("ops", ctypes.c_void_p), ("packs", ctypes.c_void_p), ("runs", ctypes.c_void_p),
                ("segs", ctypes.c_void_p), ("dsegs", ctypes.c_void_p), ("mirrors", ctypes.c_void_p),
                ("scratch", ctypes.c_void_p), ("staging", ctypes.c_void_p), ("fs_bytes", ctypes.c_longlong),
                ("nseries", ctypes.c_int), ("nsamplers", ctypes.c_int), ("series", ctypes.c_void_p),
                ("svals", ctypes.c_void_p), ("sslopes", ctypes.c_void_p), ("zonal", ctypes.c_void_p),
                ("samplers", ctypes.c_void_p), ("part", ctypes.c_void_p), ("peer_stg", ctypes.c_void_p * 4),
                ("ipc_peer", ctypes.c_int * 4)]


XCHG_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(HaloOp),
                           ctypes.c_int)
ALLRED_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong)

TRANSPORT_CODE = {"copy": 0, "rccl": 1, "callback": 2, "ipc": 3}
_SIZES = (("plan", LoopPlan), ("stage", StagePlan), ("part", PartPlan), ("pack", PackOp), ("series", SeriesEntry),
          ("seg", SegOp), ("mirror", MirrorSpec))


class NativeDistError(RuntimeError):
    pass


def rccl_path() -> str:
    """the RCCL library torch loaded (one RCCL instance per process)"""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "/opt/rocm/lib/librccl.so"


_host = None
_dev = None
_ctx_cache: Dict[tuple, int] = {}
_lock = threading.Lock()


def _host_lib():
    global _host
    if _host is None:
        from ..ops import host
        L = host.lib()
        P, i = ctypes.c_void_p, ctypes.c_int
        L.tclb_loop_iterate_cpu.argtypes = [P, i, i, i, i, i, P, i, i, P, P, P, P, P]
        L.tclb_loop_iterate_cpu.restype = i
        L.tclb_ad_segment_cpu.argtypes = [P, P, P]
        L.tclb_ad_segment_cpu.restype = i
        for name, st in _SIZES:
            if getattr(L, f"tclb_loop_sizeof_{name}_cpu")() != ctypes.sizeof(st):
                raise NativeDistError(f"ABI mismatch of the loop {name} struct in libtclb_host.so")
        if L.tclb_dist_sizeof_op_cpu() != ctypes.sizeof(HaloOp):
            raise NativeDistError("ABI mismatch of HaloOp in libtclb_host.so")
        _host = L
    return _host


def _dev_lib():
    global _dev
    if _dev is None:
        from ..ops import device
        L = device.lib()
        P, i = ctypes.c_void_p, ctypes.c_int
        L.tclb_dist_last_error.restype = ctypes.c_char_p
        L.tclb_dist_unique_id.argtypes = [ctypes.c_char_p, P]
        L.tclb_dist_unique_id.restype = i
        L.tclb_dist_ctx_create.argtypes = [ctypes.c_char_p, i, i, i, P]
        L.tclb_dist_ctx_create.restype = P
        L.tclb_dist_ctx_destroy.argtypes = [P]
        L.tclb_loop_iterate.argtypes = [P, P, i, i, i, i, i, P, P, P]
        L.tclb_loop_iterate.restype = i
        L.tclb_ad_segment.argtypes = [P, P, P]
        L.tclb_ad_segment.restype = i
        L.tclb_loop_exchange.argtypes = [P, P, P, i, i, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_longlong, i, P]
        L.tclb_loop_exchange.restype = i
        L.tclb_dist_exchange.argtypes = [P, P, P, i, P]
        L.tclb_dist_exchange.restype = i
        L.tclb_dist_wait.argtypes = [P, P, i]
        L.tclb_dist_wait.restype = i
        L.tclb_part_tmp_bytes.argtypes = [i, i]
        L.tclb_part_tmp_bytes.restype = ctypes.c_longlong
        L.tclb_ipc_alloc.argtypes = [ctypes.c_longlong, P]
        L.tclb_ipc_alloc.restype = P
        L.tclb_ipc_free.argtypes = [P]
        L.tclb_ipc_open.argtypes = [P]
        L.tclb_ipc_open.restype = P
        L.tclb_ipc_close.argtypes = [P]
        L.tclb_dist_sig_handle.argtypes = [P, P]
        L.tclb_dist_sig_handle.restype = i
        L.tclb_dist_sig_attach.argtypes = [P, ctypes.c_char_p]
        L.tclb_dist_sig_attach.restype = i
        L.tclb_dist_ipc_error.argtypes = [P]
        L.tclb_dist_ipc_error.restype = i
        for name, st in _SIZES:
            if getattr(L, f"tclb_loop_sizeof_{name}")() != ctypes.sizeof(st):
                raise NativeDistError(f"ABI mismatch of the loop {name} struct in libtclb_device.so")
        if L.tclb_dist_sizeof_op() != ctypes.sizeof(HaloOp):
            raise NativeDistError("ABI mismatch of HaloOp in libtclb_device.so")
        _dev = L
    return _dev


def _err() -> str:
    return _dev_lib().tclb_dist_last_error().decode(errors="replace")


def choose_transport(comm, gpu: bool) -> str:
    """GPU ranks: RCCL (default) or IPC (TCLB_DIST_TRANSPORT=ipc, or a gloo process group:
    several processes on one device, which RCCL refuses); CPU ranks: gloo callbacks; one
    rank: device copies, or RCCL / IPC to itself when asked (the multi-rank code on one
    GPU)"""
    env = os.environ.get("TCLB_DIST_TRANSPORT", "auto")
    if isinstance(comm, TorchDistComm):
        if gpu:
            if env == "ipc" or comm.backend != "nccl":
                return "ipc"
            return "rccl"
        return "callback"
    if env in ("rccl", "ipc") and gpu:
        return env             # one rank sending to / pulling from itself
    return "copy"


def gpu_context(comm, transport: str, device: torch.device) -> int:
    """this rank's native context (RCCL communicator or copy transport, comm stream,
    events), one per (communicator, device, transport) for the life of the process"""
    key = (id(comm) if isinstance(comm, TorchDistComm) else "self", device.index, transport)
    with _lock:
        ctx = _ctx_cache.get(key)
        if ctx:
            return ctx
        L = _dev_lib()
        path = rccl_path().encode()
        uid = ctypes.create_string_buffer(128)
        size, rank = (comm.size, comm.rank) if isinstance(comm, TorchDistComm) else (1, 0)
        if transport == "rccl":
            if rank == 0:
                r = L.tclb_dist_unique_id(path, uid)
                if r != 0:
                    raise NativeDistError(f"ncclGetUniqueId failed ({r}): {_err()}")
            if size > 1:
                raw = comm.bcast_object(bytes(uid.raw) if rank == 0 else None)
                ctypes.memmove(uid, raw, 128)
        with torch.cuda.device(device):
            ctx = L.tclb_dist_ctx_create(path, TRANSPORT_CODE[transport], size, rank, uid)
            if not ctx:
                raise NativeDistError(f"native dist context ({transport}) failed: {_err()}")
            if transport == "ipc":
                # every rank maps every other rank's signal block (counters of the pulls)
                hb = ctypes.create_string_buffer(HANDLE_BYTES)
                if L.tclb_dist_sig_handle(ctx, hb) != 0:
                    raise NativeDistError(f"IPC signal handle failed: {_err()}")
                hs = comm.gather_objects(bytes(hb.raw)) if size > 1 else [bytes(hb.raw)]
                if L.tclb_dist_sig_attach(ctx, b"".join(hs)) != 0:
                    raise NativeDistError(f"IPC signal attach failed: {_err()}")
        _ctx_cache[key] = ctx
        return ctx


HANDLE_BYTES = 64     # hipIpcMemHandle_t


class IpcBuf:
    """device memory another process of the node can map (tclb_ipc_alloc: zeroed)"""

    def __init__(self, nbytes: int, device: torch.device):
        self.handle = ctypes.create_string_buffer(HANDLE_BYTES)
        with torch.cuda.device(device):
            self.ptr = _dev_lib().tclb_ipc_alloc(int(nbytes), self.handle)
        if not self.ptr:
            raise NativeDistError(f"IPC buffer of {nbytes} bytes: {_err()}")
        self.nbytes = int(nbytes)

    def __del__(self):
        if getattr(self, "ptr", None) and _dev is not None:
            _dev.tclb_ipc_free(self.ptr)
            self.ptr = None


class IpcMap:
    """another rank's IpcBuf mapped into this process"""

    def __init__(self, handle: bytes, device: torch.device):
        with torch.cuda.device(device):
            self.ptr = _dev_lib().tclb_ipc_open(handle)
        if not self.ptr:
            raise NativeDistError(f"IPC open failed: {_err()}")

    def __del__(self):
        if getattr(self, "ptr", None) and _dev is not None:
            _dev.tclb_ipc_close(self.ptr)
            self.ptr = None


def _runs(idx: List[int]) -> List[Tuple[int, int]]:
    out: List[Tuple[int, int]] = []
    for i in idx:
        if out and out[-1][1] == i:
            out[-1] = (out[-1][0], i + 1)
        else:
            out.append((i, i + 1))
    return out


def _carr(ctype, items):
    a = (ctype * max(1, len(items)))()
    for i, it in enumerate(items):
        for k, v in it.items():
            setattr(a[i], k, v)
    return a


_OPF = ("off", "bytes", "kind", "peer", "tag", "buf")


class NativeLoop:
    """the native action loop of one lattice (tclb_amd.lattice.Lattice): one rank or many,
    slab or Y x Z grid"""

    def __init__(self, lat):
        self.lat = lat
        comm = lat.comm
        self.gpu = lat.is_gpu
        self.multi = isinstance(comm, TorchDistComm)
        self.transport = choose_transport(comm, self.gpu) if comm.distributed else "copy"
        self.rank = comm.rank if self.multi else 0
        self._plans: Dict[tuple, tuple] = {}
        self.ctx = gpu_context(comm if comm.distributed else LoopbackComm(), self.transport, lat.device) \
            if self.gpu else None
        cb = not self.gpu and self.transport == "callback"
        self._cb = XCHG_FN(self._exchange_cb) if cb else None
        self._ared = ALLRED_FN(self._allreduce_cb) if cb else None
        self._cb_error: Optional[str] = None
        self._staging: Dict[int, torch.Tensor] = {}     # data_ptr -> the plans' staging buffers
        self._part_tmp: Optional[torch.Tensor] = None

    @staticmethod
    def supported(lat) -> bool:
        """what the loop steps: one rank without ghosts, slab splits with every halo
        contiguous per field (z slabs, or y slabs of 2-D lattices), and the Y x Z grid"""
        ax = lat.slab.axis
        if lat.g == 0:
            return True
        return ax == 3 or ax == 2 or (ax == 1 and lat.NZ == 1)

    # ------------------------------------------------------------------ plan
    def _peers(self, axis: int) -> Tuple[int, int]:
        return self.lat.slab.neighbours(axis) if self.multi else (0, 0)

    def ops_for(self, fields) -> list:
        """the direct (contiguous plane) halo ops of one stage saving `fields`: along the
        slab axis, or the z phase of the grid (see dist_loop.hpp for the order)"""
        lat = self.lat
        ax = 2 if lat.slab.axis == 3 else lat.slab.axis
        g = lat.gz if lat.slab.axis == 3 else lat.g
        n = lat.shape[2] if ax == 2 else lat.shape[1]
        plane = lat.NY * lat.px if ax == 2 else lat.px
        es = lat.snaps[0].element_size()
        prev, nxt = self._peers(ax)
        fs = set(fields)
        lo_set, hi_set = lat.halo_sets[ax]
        lo = [i for i in lo_set if i in fs]        # read from below: my top planes go up
        hi = [i for i in hi_set if i in fs]        # read from above: my bottom planes go down
        b = g * plane * es
        ops = []
        for f in lo:
            ops.append(((f * lat.fs + n * plane) * es, b, 0, nxt, f, 0))
        for f in hi:
            ops.append(((f * lat.fs + g * plane) * es, b, 0, prev, TAG_HI + f, 0))
        for f in lo:
            ops.append((f * lat.fs * es, b, 1, prev, f, 0))
        for f in hi:
            ops.append(((f * lat.fs + (n + g) * plane) * es, b, 1, nxt, TAG_HI + f, 0))
        return ops

    def phase_a(self, fields, stg_off: int, k: int = 0, lay=None, peer_off=None):
        """the packed exchange of stage k along the slab axis (or the z phase of the
        grid): ONE message per neighbour and direction.  The border launches mirror their
        stores of the exchanged fields into the send buffers (MirrorSpec; a launch that
        cannot — no overlap split, out-of-place stages — is followed by pack segments), the
        received buffers are unpacked into the ghost planes by one copy launch.  Staging
        layout [send up][send down][recv below][recv above], each [field][g planes]; the
        copy transport (this rank is its own neighbour) receives nothing: its send buffers
        are unpacked directly; the IPC transport receives nothing either: it pulls the
        neighbours' send buffers straight into its ghost planes (dir 2 segments, source
        offsets from the neighbour's own layout, peer_off).  Ops in the issue order every
        rank shares: send up, send down, receive from below, receive from above.  Returns
        (ops, packs, unpacks, mirrors (lo launch, hi launch), staging bytes)."""
        lat = self.lat
        grid = lat.slab.axis == 3
        ax = 2 if grid else lat.slab.axis
        g = lat.gz if grid else lat.g
        n = lat.shape[2] if ax == 2 else lat.shape[1]
        plane = lat.NY * lat.px if ax == 2 else lat.px
        es = lat.snaps[0].element_size()
        prev, nxt = self._peers(ax)
        fs = set(fields)
        lo_set, hi_set = lat.halo_sets[ax]
        lo = [i for i in lo_set if i in fs]        # read from below: my top planes go up
        hi = [i for i in hi_set if i in fs]        # read from above: my bottom planes go down
        per = g * plane * es
        off = stg_off
        su, off = off, off + per * len(lo)
        sd, off = off, off + per * len(hi)
        if lay is not None:
            lay[(k, "A_su")], lay[(k, "A_sd")] = su, sd
        ipc = self.transport == "ipc"
        if self.transport == "copy":
            rb, ra = su, sd
        elif not ipc:
            rb, off = off, off + per * len(lo)
            ra, off = off, off + per * len(hi)
        ops = []
        if self.transport not in ("copy", "ipc"):
            if lo:
                ops.append((su, per * len(lo), 0, nxt, 0, 1))
            if hi:
                ops.append((sd, per * len(hi), 0, prev, TAG_HI, 1))
            if lo:
                ops.append((rb, per * len(lo), 1, prev, 0, 1))
            if hi:
                ops.append((ra, per * len(hi), 1, nxt, TAG_HI, 1))
        fsb = lat.fs * es
        packs = [(su + j * per, f * fsb + n * plane * es, per, 0, 0) for j, f in enumerate(lo)] + \
                [(sd + j * per, f * fsb + g * plane * es, per, 0, 0) for j, f in enumerate(hi)]
        if ipc:
            pu = peer_off(0, k, "A_su") if lo else 0      # the rank below's send-up buffer
            pd = peer_off(1, k, "A_sd") if hi else 0      # the rank above's send-down buffer
            unpacks = [(f * fsb, pu + j * per, per, 2, 0) for j, f in enumerate(lo)] + \
                      [(f * fsb + (n + g) * plane * es, pd + j * per, per, 2, 1) for j, f in enumerate(hi)]
        else:
            unpacks = [(f * fsb, rb + j * per, per, 1, 0) for j, f in enumerate(lo)] + \
                      [(f * fsb + (n + g) * plane * es, ra + j * per, per, 1, 0) for j, f in enumerate(hi)]

        def mirror(flist, boff, r0):
            if not flist:
                return None
            slot = [-1] * abi.MIRROR_FIELDS
            for j, f in enumerate(flist):
                slot[f] = j
            if ax == 2:
                spec = (g * plane, lat.px, lat.NY * lat.px, lat.gy, -r0)
            else:
                spec = (g * plane, lat.px, g * lat.px, -r0, lat.gz)
            return (boff,) + spec + (slot,)
        mirrors = (mirror(hi, sd, 0), mirror(lo, su, n - g))
        return ops, packs, unpacks, mirrors, off - stg_off

    def y_phase(self, fields, stg_off: int, k: int = 0, lay=None, peer_off=None):
        """the grid's y phase of stage k: rows [n, n+g) of the fields read from below go
        up, rows [g, 2g) of those read from above go down, over the ghost-inclusive z
        extent, through staging messages [send up][send down][recv below][recv above];
        the IPC transport pulls the y neighbours' send messages into its receive buffers
        (dir 3 segments) instead of exchanging them.  Returns (ops, packs, pulls, bytes)"""
        lat = self.lat
        g, n = lat.gy, lat.shape[1]
        es = lat.snaps[0].element_size()
        prev, nxt = self._peers(1)
        fs = set(fields)
        lo_set, hi_set = lat.halo_sets[1]
        lo = [i for i in lo_set if i in fs]
        hi = [i for i in hi_set if i in fs]
        per = lat.NZ * g * lat.px * es             # one field's rows
        ops, packs, pulls = [], [], []
        msgs, off = {}, stg_off
        for name, flist in (("su", lo), ("sd", hi), ("rb", lo), ("ra", hi)):
            msgs[name] = off
            off += per * len(flist)
        if lay is not None:
            lay[(k, "B_su")], lay[(k, "B_sd")] = msgs["su"], msgs["sd"]
        ipc = self.transport == "ipc"

        def pk(base, flist, y0, unpack):
            o = base
            for r0, r1 in _runs(flist):
                packs.append({"boff": o, "field0": r0, "nfield": r1 - r0, "y0": y0, "ny": g, "z0": 0,
                              "nz": lat.NZ, "unpack": unpack})
                o += per * (r1 - r0)
        if lo:
            pk(msgs["su"], lo, n, 0)
            if not ipc:
                ops.append((msgs["su"], per * len(lo), 0, nxt, TAG_Y, 1))
        if hi:
            pk(msgs["sd"], hi, g, 0)
            if not ipc:
                ops.append((msgs["sd"], per * len(hi), 0, prev, TAG_Y + TAG_HI, 1))
        if lo:
            if ipc:
                pulls.append((msgs["rb"], peer_off(2, k, "B_su"), per * len(lo), 3, 2))
            else:
                ops.append((msgs["rb"], per * len(lo), 1, prev, TAG_Y, 1))
            pk(msgs["rb"], lo, 0, 1)
        if hi:
            if ipc:
                pulls.append((msgs["ra"], peer_off(3, k, "B_sd"), per * len(hi), 3, 3))
            else:
                ops.append((msgs["ra"], per * len(hi), 1, nxt, TAG_Y + TAG_HI, 1))
            pk(msgs["ra"], hi, n + g, 1)
        return ops, packs, pulls, off - stg_off

    @staticmethod
    def stage_mode(k: int, st) -> int:
        """0 plain, 1 out of place (snapshot reads), 2 fixed point (lattice.py run_action)"""
        if k > 0 and st.fixed_point:
            return 2
        if k > 0 and st.snapshot_reads:
            return 1
        return 0

    def _ipc_ranks(self) -> List[int]:
        """ranks of the IPC peers 0..3: below / above along the slab axis (the grid's z),
        then below / above along the grid's y (-1: none)"""
        lat = self.lat
        if lat.g == 0:
            return [-1] * 4
        if lat.slab.axis == 3:
            return list(self._peers(2)) + list(self._peers(1))
        return list(self._peers(lat.slab.axis)) + [-1, -1]

    def _build(self, P: LoopPlan, stages, lay, peer_off, field_lists=None):
        """fill P's stages (field_lists: exchange-only stages of these field sets);
        returns (ops, packs, runs, segs, mirrors, staging bytes, needs the scratch
        snapshot)"""
        lat = self.lat
        m = lat.model
        ax = P.axis
        allops, allpacks, runs, segs, mirrors = [], [], [], [], []
        stg_bytes = 0
        need_scratch = False
        for k, si in enumerate(stages):
            st = m.stages[si]
            fields = lat._saved_fields(st) if field_lists is None else field_lists[k]
            mode = self.stage_mode(k, st) if field_lists is None else 0
            need_scratch |= mode > 0
            S = P.st[k]
            S.stage, S.mode, S.sweeps = si, mode, FIXED_POINT_SWEEPS if mode == 2 else 1
            S.particle = 1 if st.particle and field_lists is None else 0
            S.run0, S.nruns = len(runs), len(_runs(fields)) if mode > 0 else 0
            if mode > 0:
                runs += _runs(fields)
            S.mir_lo = S.mir_hi = -1
            # a split stage's class-0 nodes store nothing (not even into the mirror): its
            # send buffers are packed from the snapshot instead
            S.mirror = 0 if (st.split or field_lists is not None) else 1
            if ax > 0:
                ops, pks, ups, mirs, nb = self.phase_a(fields, stg_bytes, k, lay, peer_off)
                if not S.mirror:
                    mirs = (None, None)
                stg_bytes += nb
                S.op0, S.nops = len(allops), len(ops)
                allops += ops
                S.seg0, S.npack, S.nunpack = len(segs), len(pks), len(ups)
                segs += pks + ups
                for side, mspec in zip(("mir_lo", "mir_hi"), mirs):
                    if mspec is not None:
                        setattr(S, side, len(mirrors))
                        mirrors.append(mspec)
                if ax == 3:
                    yops, ypk, ypull, yb = self.y_phase(fields, stg_bytes, k, lay, peer_off)
                    S.opb0, S.nopsb = len(allops), len(yops)
                    S.pk0, S.npk = len(allpacks), len(ypk)
                    S.yseg0, S.nyseg = len(segs), len(ypull)
                    segs += ypull
                    allops += yops
                    allpacks += ypk
                    stg_bytes += yb
        return allops, allpacks, runs, segs, mirrors, stg_bytes, need_scratch

    def plan(self, action: str, fields: Optional[Tuple[int, ...]] = None):
        """the loop plan of `action` (cached); fields: instead a one-stage plan that only
        exchanges these fields (exchange_fields)"""
        lat = self.lat
        m = lat.model
        key = (action, lat.g, lat.overlap, fields)
        p = self._plans.get(key)
        if p is not None:
            return p
        stages = [m.stage_index(s) for s in m.action(action).stages] if fields is None else [0]
        flists = None if fields is None else [list(fields)]
        if len(stages) > MAX_STAGES:
            raise NativeDistError(f"action of {len(stages)} stages (max {MAX_STAGES})")
        P = LoopPlan()
        ax = lat.slab.axis if lat.g > 0 else 0
        P.axis = ax
        # overlap 2 (GPU): border launches + exchange on the comm stream, concurrent with
        # the interior launch (TCLB_CONCURRENT_BORDERS=0: before it, on the compute stream)
        conc = self.gpu and os.environ.get("TCLB_CONCURRENT_BORDERS", "1") != "0"
        P.overlap = (2 if conc else 1) if lat.overlap else 0
        if ax in (1, 2):
            P.n = lat.shape[2] if ax == 2 else lat.shape[1]
            P.g = lat.g
        elif ax == 3:
            P.ny, P.nz, P.gy, P.gz = lat.shape[1], lat.shape[2], lat.gy, lat.gz
        P.nstages = len(stages)
        keep: list = []
        ipc = self.transport == "ipc" and ax > 0
        peer_off = None
        if ipc:
            # two passes: this rank's staging layout, then (its buffer allocated and every
            # rank's layout and handle gathered) the pulls from the neighbours' layouts
            lay: Dict[tuple, int] = {}
            nb = self._build(P, stages, lay, lambda *a: 0, flists)[5]
            buf = IpcBuf(max(nb, 16), lat.device)
            keep.append(buf)
            mine = (lay, bytes(buf.handle.raw))
            every = lat.comm.gather_objects(mine) if self.multi else [mine]
            ranks = self._ipc_ranks()
            maps: Dict[int, int] = {}
            for r in ranks:
                if r >= 0 and r not in maps:
                    if r == self.rank:
                        maps[r] = buf.ptr
                    else:
                        mp_ = IpcMap(every[r][1], lat.device)
                        keep.append(mp_)
                        maps[r] = mp_.ptr
            for i, r in enumerate(ranks):
                P.ipc_peer[i] = r
                P.peer_stg[i] = maps[r] if r >= 0 else None
            peer_off = lambda i, k, name: every[ranks[i]][0][(k, name)]  # noqa: E731
        else:
            for i in range(4):
                P.ipc_peer[i] = -1
        allops, allpacks, runs, segs, mirrors, stg_bytes, need_scratch = self._build(P, stages, None, peer_off, flists)
        arr = _carr(HaloOp, [dict(zip(_OPF, o)) for o in allops])
        pks = _carr(PackOp, allpacks)
        rarr = (ctypes.c_int * max(2, 2 * len(runs)))(*[v for r in runs for v in r])
        P.ops = ctypes.cast(arr, ctypes.c_void_p)
        P.packs = ctypes.cast(pks, ctypes.c_void_p)
        P.runs = ctypes.cast(rarr, ctypes.c_void_p)
        P.fs_bytes = lat.fs * lat.snaps[0].element_size()
        sarr = _carr(SegOp, [dict(zip(("dst", "src", "bytes", "dir", "peer"), o)) for o in segs])
        marr = (MirrorSpec * max(1, len(mirrors)))()
        for i, (boff, mfs, msy, msz, moy, moz, slot) in enumerate(mirrors):
            M = marr[i]
            M.boff, M.mfs, M.msy, M.msz, M.moy, M.moz = boff, mfs, msy, msz, moy, moz
            M.slot[:] = slot
        P.segs = ctypes.cast(sarr, ctypes.c_void_p)
        P.mirrors = ctypes.cast(marr, ctypes.c_void_p)
        keep += [arr, pks, rarr, sarr, marr]
        if self.gpu and segs:
            dsg = torch.frombuffer(bytearray(bytes(sarr)), dtype=torch.uint8).to(lat.device)
            keep.append(dsg)
            P.dsegs = dsg.data_ptr()
        else:
            P.dsegs = P.segs
        if need_scratch:
            sc = lat._scratch_snapshot()
            P.scratch = sc.data_ptr()
        if ipc:
            P.staging = keep[0].ptr
        elif stg_bytes:
            # each plan owns its staging buffer (kept alive with the plan): a buffer shared
            # by the cached plans and regrown for a larger one would leave the earlier
            # plans' raw pointers dangling
            stg = torch.zeros(stg_bytes, dtype=torch.uint8, device=lat.device)
            keep.append(stg)
            P.staging = stg.data_ptr()
            self._staging[P.staging] = stg
        p = self._plans[key] = (P, keep)
        return p

    # ------------------------------------------------------------------ per-call parts
    def _series(self, P: LoopPlan, keep: list):
        lat = self.lat
        if not lat.zseries:
            P.nseries = 0
            return
        nzs, nzones = lat.zvals.shape
        ents, vals, slopes = [], [], []
        for (zi, z), v in lat.zseries.items():
            n = len(v)
            for k in range(n):
                lo, hi = max(k - 1, 0), min(k + 1, n - 1)
                slopes.append((v[hi] - v[lo]) / max(hi - lo, 1))
            ents.append({"idx": zi * nzones + z, "dtidx": nzs * nzones + zi * nzones + z, "len": n,
                         "off": len(vals)})
            vals += [float(x) for x in v]
        E = _carr(SeriesEntry, ents)
        if self.gpu:
            Ed = torch.frombuffer(bytearray(bytes(E)), dtype=torch.uint8).to(lat.device)
            keep.append(Ed)
            P.series = Ed.data_ptr()
        else:
            keep.append(E)
            P.series = ctypes.cast(E, ctypes.c_void_p)
        vt = torch.tensor(vals, dtype=torch.float64, device=lat.device)
        sl = torch.tensor(slopes, dtype=torch.float64, device=lat.device)
        keep += [vt, sl]
        P.nseries, P.svals, P.sslopes = len(ents), vt.data_ptr(), sl.data_ptr()
        P.zonal = lat.zonal_t.data_ptr()

    def _samplers(self, P: LoopPlan, n: int, keep: list):
        smps = self.lat.samplers
        P.nsamplers = len(smps)
        if not smps:
            P.samplers = None
            return
        arr = (abi.SamplePlan * len(smps))()
        for i, s in enumerate(smps):
            sp = s.plan_for(n)
            ctypes.memmove(ctypes.byref(arr[i]), ctypes.byref(sp), ctypes.sizeof(abi.SamplePlan))
        keep.append(arr)
        P.samplers = ctypes.cast(arr, ctypes.c_void_p)

    def _particles(self, P: LoopPlan, keep: list):
        lat = self.lat
        ps = lat.particles
        if ps is None:
            P.part = None
            return
        ps._ensure(lat)
        d = ps._d
        Q = PartPlan()
        n = ps.n
        Q.P, Q.acc, Q.m, Q.free_, Q.n = d["P"].data_ptr(), d["acc"].data_ptr(), d["m"].data_ptr(), \
            d["free"].data_ptr(), n
        kind = d["kind"]
        Q.container = {None: 0, "grid": 1, "tree": 2}[kind]
        if kind is not None:
            Q.grid, Q.grid_n = d["grid"].data_ptr(), d["grid"].numel()
        if kind == "grid":
            Q.gdim[0], Q.gdim[1], Q.gdim[2] = d["gdim"]
            Q.cell, Q.ncell = d["cell"], d["ncell"]
        if kind == "tree":
            Q.nl, Q.mscale = d["nl"], d["mscale"]
        if kind is not None and self.gpu:
            need = int(_dev_lib().tclb_part_tmp_bytes(n, Q.ncell if kind == "grid" else 0))
            if self._part_tmp is None or self._part_tmp.numel() < need:
                self._part_tmp = torch.empty(need, dtype=torch.uint8, device=lat.device)
            Q.tmp, Q.tmp_bytes = self._part_tmp.data_ptr(), self._part_tmp.numel()
        integ = ps.native_integrator()
        if integ is not None:
            Q.integrate = 1
            for k in range(3):
                Q.a[k], Q.period[k] = float(integ["a"][k]), float(integ["period"][k])
            Q.periodic = int(integ["periodic"])
        Q.allreduce = 1 if (lat.comm.distributed and lat.comm.size > 1) else 0
        Q.nslots = d.get("nslots", 1)
        if Q.allreduce and self.gpu and self.transport == "ipc":
            Q.accbuf, Q.accs = self._ipc_acc(max(n, 1))
        keep.append(Q)
        P.part = ctypes.cast(ctypes.pointer(Q), ctypes.c_void_p)

    def _ipc_acc(self, n: int):
        """the IPC all-reduce of the particle forces: this rank's shared copy of the
        accumulator and a device table of every rank's (collective on first use and when
        the particle count grows — the count is global, so every rank grows together)"""
        cur = getattr(self, "_acc_ipc", None)
        if cur is None or cur[0] < n:
            lat = self.lat
            buf = IpcBuf(48 * n, lat.device)
            hs = lat.comm.gather_objects(bytes(buf.handle.raw))
            maps, ptrs = [], []
            for r, h in enumerate(hs):
                if r == self.rank:
                    ptrs.append(buf.ptr)
                else:
                    mp_ = IpcMap(h, lat.device)
                    maps.append(mp_)
                    ptrs.append(mp_.ptr)
            tab = torch.tensor(ptrs, dtype=torch.int64, device=lat.device)
            self._acc_ipc = cur = (n, buf, maps, tab)
        return cur[1].ptr, cur[3].data_ptr()

    # ------------------------------------------------------------------ run
    def iterate(self, L: abi.Launch, n: int, action: str, glob_last: bool):
        lat = self.lat
        P, _ = self.plan(action)
        keep: list = []
        self._series(P, keep)
        if action == "Init":
            P.nsamplers, P.samplers = 0, None        # Init records no probe row (lattice.py init)
        else:
            self._samplers(P, n, keep)
        self._particles(P, keep)
        lib = lat.lib
        run = ctypes.cast(lib._run, ctypes.c_void_p)
        sample = ctypes.cast(lib._smp, ctypes.c_void_p)
        es = lat.snaps[0].element_size()
        init = 1 if action == "Init" else 0
        if self.gpu:
            r = _dev_lib().tclb_loop_iterate(self.ctx, ctypes.byref(L), lat.prec, es, n, 1 if glob_last else 0, init,
                                             ctypes.byref(P), run, sample)
            if r != 0:
                raise NativeDistError(f"native action loop failed ({r}): {_err()}")
            return
        self._cb_error = None
        r = _host_lib().tclb_loop_iterate_cpu(ctypes.byref(L), lat.prec, es, n, 1 if glob_last else 0, init,
                                              ctypes.byref(P), TRANSPORT_CODE[self.transport], self.rank,
                                              ctypes.cast(self._cb, ctypes.c_void_p) if self._cb else None,
                                              ctypes.cast(self._ared, ctypes.c_void_p) if self._ared else None,
                                              None, run, sample)
        if r != 0:
            raise NativeDistError(f"native action loop failed ({r})" +
                                  (f": {self._cb_error}" if self._cb_error else ""))

    def wait(self, timeout_ms: Optional[int] = None):
        """wait for this rank's queued work with the RCCL communicator watched (a dead peer
        aborts the communicator and raises instead of hanging the rank)"""
        if not self.gpu or self.transport not in ("rccl", "ipc"):
            return
        t = int(os.environ.get("TCLB_DIST_TIMEOUT_MS", "600000")) if timeout_ms is None else timeout_ms
        stream = torch.cuda.current_stream(self.lat.device).cuda_stream
        r = _dev_lib().tclb_dist_wait(self.ctx, stream, t)
        if r != 0:
            raise NativeDistError(f"native loop wait failed ({r}): {_err()}")

    def exchange_fields(self, buf: torch.Tensor, fields=None):
        """one halo exchange of `fields` (None: all) of snapshot `buf` through the loop's
        own plan and transport (GPU ranks: RCCL or IPC); collective"""
        lat = self.lat
        fl = tuple(range(lat.nf)) if fields is None else tuple(sorted(set(fields)))
        P, _ = self.plan("Iteration", fl)
        if P.axis == 0:
            return
        stream = torch.cuda.current_stream(lat.device).cuda_stream
        L = lat._L
        r = _dev_lib().tclb_loop_exchange(self.ctx, buf.data_ptr(), ctypes.byref(P), 0, buf.element_size(),
                                          L.fs, L.sz, L.sy, L.px, stream)
        if r != 0:
            raise NativeDistError(f"native halo exchange failed ({r}): {_err()}")

    def exchange(self, buf: torch.Tensor, fields):
        """one exchange of `fields` of snapshot `buf` through the native transport (GPU)"""
        ops = self.ops_for(fields)
        if not ops:
            return
        arr = _carr(HaloOp, [dict(zip(_OPF, o)) for o in ops])
        stream = torch.cuda.current_stream(self.lat.device).cuda_stream
        r = _dev_lib().tclb_dist_exchange(self.ctx, buf.data_ptr(), ctypes.cast(arr, ctypes.c_void_p), len(ops),
                                          stream)
        if r != 0:
            raise NativeDistError(f"native halo exchange failed ({r}): {_err()}")

    def _flat(self, base: int) -> torch.Tensor:
        lat = self.lat
        for s in lat.snaps + [getattr(lat, "_scratch", None)]:
            if s is not None and s.data_ptr() == base:
                return torch.as_strided(s, (lat.nf * lat.fs,), (1,), s.storage_offset())
        raise NativeDistError("exchange of an unknown snapshot")

    def _exchange_cb(self, user, base, staging, ops, nops) -> int:
        """transport 'callback': one phase's ops as gloo isend/irecv"""
        try:
            comm = self.lat.comm
            d = comm.dist
            flat = self._flat(base)
            es = flat.element_size()
            stg = self._staging.get(staging) if staging else None
            p2p = []
            # TCLB_DIST_ORDER_MATCH=1: pair sends and receives by issue order per peer (the
            # k-th send to a peer with that peer's k-th receive from us), ignoring the plan's
            # tags — the matching RCCL applies to a group of ncclSend/ncclRecv, rehearsed on
            # gloo ranks (tests/test_distributed.py)
            order = os.environ.get("TCLB_DIST_ORDER_MATCH", "0") == "1"
            seq: Dict[Tuple[int, int], int] = {}
            for i in range(nops):
                o = ops[i]
                t = stg[o.off:o.off + o.bytes] if o.buf else flat[o.off // es:(o.off + o.bytes) // es]
                tag = o.tag
                if order:
                    k = (o.kind, o.peer)
                    tag = seq.get(k, 0)
                    seq[k] = tag + 1
                p2p.append(d.P2POp(d.isend if o.kind == 0 else d.irecv, t, comm._g(o.peer), comm.group, tag))
            for w in d.batch_isend_irecv(p2p):
                w.wait()
            return 0
        except Exception:  # noqa: BLE001 - reported through the loop's return code
            self._cb_error = traceback.format_exc(limit=4)
            return -5

    def _allreduce_cb(self, user, a, n) -> int:
        """transport 'callback': sum of the particle force accumulator over the ranks"""
        try:
            acc = self.lat.particles._d["acc"]
            if acc.data_ptr() != a or acc.numel() < n:
                raise NativeDistError("all-reduce of an unknown buffer")
            acc.copy_(self.lat.comm.allreduce_globals(acc.reshape(-1).clone(), acc.numel()).reshape(acc.shape))
            return 0
        except Exception:  # noqa: BLE001
            self._cb_error = traceback.format_exc(limit=4)
            return -6


NativeDist = NativeLoop


def native_dist_enabled() -> bool:
    return os.environ.get("TCLB_DIST_NATIVE", "1") != "0"


__all__ = ["NativeLoop", "NativeDist", "NativeDistError", "native_dist_enabled", "choose_transport", "LoopbackComm"]
