"""Native multi-rank iteration: the n steps of an action of a slab-decomposed lattice run
in one C++ call (csrc/include/tclb_rt/dist_loop.hpp) — border launches, halo exchange,
interior launch, per stage and step, with no Python in between.

Reference: each MPI rank runs Lattice::Iterate in C++, RunBorder -> MPIStream_A ->
RunInterior -> MPIStream_B (src/Lattice.cu.Rt:466-533,900-989), with received margins
copied into the next snapshot's margin blocks (src/Lattice.cu.Rt:371-378,439-456).

Transports (``TCLB_DIST_TRANSPORT`` = auto | rccl | copy):

* ``rccl``     — GPU: this module's own RCCL communicator (librccl dlopen'ed from torch's
  lib dir; the unique id travels through torch.distributed), grouped ncclSend/ncclRecv of
  each halo field's planes straight from / into the output snapshot on a high-priority
  comm stream (no pack, no unpack).  With one rank (LoopbackComm) the peer is the rank
  itself: RCCL self send/receive, so a single MI355X exercises the multi-GPU code.
* ``copy``     — one rank as its own neighbour, the plan executed as device-to-device
  copies (GPU) or memcpy (CPU).
* ``callback`` — CPU ranks (gloo): the loop calls back into Python per exchange, which
  runs the plan's ops as torch.distributed isend/irecv.  Same plan, same loop.
"""
from __future__ import annotations

import ctypes
import os
import threading
import traceback
from typing import Dict, Optional, Tuple

import torch

from ..ops import abi
from .comm import LoopbackComm, TorchDistComm

MAX_STAGES = 32       # dist_loop.hpp DIST_MAX_STAGES
TAG_HI = 1 << 12      # tag offset of the fields read from above


class HaloOp(ctypes.Structure):
    _fields_ = [("off", ctypes.c_longlong), ("bytes", ctypes.c_longlong), ("kind", ctypes.c_int),
                ("peer", ctypes.c_int), ("tag", ctypes.c_int), ("reserved", ctypes.c_int)]


class DistPlan(ctypes.Structure):
    _fields_ = [("axis", ctypes.c_int), ("n", ctypes.c_int), ("g", ctypes.c_int), ("overlap", ctypes.c_int),
                ("nstages", ctypes.c_int), ("stage", ctypes.c_int * MAX_STAGES),
                ("op0", ctypes.c_int * MAX_STAGES), ("nops", ctypes.c_int * MAX_STAGES),
                ("ops", ctypes.c_void_p)]


XCHG_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(HaloOp), ctypes.c_int)

TRANSPORT_CODE = {"copy": 0, "rccl": 1, "callback": 2}


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
        L.tclb_dist_iterate_cpu.argtypes = [P, i, i, i, P, i, i, P, P, P, P, P]
        L.tclb_dist_iterate_cpu.restype = i
        if L.tclb_dist_sizeof_plan_cpu() != ctypes.sizeof(DistPlan) or \
                L.tclb_dist_sizeof_op_cpu() != ctypes.sizeof(HaloOp):
            raise NativeDistError("ABI mismatch of DistPlan/HaloOp in libtclb_host.so")
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
        L.tclb_dist_iterate.argtypes = [P, P, i, i, i, P, P, P, P]
        L.tclb_dist_iterate.restype = i
        L.tclb_dist_exchange.argtypes = [P, P, P, i, P]
        L.tclb_dist_exchange.restype = i
        if L.tclb_dist_sizeof_plan() != ctypes.sizeof(DistPlan) or L.tclb_dist_sizeof_op() != ctypes.sizeof(HaloOp):
            raise NativeDistError("ABI mismatch of DistPlan/HaloOp in libtclb_device.so")
        _dev = L
    return _dev


def _err() -> str:
    return _dev_lib().tclb_dist_last_error().decode(errors="replace")


def choose_transport(comm, gpu: bool) -> str:
    env = os.environ.get("TCLB_DIST_TRANSPORT", "auto")
    if isinstance(comm, TorchDistComm):
        if gpu:
            if comm.backend != "nccl":
                raise NativeDistError(f"native GPU loop needs the nccl (RCCL) backend, not {comm.backend}")
            return "rccl"
        return "callback"
    if env == "rccl" and gpu:
        return "rccl"          # one rank, RCCL send/receive to itself
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
        _ctx_cache[key] = ctx
        return ctx


class NativeDist:
    """the native loop of one lattice (tclb_amd.lattice.Lattice) over its slab split"""

    def __init__(self, lat):
        self.lat = lat
        comm = lat.comm
        self.gpu = lat.is_gpu
        self.transport = choose_transport(comm, self.gpu)
        self.rank = comm.rank if isinstance(comm, TorchDistComm) else 0
        self._plans: Dict[Tuple[int, ...], tuple] = {}
        self.ctx = gpu_context(comm, self.transport, lat.device) if self.gpu else None
        self._cb = XCHG_FN(self._exchange_cb) if (not self.gpu and self.transport == "callback") else None
        self._cb_error: Optional[str] = None

    @staticmethod
    def supported(lat) -> bool:
        """slab split with every halo contiguous per field: z slabs, or y slabs of 2-D
        lattices (one z plane)"""
        ax = lat.slab.axis
        return lat.g > 0 and (ax == 2 or (ax == 1 and lat.NZ == 1))

    # ------------------------------------------------------------------ plan
    def ops_for(self, fields) -> list:
        """the halo ops of one stage saving `fields` (see dist_loop.hpp for the order)"""
        lat = self.lat
        ax = lat.slab.axis
        g = lat.g
        n = lat.shape[2] if ax == 2 else lat.shape[1]
        plane = lat.NY * lat.px if ax == 2 else lat.px
        es = lat.snaps[0].element_size()
        if isinstance(lat.comm, TorchDistComm):
            prev, nxt = lat.slab.neighbours(ax)
        else:
            prev = nxt = 0
        fs = set(fields)
        lo = [i for i in lat.halo_lo if i in fs]        # read from below: my top planes go up
        hi = [i for i in lat.halo_hi if i in fs]        # read from above: my bottom planes go down
        b = g * plane * es
        ops = []
        for f in lo:
            ops.append(((f * lat.fs + n * plane) * es, b, 0, nxt, f))
        for f in hi:
            ops.append(((f * lat.fs + g * plane) * es, b, 0, prev, TAG_HI + f))
        for f in lo:
            ops.append((f * lat.fs * es, b, 1, prev, f))
        for f in hi:
            ops.append(((f * lat.fs + (n + g) * plane) * es, b, 1, nxt, TAG_HI + f))
        return ops

    def plan(self, stages: Tuple[int, ...]):
        p = self._plans.get(stages)
        if p is not None:
            return p
        lat = self.lat
        m = lat.model
        if len(stages) > MAX_STAGES:
            raise NativeDistError(f"action of {len(stages)} stages (max {MAX_STAGES})")
        P = DistPlan()
        P.axis = lat.slab.axis
        P.n = lat.shape[2] if P.axis == 2 else lat.shape[1]
        P.g = lat.g
        P.overlap = 1 if lat.overlap else 0
        P.nstages = len(stages)
        allops = []
        for k, si in enumerate(stages):
            ops = self.ops_for(lat._saved_fields(m.stages[si]))
            P.stage[k] = si
            P.op0[k] = len(allops)
            P.nops[k] = len(ops)
            allops += ops
        arr = (HaloOp * max(1, len(allops)))()
        for i, (off, b, kind, peer, tag) in enumerate(allops):
            arr[i].off, arr[i].bytes, arr[i].kind, arr[i].peer, arr[i].tag = off, b, kind, peer, tag
        P.ops = ctypes.cast(arr, ctypes.c_void_p)
        p = self._plans[stages] = (P, arr)
        return p

    # ------------------------------------------------------------------ run
    def iterate(self, L: abi.Launch, prec: int, n: int, stages, glob_last: bool, sp=None):
        P, _ = self.plan(tuple(stages))
        lib = self.lat.lib
        run = ctypes.cast(lib._run, ctypes.c_void_p)
        sample = ctypes.cast(lib._smp, ctypes.c_void_p)
        spp = ctypes.byref(sp) if sp is not None else None
        if self.gpu:
            r = _dev_lib().tclb_dist_iterate(self.ctx, ctypes.byref(L), prec, n, 1 if glob_last else 0,
                                              ctypes.byref(P), run, sample, spp)
            if r != 0:
                raise NativeDistError(f"native multi-rank loop failed ({r}): {_err()}")
            return
        self._cb_error = None
        r = _host_lib().tclb_dist_iterate_cpu(ctypes.byref(L), prec, n, 1 if glob_last else 0, ctypes.byref(P),
                                              TRANSPORT_CODE[self.transport], self.rank,
                                              ctypes.cast(self._cb, ctypes.c_void_p) if self._cb else None,
                                              None, run, sample, spp)
        if r != 0:
            raise NativeDistError(f"native multi-rank loop failed ({r})" +
                                  (f": {self._cb_error}" if self._cb_error else ""))

    def exchange(self, buf: torch.Tensor, fields):
        """one exchange of `fields` of snapshot `buf` through the native transport (GPU)"""
        ops = self.ops_for(fields)
        if not ops:
            return
        arr = (HaloOp * len(ops))()
        for i, (off, b, kind, peer, tag) in enumerate(ops):
            arr[i].off, arr[i].bytes, arr[i].kind, arr[i].peer, arr[i].tag = off, b, kind, peer, tag
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

    def _exchange_cb(self, user, base, ops, nops) -> int:
        """transport 'callback': one stage's ops as gloo isend/irecv"""
        try:
            comm = self.lat.comm
            d = comm.dist
            flat = self._flat(base)
            es = flat.element_size()
            p2p = []
            for i in range(nops):
                o = ops[i]
                t = flat[o.off // es:(o.off + o.bytes) // es]
                p2p.append(d.P2POp(d.isend if o.kind == 0 else d.irecv, t, comm._g(o.peer), comm.group, o.tag))
            for w in d.batch_isend_irecv(p2p):
                w.wait()
            return 0
        except Exception:  # noqa: BLE001 - reported through the loop's return code
            self._cb_error = traceback.format_exc(limit=4)
            return -5


def native_dist_enabled() -> bool:
    return os.environ.get("TCLB_DIST_NATIVE", "1") != "0"


__all__ = ["NativeDist", "NativeDistError", "native_dist_enabled", "choose_transport", "LoopbackComm"]
