"""ctypes binding of the model-independent HIP runtime kernels (csrc/device/*.hip,
libtclb_device.so): the per-step particle kernels.  On a GPU the library must be there
(built by ``tclb_amd.build``); a missing or stale one is an error, not a silent switch to
tensor ops."""
from __future__ import annotations

import ctypes
import os
import threading

_lib = None
_lock = threading.Lock()


class DeviceRuntimeError(RuntimeError):
    pass


def lib():
    global _lib
    with _lock:
        if _lib is None:
            from .. import build as B
            path = os.path.join(B.LIB, "libtclb_device.so")
            stale = B.device_runtime_stale()
            if stale is not None:
                if os.path.exists(B.HIPCC) and not os.environ.get("TCLB_NO_BUILD"):
                    B.build_device_runtime()
                else:
                    raise DeviceRuntimeError(f"device runtime library not usable ({stale}): {path}")
            L = ctypes.CDLL(path)
            P, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
            L.tclb_part_nan_to_zero.argtypes = [P, i, P]
            L.tclb_part_nan_to_zero.restype = i
            L.tclb_part_acc_slots.argtypes = [P, i, i, P]
            L.tclb_part_acc_slots.restype = i
            L.tclb_part_rigid_step.argtypes = [P, P, P, P, i, d, d, d, i, d, d, d, P]
            L.tclb_part_rigid_step.restype = i
            L.tclb_part_build_grid.argtypes = [P, i, P, i, i, i, i, i, P, ctypes.c_longlong, P]
            L.tclb_part_build_grid.restype = i
            L.tclb_part_build_tree.argtypes = [P, i, P, i, d, P, ctypes.c_longlong, P]
            L.tclb_part_build_tree.restype = i
            L.tclb_snap_probe.argtypes = [P, P, ctypes.c_longlong, ctypes.c_longlong, i, i, i, P]
            L.tclb_snap_probe.restype = i
            L.tclb_snap_alloc.argtypes = [ctypes.POINTER(P), ctypes.c_size_t, i, i]
            L.tclb_snap_alloc.restype = i
            L.tclb_snap_free.argtypes = [P, i]
            L.tclb_snap_free.restype = i
            _lib = L
    return _lib


def _check(r: int, what: str):
    if r != 0:
        raise DeviceRuntimeError(f"{what} failed: HIP error {r}")


def nan_to_zero(t, stream: int):
    """t (contiguous fp64 device tensor): NaN -> 0 in place"""
    _check(lib().tclb_part_nan_to_zero(t.data_ptr(), t.numel(), stream), "particle NaN guard")


def acc_slots(acc, n6: int, nslots: int, stream: int):
    """the accumulator copies of a particle stage summed into the first (core.hpp particle_acc)"""
    _check(lib().tclb_part_acc_slots(acc.data_ptr(), int(n6), int(nslots), stream), "particle accumulator copies")


def rigid_step(P, acc, m, free, n: int, a, periodic: int, period, stream: int):
    _check(lib().tclb_part_rigid_step(P.data_ptr(), acc.data_ptr(), m.data_ptr(), free.data_ptr(), n,
                                      float(a[0]), float(a[1]), float(a[2]), periodic,
                                      float(period[0]), float(period[1]), float(period[2]), stream),
           "particle integration")


SNAP_ALLOC_MODES = {"torch": -1, "hip": 0, "contiguous": 1, "vmm": 2}


class _SnapBlock:
    """owner of one tclb_snap_alloc range, exposed through __cuda_array_interface__ (the
    torch tensor made from it keeps this object alive; the range is freed with it)"""

    def __init__(self, nbytes: int, mode: int, device: int):
        p = ctypes.c_void_p()
        _check(lib().tclb_snap_alloc(ctypes.byref(p), nbytes, mode, device), f"snapshot allocation (mode {mode})")
        self.ptr, self.nbytes, self.mode = p.value, nbytes, mode
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 2, "strides": None}

    def __del__(self):
        if self.ptr and _lib is not None:
            _lib.tclb_snap_free(ctypes.c_void_p(self.ptr), self.mode)
            self.ptr = None


def snap_buffer(nbytes: int, mode: str, device):
    """a uint8 device tensor of nbytes from the native snapshot allocator
    (csrc/device/snapalloc.hip): mode "hip" (hipMalloc), "contiguous" (one physically
    contiguous range) or "vmm" (hipMemCreate + a 1 GiB-aligned reservation)"""
    import torch
    m = SNAP_ALLOC_MODES[mode]
    dev = torch.device(device)
    blk = _SnapBlock(int(nbytes), m, dev.index or 0)
    t = torch.as_tensor(blk, device=dev)
    assert t.data_ptr() == blk.ptr and t.numel() == nbytes
    return t


def snap_probe_ms(buf, nf: int, fs: int, reps: int = 2):
    """(read ms, write ms) of the nf field planes (fs elements apart) of snapshot candidate
    `buf` (a device tensor): best of `reps` streaming passes (csrc/device/snapalloc.hip
    tclb_snap_probe); the write pass leaves the planes zero"""
    import torch
    dev = buf.device
    stream = torch.cuda.current_stream(dev).cuda_stream
    sink = torch.zeros(4, dtype=buf.dtype, device=dev)
    es = buf.element_size()
    out = []
    for op in (1, 2):
        best = float("inf")
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _check(lib().tclb_snap_probe(buf.data_ptr(), sink.data_ptr(), fs, fs, nf, es, op, stream),
                   "snapshot probe")
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        out.append(best)
    return out[0], out[1]
