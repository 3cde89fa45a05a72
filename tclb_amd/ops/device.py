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
                if os.path.exists(B.HIPCC):
                    B.build_device_runtime()
                else:
                    raise DeviceRuntimeError(f"device runtime library not usable ({stale}): {path}")
            L = ctypes.CDLL(path)
            P, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
            L.tclb_part_nan_to_zero.argtypes = [P, i, P]
            L.tclb_part_nan_to_zero.restype = i
            L.tclb_part_rigid_step.argtypes = [P, P, P, P, i, d, d, d, i, d, d, d, P]
            L.tclb_part_rigid_step.restype = i
            _lib = L
    return _lib


def _check(r: int, what: str):
    if r != 0:
        raise DeviceRuntimeError(f"{what} failed: HIP error {r}")


def nan_to_zero(t, stream: int):
    """t (contiguous fp64 device tensor): NaN -> 0 in place"""
    _check(lib().tclb_part_nan_to_zero(t.data_ptr(), t.numel(), stream), "particle NaN guard")


def rigid_step(P, acc, m, free, n: int, a, periodic: int, period, stream: int):
    _check(lib().tclb_part_rigid_step(P.data_ptr(), acc.data_ptr(), m.data_ptr(), free.data_ptr(), n,
                                      float(a[0]), float(a[1]), float(a[2]), periodic,
                                      float(period[0]), float(period[1]), float(period[2]), stream),
           "particle integration")
