"""roctx ranges around actions, stages, halo exchanges and global reductions (reference
NVTX ranges, src/Lattice.cu.Rt:22-29 and 468-525), seen by
``rocprofv3 --marker-trace``.  Enabled with TCLB_ROCTX=1; otherwise every call is a
no-op with no library load and negligible cost.

Also the per-launch synchronisation debug mode (reference CROSS_SYNC,
src/configure.ac:827-837): TCLB_SYNC=1 makes every stage launch wait for the device
and check for errors, so a faulting kernel is named at its launch.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional

_LIB: Optional[ctypes.CDLL] = None
ENABLED = os.environ.get("TCLB_ROCTX", "0") not in ("", "0")
SYNC = os.environ.get("TCLB_SYNC", "0") not in ("", "0")


def _lib() -> Optional[ctypes.CDLL]:
    global _LIB, ENABLED
    if _LIB is None and ENABLED:
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"):
            for d in ("/opt/rocm/lib", ""):
                try:
                    _LIB = ctypes.CDLL(os.path.join(d, name) if d else name)
                    break
                except OSError:
                    continue
            if _LIB is not None:
                break
        if _LIB is None:
            ENABLED = False
        else:
            _LIB.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _LIB.roctxRangePushA.restype = ctypes.c_int
            _LIB.roctxRangePop.restype = ctypes.c_int
    return _LIB


def push(name: str):
    if ENABLED and _lib() is not None:
        _LIB.roctxRangePushA(name.encode())


def pop():
    if ENABLED and _LIB is not None:
        _LIB.roctxRangePop()


@contextlib.contextmanager
def span(name: str):
    if not ENABLED:
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()


def after_launch(lat, what: str):
    """TCLB_SYNC=1: synchronise and surface a device error right after a launch"""
    if SYNC and lat.is_gpu:
        import torch
        try:
            torch.cuda.synchronize(lat.device)
        except RuntimeError as e:
            raise RuntimeError(f"device error after {what} (iteration {lat.iter}): {e}") from e
