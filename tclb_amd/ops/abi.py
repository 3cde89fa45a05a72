"""ctypes mirror of ``tclb::Launch`` (csrc/include/tclb/core.hpp) and the per-model
kernel-library loader.

The kernel libraries are plain C-ABI shared objects (no torch headers), loaded after
``import torch`` so that they bind to the HIP runtime torch already loaded (both
share the soname ``libamdhip64.so.7``).  On a GPU box a missing or failing HIP
library is an error — there is no silent fallback to the CPU executor.
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading
from typing import Dict, Optional

import torch  # noqa: F401  (must be imported before loading HIP libraries)

MIRROR_FIELDS = 128     # core.hpp TCLB_MIRROR_FIELDS
GSLOTS = 64             # core.hpp TCLB_GSLOTS: globals accumulate in GSLOTS slots ...


def gstride(ng: int) -> int:
    """... of gstride(NG) doubles each (core.hpp gstride)"""
    return (ng + 15) // 16 * 16


class Launch(ctypes.Structure):
    _fields_ = [
        ("in_", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("flags", ctypes.c_void_p),
        ("settings", ctypes.c_void_p),
        ("zonal", ctypes.c_void_p),
        ("globals_", ctypes.c_void_p),
        ("aux", ctypes.c_void_p),
        ("stream", ctypes.c_void_p),
        ("sy", ctypes.c_longlong),
        ("sz", ctypes.c_longlong),
        ("fs", ctypes.c_longlong),
        ("nx", ctypes.c_int), ("ny", ctypes.c_int), ("nz", ctypes.c_int), ("px", ctypes.c_int),
        ("gy", ctypes.c_int), ("gz", ctypes.c_int),
        ("x0", ctypes.c_int), ("y0", ctypes.c_int), ("z0", ctypes.c_int),
        ("gnx", ctypes.c_int), ("gny", ctypes.c_int), ("gnz", ctypes.c_int),
        ("xlo", ctypes.c_int), ("xhi", ctypes.c_int),
        ("ylo", ctypes.c_int), ("yhi", ctypes.c_int),
        ("zlo", ctypes.c_int), ("zhi", ctypes.c_int),
        ("iter", ctypes.c_int),
        ("nzones", ctypes.c_int),
        ("stage", ctypes.c_int),
        ("glob", ctypes.c_int),
        ("quantity", ctypes.c_int),
        ("qcomp", ctypes.c_int),
        ("qscale", ctypes.c_double),
        ("qsy", ctypes.c_longlong),
        ("qsz", ctypes.c_longlong),
        ("block_x", ctypes.c_int), ("block_y", ctypes.c_int),
        ("reserved0", ctypes.c_int), ("reserved1", ctypes.c_int),
        ("ext", ctypes.c_void_p * 6),
        ("next", ctypes.c_longlong * 6),
        ("time_shift", ctypes.c_double),
        ("storage_shift", ctypes.c_int),
        ("reserved2", ctypes.c_int),
        # halo mirror of the border launches (core.hpp mirror_store)
        ("mbase", ctypes.c_void_p),
        ("mfs", ctypes.c_longlong),
        ("msy", ctypes.c_longlong),
        ("msz", ctypes.c_longlong),
        ("moy", ctypes.c_int),
        ("moz", ctypes.c_int),
        ("mslot", ctypes.c_byte * MIRROR_FIELDS),
        # log2 of the tile windows of the GPU block -> tile map (executor_hip.hpp tile_id)
        ("tile_split", ctypes.c_int),
        # identity of the node types (Lattice.flags_version; executor_hip.hpp class tile lists)
        ("flags_gen", ctypes.c_int),
    ]


# precision name -> (C ABI code of the compute/storage instantiation, shifted storage);
# reference --with-storage=double|float|float-shift|half|half-shift (src/configure.ac:213-233)
PRECISIONS = {
    "double": (0, False),          # fp64 compute, fp64 storage
    "float": (1, False),           # fp32 compute, fp32 storage
    "float-shift": (1, True),      # fp32 compute, fp32 storage of f - w
    "mixed": (2, False),           # fp64 compute, fp32 storage
    "mixed-shift": (2, True),      # fp64 compute, fp32 storage of f - w
    "half": (3, False),            # fp32 compute, fp16 storage
    "half-shift": (3, True),       # fp32 compute, fp16 storage of f - w
}
PREC = {k: v[0] for k, v in PRECISIONS.items()}

SAMPLE_MAXQ = 32


class SamplePlan(ctypes.Structure):
    """mirror of tclb::SamplePlan (csrc/include/tclb/core.hpp)"""
    _fields_ = [
        ("points", ctypes.c_void_p),
        ("out", ctypes.c_void_p),
        ("np", ctypes.c_int), ("width", ctypes.c_int),
        ("row", ctypes.c_int), ("rows", ctypes.c_int),
        ("nq", ctypes.c_int),
        ("q", ctypes.c_int * SAMPLE_MAXQ),
        ("ncomp", ctypes.c_int * SAMPLE_MAXQ),
        ("offset", ctypes.c_int * SAMPLE_MAXQ),
        ("scale", ctypes.c_double * SAMPLE_MAXQ),
    ]


class AdCtx(ctypes.Structure):
    """mirror of tclb::AdCtx (csrc/include/tclb/ad.hpp)"""
    _fields_ = [
        ("aout", ctypes.c_void_p),
        ("ain", ctypes.c_void_p),
        ("gset", ctypes.c_void_p),
        ("gzon", ctypes.c_void_p),
        ("set_mask", ctypes.c_void_p),
        ("zon_mask", ctypes.c_void_p),
        ("obj_weight", ctypes.c_double),
        ("overflow", ctypes.c_int),
        ("reserved", ctypes.c_int),
    ]


ADCTX_OVERFLOW_OFFSET = AdCtx.overflow.offset


class AdLib:
    """the adjoint (AD) executor library of one model: libtclb_<model>_ad.so (CPU) or
    libtclb_<model>_adhip.so (GPU, tclb_ad/executor_ad_hip.hpp)"""

    def __init__(self, model: str, path: str, kind: str = "ad"):
        self.model = model
        self.kind = kind
        self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        self._adj = getattr(self.lib, f"tclb_{model}_adjoint")
        self._adj.argtypes = [ctypes.POINTER(Launch)]
        self._adj.restype = ctypes.c_int
        self.tangents = getattr(self.lib, f"tclb_{model}_ad_tangents")()
        # GPU executor: tangents per pass (TCLB_AD_WINDOW); the CPU executor carries all at once
        win = getattr(self.lib, f"tclb_{model}_ad_window", None)
        self.window = win() if win is not None else self.tangents
        sz = getattr(self.lib, f"tclb_{model}_sizeof_launch")()
        if sz != ctypes.sizeof(Launch):
            raise KernelError(f"ABI mismatch for {path}")

    def run(self, L: Launch):
        r = self._adj(ctypes.byref(L))
        if r != 0:
            raise KernelError(f"{self.model}[ad] stage {L.stage} failed: code {r}")


def load_ad(model: str, gpu: bool = False) -> AdLib:
    from .. import build as B
    kind = "adhip" if gpu else "ad"
    # TCLB_AD_VARIANT: tangent-window build of the GPU executor (build.AD_VARIANTS, A/B only)
    variant = os.environ.get("TCLB_AD_VARIANT", "") if gpu else ""
    key = (model, kind, variant)
    with _lock:
        if key in _libs:
            return _libs[key]
        path = B.lib_path(model, kind, variant)
        stale = B.stale_reason(model, kind, variant)
        if stale is not None:
            if os.environ.get("TCLB_NO_BUILD"):
                raise KernelError(f"adjoint library for model '{model}' [{kind}] is not usable ({stale}): {path}")
            B.build_model(model, kinds=(kind,), variant=variant)
        if not os.path.exists(path):
            raise KernelError(f"adjoint library for model '{model}' [{kind}] not built: {path}")
        lib = AdLib(model, path, kind)
        _libs[key] = lib
        return lib


class KernelError(RuntimeError):
    pass


class ModelLib:
    """Handle on one compiled model library (HIP or CPU)."""

    def __init__(self, model: str, kind: str, path: str):
        self.model = model
        self.kind = kind
        self.path = path
        self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        self._run = getattr(self.lib, f"tclb_{model}_run")
        self._run.argtypes = [ctypes.POINTER(Launch), ctypes.c_int]
        self._run.restype = ctypes.c_int
        self._q = getattr(self.lib, f"tclb_{model}_quantity")
        self._q.argtypes = [ctypes.POINTER(Launch), ctypes.c_int]
        self._q.restype = ctypes.c_int
        sz = getattr(self.lib, f"tclb_{model}_sizeof_launch")()
        if sz != ctypes.sizeof(Launch):
            raise KernelError(f"ABI mismatch for {path}: sizeof(Launch) {sz} != {ctypes.sizeof(Launch)}")
        sp = getattr(self.lib, f"tclb_{model}_sizeof_sample_plan")()
        if sp != ctypes.sizeof(SamplePlan):
            raise KernelError(f"ABI mismatch for {path}: sizeof(SamplePlan) {sp} != {ctypes.sizeof(SamplePlan)}")
        self._it = getattr(self.lib, f"tclb_{model}_iterate")
        self._it.argtypes = [ctypes.POINTER(Launch), ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                             ctypes.c_int, ctypes.c_int, ctypes.POINTER(SamplePlan)]
        self._it.restype = ctypes.c_int
        self._smp = getattr(self.lib, f"tclb_{model}_sample")
        self._smp.argtypes = [ctypes.POINTER(Launch), ctypes.c_int, ctypes.POINTER(SamplePlan)]
        self._smp.restype = ctypes.c_int

    @property
    def has_iterate(self) -> bool:
        return True

    def iterate(self, L: Launch, prec: int, n: int, stages, glob_last: bool, plan: Optional[SamplePlan] = None):
        """n steps of an action in native code (tclb::iterate_action), recording the
        sampler probes of every step when a plan is given"""
        arr = (ctypes.c_int * len(stages))(*stages)
        r = self._it(ctypes.byref(L), prec, n, arr, len(stages), 1 if glob_last else 0,
                     ctypes.byref(plan) if plan is not None else None)
        if r != 0:
            raise KernelError(f"{self.model}[{self.kind}] native iterate failed: code {r}")

    def sample(self, L: Launch, prec: int, plan: SamplePlan):
        r = self._smp(ctypes.byref(L), prec, ctypes.byref(plan))
        if r != 0:
            raise KernelError(f"{self.model}[{self.kind}] sample failed: code {r}")

    def run(self, L: Launch, prec: int):
        r = self._run(ctypes.byref(L), prec)
        if r != 0:
            raise KernelError(f"{self.model}[{self.kind}] stage {L.stage} launch failed: code {r}")

    def quantity(self, L: Launch, prec: int):
        r = self._q(ctypes.byref(L), prec)
        if r != 0:
            raise KernelError(f"{self.model}[{self.kind}] quantity {L.quantity} failed: code {r}")


_libs: Dict[tuple, ModelLib] = {}
_lock = threading.Lock()


def load(model: str, kind: str, build_if_missing: bool = True, variant: Optional[str] = None) -> ModelLib:
    from .. import build as B
    if variant is None:
        variant = B.DEFAULT_VARIANT if kind == "hip" else ""
    key = (model, kind, variant)
    with _lock:
        if key in _libs:
            return _libs[key]
        path = B.lib_path(model, kind, variant)
        # a library built from other sources than the current ones is never loaded
        # silently: rebuild it (hash-stamped, usually seconds) or fail
        stale = "forced" if os.environ.get("TCLB_REBUILD") else B.stale_reason(model, kind, variant)
        if stale is not None:
            if not build_if_missing or os.environ.get("TCLB_NO_BUILD"):
                raise KernelError(f"kernel library for model '{model}' [{kind}] is not usable ({stale}): {path}; "
                                  f"run python -m tclb_amd.build {model}")
            if stale != "missing":
                print(f"[tclb] rebuilding {os.path.basename(path)}: {stale}", file=sys.stderr, flush=True)
            B.build_model(model, kinds=(kind,), variant=variant)
        if not os.path.exists(path):
            raise KernelError(f"kernel library for model '{model}' [{kind}] not built: {path}")
        lib = ModelLib(model, kind, path)
        _libs[key] = lib
        return lib
