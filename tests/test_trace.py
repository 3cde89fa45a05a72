"""roctx ranges (reference NVTX ranges, src/Lattice.cu.Rt:22-29,468-525): every pushed
range is popped, names follow action / stage; the roctx library itself loads."""
import numpy as np

from tclb_amd.lattice import Lattice
from tclb_amd.utils import trace


def test_ranges_balanced_and_named(monkeypatch):
    stack, seen = [], []
    monkeypatch.setattr(trace, "ENABLED", True)
    monkeypatch.setattr(trace, "push", lambda n: (stack.append(n), seen.append(n)))
    monkeypatch.setattr(trace, "pop", lambda: stack.pop())
    lat = Lattice("d2q9", (16, 8, 1), native_loop=False)
    lat.set_flags(np.full((lat.NZ, lat.NY, 16), lat.model.node_type("MRT").value, dtype=np.uint16))
    lat.init()
    lat.iterate(2)
    assert stack == []
    assert "action Iteration" in seen and "stage BaseIteration" in seen and "action Init" in seen


def test_roctx_library_loads(monkeypatch):
    monkeypatch.setattr(trace, "ENABLED", True)
    monkeypatch.setattr(trace, "_LIB", None)
    lib = trace._lib()
    if lib is not None:                        # absent ROCm: ranges silently disabled
        trace.push("x")
        trace.pop()
