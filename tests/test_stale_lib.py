"""ops.abi.load never loads a kernel library built from other sources than the current
ones: the <lib>.src stamp (Python model definition + emitter + csrc + compile command)
is compared on every load; a stale library is rebuilt, or rejected under TCLB_NO_BUILD."""
import pytest

from tclb_amd import build as B
from tclb_amd.ops import abi


@pytest.fixture
def fresh(monkeypatch):
    B.build_model("d2q9", kinds=("cpu",))
    monkeypatch.setattr(abi, "_libs", {})
    return monkeypatch


def test_current_library_loads(fresh):
    assert B.stale_reason("d2q9", "cpu") is None
    assert abi.load("d2q9", "cpu").has_iterate


def test_stale_library_rejected_without_build(fresh):
    real = B.source_stamp
    fresh.setattr(B, "source_stamp", lambda *a, **k: real(*a, **k) + "-edited")
    assert B.stale_reason("d2q9", "cpu") == "sources changed since it was built"
    fresh.setenv("TCLB_NO_BUILD", "1")
    with pytest.raises(abi.KernelError, match="sources changed"):
        abi.load("d2q9", "cpu")


def test_stale_library_is_rebuilt(fresh):
    real = B.source_stamp
    fresh.setattr(B, "source_stamp", lambda *a, **k: real(*a, **k) + "-edited")
    calls = []
    fresh.setattr(B, "build_model", lambda name, kinds, variant="": calls.append((name, kinds)))
    abi.load("d2q9", "cpu")
    assert calls == [("d2q9", ("cpu",))]


def test_stamp_ignores_tree_location():
    # the GPU box runs a copy of the tree at another path: same stamp
    s = B._rel_hash([B.__file__], B._PKG + "/x")
    assert s == B._rel_hash([B.__file__], "<pkg>/x")
