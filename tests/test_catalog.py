"""Catalog-wide checks: every registered model builds, initialises and iterates on the CPU
executor with finite results; on a GPU box the HIP kernels must reproduce the CPU
executor (fp64) for every model, and the multi-rank halo path (border/interior split,
pack/exchange/unpack) must reproduce the loopback path."""
import numpy as np
import pytest
import torch

from model_cases import run
from tclb_amd.models import registry
from tclb_amd.parallel.comm import LoopbackComm

MODELS = registry.names()
needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


@pytest.mark.parametrize("name", MODELS)
def test_model_cpu_smoke(name):
    lat = run(name, "cpu", steps=3)
    assert torch.isfinite(lat.fields_interior()).all()
    for q in lat.model.quantities:
        assert torch.isfinite(lat.quantity(q.name)).all(), q.name
    for k, v in lat.globals.items():
        assert np.isfinite(v), k


@pytest.mark.gpu
@needs_gpu
@pytest.mark.parametrize("name", MODELS)
def test_model_hip_matches_cpu(name):
    a = run(name, "cuda", steps=3)
    b = run(name, "cpu", steps=3)
    assert a.lib.kind == "hip"
    fa, fb = a.fields_interior().cpu(), b.fields_interior()
    scale = fb.abs().max().item() + 1e-300
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), (fa - fb).abs().max().item()
    for q in a.model.quantities:
        qa, qb = a.quantity(q.name).cpu(), b.quantity(q.name)
        s = qb.abs().max().item() + 1e-300
        # quantities that are differences of O(1) populations (e.g. forces that vanish in
        # the bulk) carry FMA-contraction noise relative to the populations however small their maximum is
        assert torch.allclose(qa, qb, atol=1e-10 * s + 1e-12 * scale, rtol=1e-10), (q.name, (qa - qb).abs().max().item())


# multi-rank step paths: the native C++ loop (parallel/native.py; on the GPU with the RCCL
# transport sending to this rank itself, or device copies) and the Python step path
# (halo mirror in the border kernels, or separate pack kernels)
DIST_PATHS = {
    "native-rccl": {"TCLB_DIST_NATIVE": "1", "TCLB_DIST_TRANSPORT": "rccl"},
    "native-copy": {"TCLB_DIST_NATIVE": "1", "TCLB_DIST_TRANSPORT": "copy"},
    "native-ipc": {"TCLB_DIST_NATIVE": "1", "TCLB_DIST_TRANSPORT": "ipc"},
    "py-mirror": {"TCLB_DIST_NATIVE": "0", "TCLB_HALO_MIRROR": "1"},
    "py-pack": {"TCLB_DIST_NATIVE": "0", "TCLB_HALO_MIRROR": "0"},
}


def _dist_env(monkeypatch, path):
    for k, v in DIST_PATHS[path].items():
        monkeypatch.setenv(k, v)


def _check_path(lat, path):
    if path.startswith("native"):
        from tclb_amd.parallel.native import NativeDist
        if NativeDist.supported(lat) and lat._native_ok("Iteration"):
            want = path.split("-")[1] if lat.is_gpu else "copy"
            assert lat._dist is not None and lat._dist.transport == want
    else:
        assert lat._dist is None and lat.halo_mirror == (path == "py-mirror")


@pytest.mark.gpu
@needs_gpu
@pytest.mark.parametrize("path", list(DIST_PATHS))
@pytest.mark.parametrize("name", MODELS)
def test_dist_path_on_gpu_matches_loopback(name, path, monkeypatch):
    """the multi-rank step (border/interior split and halo exchange: native loop over RCCL
    self send/receive or device copies; Python path with mirror or pack kernels) equals
    the plain single-rank step bit for bit on the HIP executor, for every catalog model"""
    _dist_env(monkeypatch, path)
    a = run(name, "cuda", steps=4, comm=LoopbackComm(exercise_dist_path=True))
    b = run(name, "cuda", steps=4, comm=LoopbackComm())
    assert a.overlap and not b.overlap
    _check_path(a, path)
    fa, fb = a.fields_interior(), b.fields_interior()
    scale = fb.abs().max().item() + 1e-300
    # bitwise in practice; the tolerance only admits FMA-contraction differences between
    # the range-split launches (none observed)
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), (fa - fb).abs().max().item()


@pytest.mark.parametrize("path", ["native-copy", "py-mirror", "py-pack"])
@pytest.mark.parametrize("name", MODELS)
def test_dist_path_on_cpu_matches_loopback(name, path, monkeypatch):
    """every catalog model: the multi-rank code path with this rank as its own
    neighbour (native loop with the halo plan as copies; Python path with halo mirror or
    pack/unpack) is bitwise equal to the single-rank step.  Regression: a mirror buffer
    shared by both sides when the lo and hi field lists are equal (symmetric stencils)
    broke 38 models."""
    _dist_env(monkeypatch, path)
    a = run(name, "cpu", steps=3, comm=LoopbackComm(exercise_dist_path=True))
    b = run(name, "cpu", steps=3, comm=LoopbackComm())
    assert a.overlap
    _check_path(a, path)
    assert torch.equal(a.fields_interior(), b.fields_interior())


MODELS_3D = [n for n in MODELS if registry.get(n).dims == 3]


@pytest.mark.parametrize("name", MODELS_3D)
def test_grid_path_on_cpu_matches_loopback(name, monkeypatch):
    """the overlapped Y x Z grid step (four border slabs, two-phase z-then-y halo with the
    edge ghosts, interior) with this rank as its own neighbour on both axes
    (TCLB_GRID=1,1) equals the plain single-rank step, for every 3-D model"""
    monkeypatch.setenv("TCLB_GRID", "1,1")
    a = run(name, "cpu", steps=3, comm=LoopbackComm(exercise_dist_path=True))
    monkeypatch.delenv("TCLB_GRID")
    b = run(name, "cpu", steps=3, comm=LoopbackComm())
    assert a.slab.axis == 3 and a.overlap and a.gy > 0 and a.gz > 0
    assert torch.equal(a.fields_interior(), b.fields_interior())


@pytest.mark.gpu
@needs_gpu
@pytest.mark.parametrize("name", MODELS_3D)
def test_grid_path_on_gpu_matches_loopback(name, monkeypatch):
    """GPU twin: the halo phases run on a side stream concurrently with the interior"""
    monkeypatch.setenv("TCLB_GRID", "1,1")
    a = run(name, "cuda", steps=3, comm=LoopbackComm(exercise_dist_path=True))
    monkeypatch.delenv("TCLB_GRID")
    b = run(name, "cuda", steps=3, comm=LoopbackComm())
    assert a.slab.axis == 3 and a.overlap
    fa, fb = a.fields_interior(), b.fields_interior()
    scale = fb.abs().max().item() + 1e-300
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), (fa - fb).abs().max().item()
