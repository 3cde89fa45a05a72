"""The native action loop (tclb_rt/dist_loop.hpp action_loop, parallel/native.py) steps
every kind of action the Python step path steps — particle stages with the in-process
SimplePart integrator (grid / tree / scan solid containers), out-of-place stages that read
a field they write, fixed-point stages, zonal time series (including an Objective weight),
several samplers, the Y x Z grid — and gives the same result bit for bit.  Reference: the
C++ Lattice::Iterate does all of this per rank (src/Lattice.cu.Rt:392-437,466-533,473-477,
484,1376-1389)."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from model_cases import make_case, perturb  # noqa: E402

from tclb_amd.lattice import Lattice  # noqa: E402
from tclb_amd.parallel.comm import LoopbackComm  # noqa: E402
from tclb_amd.particles import SimplePart  # noqa: E402
from tclb_amd.sampler import Sampler  # noqa: E402

needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


def _psm_case(device, native, nparts=20, series=False, samplers=0, n=16):
    lat = Lattice("d3q27_PSM_NEBB", (n, n, n), device=torch.device(device), native_loop=native)
    lat.set_flags(np.full((lat.NZ, lat.NY, n), lat.model.node_type("BGK").value, dtype=np.uint32))
    lat.set_setting("nu", 0.1)
    lat.set_setting("aX_mean", 1e-5)
    if series:
        lat.set_zone_series("aX_mean", [1e-5, 3e-5, -2e-5, 0.0, 5e-6])
        lat.set_zone_series("TotalFluidMassInObj", [0.0, 1.0, 0.0])
    sp = SimplePart()
    rng = np.random.default_rng(3)
    for i in range(nparts):
        sp.add(rng.uniform(2, n - 2, 3), rng.uniform(0.8, 1.6), v=rng.uniform(-0.01, 0.01, 3), m=rng.uniform(5, 20))
    sp.acc = np.array([1e-6, 0.0, -2e-6])
    sp.periodic[:] = True
    sp.period[:] = n
    lat.particles = sp
    for k in range(samplers):
        lat.samplers.append(Sampler(lat, [(1 + k, 2, 3), (5, 5 + k, 7)], ["U", "Rho"], rows=4))
    lat.init()
    return lat, sp


def _compare(a, b, pa=None, pb=None):
    """bit for bit; with particles to rounding: the particle stage sums each particle's
    force over its nodes with atomics (OpenMP threads, GPU waves), in no fixed order, so
    two runs of the same path already differ in the last bits"""
    fa, fb = a.fields_interior().cpu(), b.fields_interior().cpu()
    if pa is None:
        assert torch.equal(fa, fb)
    else:
        assert torch.allclose(fa, fb, rtol=1e-12, atol=1e-15), (fa - fb).abs().max().item()
    assert a.iter == b.iter and a.cur == b.cur
    for k in a.globals:
        ga, gb = a.globals[k], b.globals[k]
        # globals: per-thread partial sums merged in thread order (executor_cpu.hpp)
        assert abs(ga - gb) <= 1e-12 * abs(gb) + 1e-15 or (np.isnan(ga) and np.isnan(gb)), k
    if pa is not None:
        for name in ("x", "v", "omega", "force", "torque"):
            assert np.allclose(getattr(pa, name), getattr(pb, name), rtol=1e-11, atol=1e-15), name
        assert pa.iteration == pb.iteration


@pytest.mark.parametrize("container", ["grid", "tree", "all"])
def test_particles_native_equals_python(monkeypatch, container):
    """SimplePart particles moving through a PSM lattice: zero / container build / stage /
    NaN guard / rigid step in the loop = the Python hooks"""
    monkeypatch.setenv("TCLB_SOLID_CONTAINER", container)
    a, pa = _psm_case("cpu", True)
    b, pb = _psm_case("cpu", False)
    assert a._native_path("Iteration") == "loop" and b._native_path("Iteration") is None
    for _ in range(2):
        a.iterate(3)
        b.iterate(3)
    _compare(a, b, pa, pb)
    assert a._dist is not None and np.abs(pa.force).max() > 0


def test_series_and_samplers_native_equals_python():
    """zonal time series (a body force and an Objective weight) and two samplers"""
    a, pa = _psm_case("cpu", True, nparts=3, series=True, samplers=2)
    b, pb = _psm_case("cpu", False, nparts=3, series=True, samplers=2)
    a.iterate(4)
    b.iterate(4)
    a.iterate(3)
    b.iterate(3)
    _compare(a, b, pa, pb)
    for sa, sb in zip(a.samplers, b.samplers):
        assert sa.row == sb.row == 7
        assert torch.equal(sa.buf[:7].cpu(), sb.buf[:7].cpu())
    # the host zonal table follows the device after a native call (entries of the last step)
    assert np.array_equal(a.zvals, b.zvals)
    assert a.globals["TotalFluidMass"] != 0.0


@pytest.mark.parametrize("name", ["d2q9_scmp_Kupershtokh_VirtualRhoWBC_ViscositySmooth_CUM", "d2q9_csf"])
def test_out_of_place_and_fixed_point_native_equals_python(name):
    """a stage that reads a field it writes (run out of place) and d2q9_csf's fixed-point
    wall-normal stage (100 Jacobi sweeps, in Init)"""
    out = []
    for native in (True, False):
        lat = make_case(name)
        lat.native_loop = native
        lat.init()
        perturb(lat)
        lat.iterate(3)
        out.append(lat)
    assert out[0]._dist is not None
    _compare(out[0], out[1])


@pytest.mark.parametrize("model", ["d3q27", "d3q27_pf_velocity_thermo"])
def test_grid_loopback_native_equals_python(monkeypatch, model):
    """one rank through the Y x Z grid path (two-phase halo: z planes, then packed y rows
    over the ghost-inclusive z extent) as its own neighbour"""
    out = []
    for native in ("1", "0"):
        monkeypatch.setenv("TCLB_DIST_NATIVE", native)
        lat = make_case(model, shape=(16, 12, 10), comm=LoopbackComm(exercise_dist_path=True), grid=(1, 1))
        lat.init()
        perturb(lat)
        lat.iterate(3)
        out.append(lat)
    assert out[0].slab.axis == 3 and out[0]._dist is not None and out[1]._dist is None
    _compare(out[0], out[1])


@pytest.mark.gpu
@needs_gpu
@pytest.mark.parametrize("container", ["grid", "tree"])
def test_particles_native_gpu_equals_python_gpu(monkeypatch, container):
    """on the GPU: the device container builds (hipcub radix sort), the particle hooks and
    the rigid step inside the loop = the Python hooks, bit for bit; and the CPU within
    rounding"""
    monkeypatch.setenv("TCLB_SOLID_CONTAINER", container)
    a, pa = _psm_case("cuda", True, series=True, samplers=2)
    b, pb = _psm_case("cuda", False, series=True, samplers=2)
    c, pc = _psm_case("cpu", True, series=True, samplers=2)
    for lat in (a, b, c):
        lat.iterate(5)
    _compare(a, b, pa, pb)
    assert torch.allclose(a.fields_interior().cpu(), c.fields_interior(), rtol=1e-11, atol=1e-13)
    assert np.allclose(pa.x, pc.x, rtol=1e-11, atol=1e-12)


@pytest.mark.gpu
@needs_gpu
@pytest.mark.parametrize("name", ["d2q9_scmp_Kupershtokh_VirtualRhoWBC_ViscositySmooth_CUM", "d2q9_csf"])
def test_special_stages_native_gpu_equals_python_gpu(name):
    out = []
    for native in (True, False):
        lat = make_case(name, "cuda")
        lat.native_loop = native
        lat.init()
        perturb(lat)
        lat.iterate(3)
        out.append(lat)
    _compare(out[0], out[1])
