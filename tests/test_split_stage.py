"""Node-class split stages (DSL add_stage(split=True), executor_hip.hpp launch_class): the
GPU runs such a stage as one kernel per node class, each over the tiles that hold nodes of
its class (tile lists found once per node-type identity, Launch.flags_gen).  The lists must
follow every change of the node types, also when a new lattice reuses the freed flag
buffer's address; the CPU executor runs the unsplit stage and is the oracle."""
import numpy as np
import pytest
import torch

from model_cases import make_case, perturb
from tclb_amd.models import registry

needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
SPLIT = ["d3q27_pf_velocity", "d3q27_tePSM_per_NEBB"]


def test_split_declared():
    for name in SPLIT:
        m = registry.get(name)
        assert any(getattr(s, "split", False) for s in m.stages), name
    # BGK builds have no separate interior path: not split
    assert not any(getattr(s, "split", False) for s in registry.get("d3q27_pf_velocity_BGK").stages)


def test_flags_version_unique():
    a = make_case("d2q9", "cpu")
    b = make_case("d2q9", "cpu")
    assert a.flags_version != b.flags_version
    v = a.flags_version
    a.set_flags(a.get_flags())
    assert a.flags_version not in (v, b.flags_version)
    a.iterate(1)
    assert a._L.flags_gen == a.flags_version


def _walls(lat, planes):
    """Wall planes (interior coordinates) added to the current node types"""
    m = lat.model
    nx = lat.shape[0]
    full = lat.flags.cpu().numpy().view(np.uint16 if m.flag_bits == 16 else np.uint32)[:, :, :nx].copy()
    wall = m.node_type("Wall").value
    gz, gy = lat.gz, lat.gy
    for ax, i in planes:
        if ax == "x":
            full[:, :, i] = wall
        elif ax == "y":
            full[:, gy + i, :] = wall
        else:
            full[gz + i, :, :] = wall
    lat.set_flags(full)


def _pair(name, shape, planes1, planes2, steps=2):
    out = []
    for dev in ("cuda", "cpu"):
        lat = make_case(name, dev, shape=shape)
        _walls(lat, planes1)
        lat.init()
        perturb(lat)
        lat.iterate(steps)
        _walls(lat, planes2)            # new node types: the class lists must follow
        lat.iterate(steps)
        out.append(lat.fields_interior().cpu().double())
    return out


@pytest.mark.gpu
@needs_gpu
@pytest.mark.parametrize("name", SPLIT)
def test_split_follows_flag_changes(name):
    # 130 x 40 x 20: several x tiles, one of them partial; walls added in the second half
    fa, fb = _pair(name, (130, 40, 20), [("x", 0)], [("x", 0), ("y", 17), ("z", 9), ("x", 129)])
    scale = fb.abs().max().item()
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), (fa - fb).abs().max().item()


@pytest.mark.gpu
@needs_gpu
def test_split_reused_flag_buffer():
    """a lattice of the same shape created after another was freed (the caching allocator
    hands back the same flag buffer): its node types are new, the lists too"""
    name = "d3q27_pf_velocity"
    shape = (64, 24, 12)
    lat = make_case(name, "cuda", shape=shape)
    _walls(lat, [("y", 5)])
    lat.init()
    lat.iterate(1)
    ptr = lat.flags.data_ptr()
    del lat
    res = []
    for dev in ("cuda", "cpu"):
        lat = make_case(name, dev, shape=shape)
        _walls(lat, [("x", 3), ("z", 7)])
        lat.init()
        perturb(lat)
        lat.iterate(3)
        if dev == "cuda":
            reused = lat.flags.data_ptr() == ptr
        res.append(lat.fields_interior().cpu().double())
    fa, fb = res
    scale = fb.abs().max().item()
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), ((fa - fb).abs().max().item(), reused)


@pytest.mark.gpu
@needs_gpu
def test_thermo_nonlocaltemp_adiabatic_nodes():
    """pf_velocity_thermo's NonLocalTemp is split with class 0 (no work) for every node but
    the EAdiabatic ones; a plane of those must come out as on the CPU, which runs the
    stage on every node"""
    name = "d3q27_pf_velocity_thermo"
    out = []
    for dev in ("cuda", "cpu"):
        lat = make_case(name, dev, shape=(40, 16, 12))
        m = lat.model
        nx = lat.shape[0]
        full = lat.flags.cpu().numpy().view(np.uint16 if m.flag_bits == 16 else np.uint32)[:, :, :nx].copy()
        full[:, :, 20] |= m.node_type("EAdiabatic").value
        lat.set_flags(full)
        lat.init()
        perturb(lat)
        lat.iterate(3)
        out.append(lat.fields_interior().cpu().double())
    fa, fb = out
    scale = fb.abs().max().item()
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), (fa - fb).abs().max().item()


@pytest.mark.gpu
@needs_gpu
def test_thermo_parabolic_surface_tension():
    """surfPower > 1 takes the out-of-line power law (d3q27_pf_velocity.inc pow_cold_, a
    real call in the GPU kernels): GPU equals CPU"""
    name = "d3q27_pf_velocity_thermo"
    out = []
    for dev in ("cuda", "cpu"):
        lat = make_case(name, dev, shape=(32, 16, 12))
        lat.set_setting("surfPower", 2.0)
        lat.set_setting("sigma_TT", 1e-4)
        lat.set_setting("T_ref", 0.5)
        lat.init()
        perturb(lat)
        lat.iterate(3)
        out.append(lat.fields_interior().cpu().double())
    fa, fb = out
    scale = fb.abs().max().item()
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), (fa - fb).abs().max().item()
