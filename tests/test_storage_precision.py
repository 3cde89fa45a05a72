"""Reduced-precision storage (reference --with-storage=float|float-shift|half|half-shift,
src/configure.ac:213-233, src/LatticeAccess.inc.cpp.Rt:14-35): the *-shift modes store
f_i - w_i, which keeps the precision of the small deviation from rest.  Oracle: the
same force-driven channel in fp64."""
import numpy as np
import pytest
import torch

from tclb_amd.emit.emitter import field_shifts
from tclb_amd.lattice import Lattice
from tclb_amd.models import registry


def _channel(model, precision, shape=(4, 12, 1), force="GravitationX", visc="Viscosity", steps=4000):
    lat = Lattice(model, shape, precision=precision)
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, shape[1] - 1, :] = m.node_type("Wall").value
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    lat.set_setting(visc, 1 / 6)
    lat.set_setting(force, 1e-6)
    lat.init()
    lat.iterate(steps, glob_last=False)
    return lat, lat.quantity("U")[0].double().numpy()


@pytest.fixture(scope="module")
def ref():
    return _channel("d2q9", "double")[1]


def _err(u, ref):
    return np.abs(u - ref).max() / np.abs(ref).max()


def test_shifts_are_lattice_weights():
    m = registry.get("d2q9")
    w = field_shifts(m)
    np.testing.assert_allclose(w[:9], [4 / 9] + [1 / 9] * 4 + [1 / 36] * 4)


def test_mixed_shift_matches_double(ref):
    # steady-state error = storage rounding of the deviation x the slowest mode's
    # relaxation time (1 / nu k^2): ~1e-6 for this 10-node channel, 6000x below plain fp32
    e_shift = _err(_channel("d2q9", "mixed-shift")[1], ref)
    e_plain = _err(_channel("d2q9", "mixed")[1], ref)
    assert e_shift <= 1e-6, e_shift
    assert e_plain > 10 * e_shift, (e_plain, e_shift)


def test_float_shift_stores_deviations(ref):
    # with fp32 compute the arithmetic, not the storage, limits the accuracy
    lat, u = _channel("d2q9", "float-shift", steps=50)
    assert lat.snaps[lat.cur][0, 0, 5, 0].abs() < 1e-6          # f0 - 4/9
    assert abs(lat.fields_interior()[0, 0, 5, 0].item() - 4 / 9) < 1e-6


def test_half_shift_runs_and_beats_half(ref):
    lat, u = _channel("d2q9", "half-shift")
    assert lat.snaps[0].dtype == torch.float16
    e_shift = _err(u, ref)
    e_plain = _err(_channel("d2q9", "half")[1], ref)
    assert e_shift < 0.05, e_shift
    assert e_plain > 3 * e_shift, (e_plain, e_shift)


def test_fields_interior_returns_true_values():
    a, _ = _channel("d2q9", "double", steps=10)
    b, _ = _channel("d2q9", "mixed-shift", steps=10)
    fa = a.fields_interior().double()
    fb = b.fields_interior().double()
    np.testing.assert_allclose(fb.numpy(), fa.numpy(), atol=1e-7)
    # round trip through set_fields_interior keeps the shifted storage consistent
    b.set_fields_interior(fb)
    np.testing.assert_allclose(b.fields_interior().double().numpy(), fb.numpy(), atol=1e-12)
