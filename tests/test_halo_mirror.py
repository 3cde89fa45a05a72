"""Border kernels that pack their own outgoing halo (Launch.mbase, core.hpp mirror_store):
the overlapped slab step with mirrored stores equals the step with separate pack
kernels and the ghost-free single-rank lattice, bit for bit, on z slabs (3-D) and y
slabs (2-D), multi-stage actions included."""
import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice
from tclb_amd.parallel.comm import LoopbackComm


def _run(model, shape, mode, steps=6, monkeypatch=None):
    if mode == "plain":
        lat = Lattice(model, shape)
    else:
        monkeypatch.setenv("TCLB_HALO_MIRROR", "1" if mode == "mirror" else "0")
        monkeypatch.setenv("TCLB_DIST_NATIVE", "0")       # the Python step path's border kernels
        lat = Lattice(model, shape, comm=LoopbackComm(exercise_dist_path=True), overlap=True)
    m = lat.model
    coll = next(t for t in m.node_types if t.group == "COLLISION")
    fl = np.full((lat.NZ, lat.NY, shape[0]), coll.value, dtype=np.uint32)
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    for s, v in (("GravitationX", 1e-5), ("ForceX", 1e-5), ("AccelX", 1e-5), ("Density_h", 1.0),
                 ("Density_l", 1.0), ("PhaseField", 0.5), ("M", 0.05)):
        if s in lat.gsettings or s in lat.zsettings:
            lat.set_setting(s, v)
    lat.init()
    rng = np.random.default_rng(3)
    f = lat.fields_interior()
    dens = sorted({m.fields.index(d.field) for d in m.densities if not d.field.parameter})
    f[dens] += torch.as_tensor(rng.uniform(0, 1e-3, f[dens].shape), dtype=f.dtype)
    lat.set_fields_interior(f)
    lat.iterate(steps)
    return lat


@pytest.mark.parametrize("model,shape", [("d3q27", (16, 8, 12)), ("d2q9", (16, 24, 1)),
                                         ("d3q19_heat", (8, 8, 10)),
                                         ("d2q9_pf_velocity", (12, 20, 1)), ("d3q27_pf_velocity", (8, 8, 12))])
def test_mirrored_border_equals_pack_and_plain(model, shape, monkeypatch):
    a = _run(model, shape, "plain")
    b = _run(model, shape, "pack", monkeypatch=monkeypatch)
    c = _run(model, shape, "mirror", monkeypatch=monkeypatch)
    assert any(k[0] == "mirror" for k in c._halo_bufs if isinstance(k, tuple) and k and isinstance(k[0], str))
    assert not any(k[0] == "mirror" for k in b._halo_bufs if isinstance(k, tuple) and k and isinstance(k[0], str))
    fa, fb, fc = a.fields_interior(), b.fields_interior(), c.fields_interior()
    assert torch.isfinite(fa).all() and not torch.equal(fa, _run(model, shape, "plain", steps=5).fields_interior())
    assert torch.equal(fa, fb)
    assert torch.equal(fa, fc)
