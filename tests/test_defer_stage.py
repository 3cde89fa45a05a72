"""Deferring split stages (DSL add_stage(split=True, defer=True), executor_hip.hpp
k_stage_defer / k_stage_deferred): the class-1 kernel hands the nodes that need a rare
heavy branch (d3q27_tePSM_per: the CHT interface closure, which depends on the media
field and so moves with the particles) to a third kernel over the queued tiles only.
Every class-1 node must be finished exactly once, by one of the two kernels: the CPU
executor, which runs every node whole, is the oracle.  Cases mix both kinds of node in
one tile and across tiles (a particle, whose coverage turns nodes into the second
medium, and a zone of another MediaNumber), over several steps as the interface forms."""
import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice
from tclb_amd.models import registry
from tclb_amd.models.dsl import Model, ModelError
from tclb_amd.particles import SimplePart

needs_gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


def test_defer_declared():
    for name in ("d3q27_tePSM_per_NEBB", "d3q27_tePSM_per_SUP"):
        st = {s.name: s for s in registry.get(name).stages}["BaseIteration"]
        assert st.split and st.defer
    # isothermal: no CHT closure, nothing to defer
    st = {s.name: s for s in registry.get("d3q27_tePSM_per_NEBB_Isothermal").stages}["BaseIteration"]
    assert st.split and not st.defer


def test_defer_needs_split():
    m = Model("x", dims=2)
    m.add_density("f[0]", 0, 0, 0)
    with pytest.raises(ModelError):
        m.add_stage("S", "Run", save_fields=True, load_densities=True, defer=True)


def test_defer_emitted():
    from tclb_amd.emit.emitter import emit_model
    paths = emit_model(registry.get("d3q27_tePSM_per_NEBB"))
    src = open(paths["header"]).read()
    assert "defer_stage(int s)" in src and "defer_heavy(bool heavy)" in src
    assert "if (!nostore_) save_stage_1();" in src
    # a model without deferring stages: the table, all zero, and no helper
    paths = emit_model(registry.get("d3q27_pf_velocity"))
    src = open(paths["header"]).read()
    assert "defer_stage(int s)" in src and "defer_heavy" not in src


def _case(model, dev, n=(40, 24, 20), steps=4):
    lat = Lattice(model, n, device=torch.device(dev))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, n[0]), m.node_type("BGK").value, dtype=np.uint32)
    lat.add_zone("m2")
    fl[:, :, 26:33] |= 1 << m.zone_shift          # a slab of the second medium
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    for k, v in dict(omegaF=1 / (3 * 0.1 + 0.5), FluidConductivity=0.2, SolidConductivity=0.5, SolidCv=2.0,
                     SolidRho=1.5, AccelX=1e-5, DNx=n[0], DNy=n[1], DNz=n[2], ViscCoeff=0.1).items():
        lat.set_setting(k, v)
    lat.set_setting("InitTemperature", 0.5)
    lat.set_setting("InitTemperature", 1.0, zone="m2")
    lat.set_setting("MediaNumber", 2, zone="m2")
    sp = SimplePart()
    sp.add([11.3, 12.6, 9.8], 4.2, fixed=True)
    lat.particles = sp
    lat.init()
    lat.iterate(steps)
    return lat


@pytest.mark.gpu
@needs_gpu
@pytest.mark.parametrize("model", ["d3q27_tePSM_per_NEBB", "d3q27_tePSM_per_SUP"])
def test_deferred_nodes_match_cpu(model):
    a = _case(model, "cuda")
    b = _case(model, "cpu")
    fa, fb = a.fields_interior().cpu(), b.fields_interior()
    scale = fb.abs().max().item()
    assert torch.allclose(fa, fb, atol=1e-11 * scale, rtol=1e-11), (fa - fb).abs().max().item()
    # the case holds interface nodes (the deferred kernel had work) and plain ones
    mi = a.model.field_index("mediaNum")
    med = fb[mi]
    assert (med == 2).any() and (med == 1).any()
    for q in ("T", "U", "Rho", "Solid"):
        qa, qb = a.quantity(q).cpu(), b.quantity(q)
        s = qb.abs().max().item() + 1e-300
        assert torch.allclose(qa, qb, atol=1e-10 * s, rtol=1e-10), (q, (qa - qb).abs().max().item())
