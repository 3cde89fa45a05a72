"""<OptSolve> = Solve with ITER_OPT iterations (reference acOptSolve.cpp:5-40,
Lattice::<Action>_Opt src/Lattice.cu.Rt:624-636, Opt() src/cuda.cu.Rt:241-253): each
iteration runs the primal step, one steady-adjoint step (parameter adjoints zeroed on
entry) and moves the design densities on DesignSpace nodes by Descent x adjoint, clamped
to [0, 1]."""
import os
import xml.etree.ElementTree as ET

import numpy as np

from tclb_amd import handlers  # noqa: F401
from tclb_amd.solver import Solver

CASE = """<CLBConfig version="2.0" output="{out}/" permissive="true">
  <Geometry nx="64" ny="24">
    <MRT><Box/></MRT>
    <WVelocity name="Inlet"><Inlet/></WVelocity>
    <EPressure name="Outlet"><Outlet/></EPressure>
    <Inlet nx="1" dx="2"><Box/></Inlet>
    <Outlet nx="1" dx="-2"><Box/></Outlet>
    <Wall mask="ALL"><Channel/></Wall>
    <DesignSpace><Box dx="20" nx="20" dy="4" ny="16"/></DesignSpace>
    <Solid><Box dx="30" nx="1" dy="0" ny="10"/></Solid>
    <None mask="DESIGNSPACE"><Box dx="30" nx="1" dy="0" ny="10"/></None>
  </Geometry>
  <Model>
    <Param name="Velocity" value="0.01"/>
    <Param name="nu" value="0.05"/>
    <Param name="PorocityTheta" value="-3"/>
    <Param name="DragInObj" value="-1.0"/>
  </Model>
  <Param name="Descent" value="{descent}"/>
  {body}
</CLBConfig>"""


def _run(tmp_path, descent, body):
    root = ET.fromstring(CASE.format(out=tmp_path, descent=descent, body=body))
    s = Solver("d2q9_adj", root, conffile=os.path.join(tmp_path, "c.xml"), device="cpu")
    s.run()
    return s


def test_optsolve_moves_design_within_bounds(tmp_path):
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    s0 = _run(tmp_path / "a", 0.0, '<OptSolve Iterations="150"/>')
    s1 = _run(tmp_path / "b", 5.0, '<OptSolve Iterations="150"/>')
    lat0, lat1 = s0.lattice, s1.lattice
    wi = lat1.model.field_index("w")
    w0 = lat0.fields_interior()[wi].numpy()
    w1 = lat1.fields_interior()[wi].numpy()
    ds = (lat1.get_flags() & lat1.model.group_masks["DESIGNSPACE"]) != 0
    assert np.abs(w1 - w0)[ds].max() > 1e-6            # the design moved ...
    assert np.abs(w1 - w0)[~ds].max() == 0.0            # ... only inside the design space
    assert w1.min() >= 0.0 and w1.max() <= 1.0
    # the adjoint state is carried and finite
    assert np.isfinite(s1.opt_state.numpy()).all() and np.abs(s1.opt_state.numpy()).max() > 0


def test_steady_step_parameter_gradient_is_local():
    """the steady step zeroes the parameter adjoint on entry (reference zeropar), so
    two successive steps at a converged state give the same parameter gradient"""
    import torch
    from tclb_amd.adjoint import Adjoint
    from tclb_amd.lattice import Lattice
    lat = Lattice("d2q9_adj", (24, 10, 1))
    m = lat.model
    fl = np.full((1, 10, 24), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, 0, :] = fl[:, 9, :] = m.node_type("Wall").value
    fl[:, 2:8, 8:14] |= m.node_type("DesignSpace").value
    fl[:, 1:9, 18] |= m.node_type("Outlet").value
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    lat.set_setting("nu", 0.1)
    lat.set_setting("ForceX", 1e-5)
    lat.set_setting("OutletFluxInObj", 1.0)
    lat.init()
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    f[wi] = 0.8
    lat.set_fields_interior(f)
    lat.iterate(3000)
    ad = Adjoint(lat)
    a = torch.zeros_like(lat.snaps[lat.cur])
    for _ in range(2000):
        a = ad.steady_step(a)
    g1 = a[wi].clone()
    a = ad.steady_step(a)
    g2 = a[wi]
    assert g1.abs().max() > 0
    assert (g2 - g1).abs().max() <= 1e-8 * g1.abs().max()


def test_optsolve_linearises_at_pre_step_state(tmp_path):
    """advisor r02: the ITER_OPT adjoint step must be taken at the pre-step primal state
    (reference Iteration(tab0 -> tab1) then Iteration_Adj(tab0, ...)), and the design
    update applied to the post-step state"""
    import torch
    from tclb_amd.adjoint import Adjoint
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    s_pre = _run(tmp_path / "a", 5.0, '<Solve Iterations="40"/>')
    s_opt = _run(tmp_path / "b", 5.0, '<Solve Iterations="40"/><OptSolve Iterations="1"/>')
    lat = s_pre.lattice
    pre = lat.snaps[lat.cur].clone()
    ad = Adjoint(lat)
    a = ad.steady_step(torch.zeros_like(pre), state=None)        # linearised at the pre-step state
    lat.iterate(1, glob_last=False)
    post = lat.snaps[lat.cur]
    assert torch.equal(lat.snaps[1 - lat.cur], pre)              # the primal step left its input intact
    assert torch.equal(s_opt.opt_state, a)
    # a linearisation at the post-step state differs (the primal is not converged)
    b = ad.steady_step(torch.zeros_like(pre))
    assert not torch.equal(a, b)
    wi = lat.model.field_index("w")
    ds = (s_opt.lattice.flags.to(torch.int64) & lat.model.group_masks["DESIGNSPACE"]) != 0
    upd = torch.where(ds, (post[wi] + a[wi] * 5.0).clamp(0.0, 1.0), post[wi])
    assert torch.equal(s_opt.lattice.snaps[s_opt.lattice.cur][wi], upd)
