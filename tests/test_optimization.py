"""Adjoint / optimisation XML handlers (tclb_amd/handlers/optimization.py; reference
src/Handlers/acUSAdjoint.cpp, acFDTest.cpp, acOptimize.cpp.Rt, InternalTopology.cpp,
OptimalControl.cpp) on the topology-optimisation model d2q9_adj: the FDTest handler's
adjoint gradients must agree with its own central finite differences, and a few
optimiser evaluations must not decrease the objective."""
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from tclb_amd import handlers  # noqa: F401
from tclb_amd.solver import Solver

CASE = """<?xml version="1.0"?>
<CLBConfig version="2.0" output="output/">
  <Geometry nx="24" ny="10">
    <MRT><Box/></MRT>
    <WVelocity><Box nx="1"/></WVelocity>
    <EPressure><Box dx="-1"/></EPressure>
    <Inlet><Box dx="2" nx="1"/></Inlet>
    <Outlet><Box dx="-3" nx="1"/></Outlet>
    <DesignSpace name="des"><Box dx="8" nx="6" dy="2" ny="6"/></DesignSpace>
    <Wall mask="ALL"><Channel/></Wall>
  </Geometry>
  <Model>
    <Param name="Velocity" value="0.01"/>
    <Param name="nu" value="0.1"/>
    <Param name="PorocityTheta" value="-2"/>
    <Param name="Porocity" value="0.4" zone="des"/>
    <Param name="PressureLossInObj" value="-1"/>
    <Param name="MaterialPenaltyInObj" value="-0.0001"/>
  </Model>
  {design}
  {body}
</CLBConfig>"""


def run(tmp_path, design, body):
    os.chdir(tmp_path)
    root = ET.fromstring(CASE.format(design=design, body=body))
    s = Solver("d2q9_adj", root, conffile=str(tmp_path / "case.xml"), device="cpu")
    s.run()
    return s


def test_fdtest_topology(tmp_path):
    s = run(tmp_path, "<InternalTopology/>",
            '<FDTest parameters="3:5" h="1e-5"><Adjoint type="unsteady"><Solve Iterations="20"/></Adjoint></FDTest>')
    assert len(s.fdtest) == 3
    for i, adj, fd in s.fdtest:
        assert abs(adj - fd) <= 1e-5 * abs(fd) + 1e-12, (i, adj, fd)
        assert abs(fd) > 0


def test_fdtest_control_setting(tmp_path):
    s = run(tmp_path, '<OptimalControl what="ForceX"/>',
            '<FDTest order="4" h="1e-6"><Adjoint type="unsteady"><Solve Iterations="15"/></Adjoint></FDTest>')
    (_, adj, fd), = s.fdtest
    assert abs(adj - fd) <= 1e-6 * abs(fd) + 1e-12, (adj, fd)


def test_optimize_improves_objective(tmp_path):
    s = run(tmp_path, "<InternalTopology/>",
            '<Optimize MaxEvaluations="4" Method="MMA"><Adjoint type="unsteady"><Solve Iterations="10"/></Adjoint></Optimize>'
            '<Threshold Level="0.5"/>')
    best, x = s.optimum
    assert np.isfinite(best) and best >= s.opt_history[0] and len(s.opt_history) >= 2
    assert x.size == 36 and ((x >= 0) & (x <= 1)).all()
    w = s.lattice.fields_interior()[s.model.field_index("w")].numpy()
    des = w[0, 2:8, 8:14]
    assert set(np.unique(des)).issubset({0.0, 1.0})


def _control_case(tmp_path, design):
    """inlet velocity as a zonal time series over a 16-iteration control window"""
    with open(tmp_path / "inlet.csv", "w") as f:
        f.write("Time,Velocity\n0,0.005\n16,0.015\n")
    body = ('<Control Iterations="16"><CSV file="inlet.csv" Time="Time"/></Control>'
            f'{design}'
            '<FDTest order="4" h="1e-6"><Adjoint type="unsteady"><Solve Iterations="16"/></Adjoint></FDTest>')
    return run(tmp_path, "", body)


def test_time_series_optimal_control_gradient(tmp_path):
    """OptimalControl of a zonal time series (reference OptimalControl.cpp over
    zSet.getLen entries): per-time-index adjoint gradients equal finite differences"""
    s = _control_case(tmp_path, '<OptimalControl what="Velocity" lower="0" upper="0.05"/>')
    assert len(s.fdtest) == 16
    for i, adj, fd in s.fdtest:
        assert abs(adj - fd) <= 1e-6 * max(abs(fd), 1e-8) + 1e-11, (i, adj, fd)   # FD round-off ~1e-12
    assert any(abs(fd) > 0 for _, _, fd in s.fdtest)


@pytest.mark.parametrize("design", ['<BSpline nodes="4"><OptimalControl what="Velocity"/></BSpline>',
                                    '<Fourier modes="3"><OptimalControl what="Velocity"/></Fourier>',
                                    '<RepeatControl length="4"><OptimalControl what="Velocity"/></RepeatControl>',
                                    '<OptimalControlSecond what="Velocity"/>'])
def test_reduced_controls_gradient(tmp_path, design):
    """BSpline / Fourier / RepeatControl / OptimalControlSecond re-parameterise the series;
    their chain-ruled adjoint gradients equal finite differences in their own parameters"""
    s = _control_case(tmp_path, design)
    assert len(s.fdtest) >= 3
    for i, adj, fd in s.fdtest:
        assert abs(adj - fd) <= 1e-6 * max(abs(fd), 1e-8) + 1e-11, (i, adj, fd)   # FD round-off ~1e-12


def test_extrude_topology_gradient(tmp_path):
    """Extrude (reference conExtrude.cpp): one smooth front per design line along x; the
    chain-ruled adjoint gradient equals finite differences of the front positions"""
    s = run(tmp_path, '<Extrude direction="x" theta="1.5"><InternalTopology/></Extrude>',
            '<FDTest h="1e-5" order="4"><Adjoint type="unsteady"><Solve Iterations="20"/></Adjoint></FDTest>')
    assert len(s.fdtest) == 6              # 6 lines (y = 2..7) through the 6x6 design box
    for i, adj, fd in s.fdtest:
        assert abs(adj - fd) <= 1e-5 * abs(fd) + 1e-12, (i, adj, fd)
        assert abs(fd) > 0


@pytest.mark.parametrize("method", ["MMA", "LBFGS", "COBYLA", "NELDERMEAD"])
def test_optimize_methods_and_material_constraint(tmp_path, method):
    """reference attribute ``method`` (NLopt names) and Material="less": the design's total
    material may not grow (tolerance 1e-3, as NLopt's inequality constraint)"""
    s = run(tmp_path, "<InternalTopology/>",
            f'<Optimize MaxEvaluations="6" method="{method}" Material="less">'
            '<Adjoint type="unsteady"><Solve Iterations="6"/></Adjoint></Optimize>')
    best, x = s.optimum
    assert np.isfinite(best) and len(s.opt_history) >= 1
    x0_sum = 36 * 1.0          # InternalTopology starts fully fluid (w = 1)
    assert x.sum() <= x0_sum + 1e-3 + 1e-9
    if method in ("MMA", "LBFGS"):
        assert best >= s.opt_history[0] - 1e-12
