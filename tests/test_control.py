"""<Control> time series (reference src/Handlers/conControl.cpp): CSV columns sampled per
iteration over the control window, the Time expression, and Param value expressions of
the form ``Column*scale+constant`` (with units)."""
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from tclb_amd import handlers  # noqa: F401
from tclb_amd.handlers.base import HandlerError
from tclb_amd.solver import Solver

CASE = """<CLBConfig version="2.0" output="{out}/">
  <Units>
    <Param name="L" value="0.01m" gauge="1"/>
    <Param name="T" value="1s" gauge="50"/>
    <Param name="rho" value="1kg/m3" gauge="1"/>
  </Units>
  <Geometry nx="24" ny="16"><MRT><Box/></MRT></Geometry>
  <Model>
    <Param name="PDX" value="4"/>
    <Param name="PDY" value="2"/>
    <Control Iterations="2s">
      <CSV file="{csv}" Time="x*2s">
        <Param name="PY" value="Sin*0.03m+0.08m"/>
        <Param name="PR" value="Cos*2+1"/>
      </CSV>
    </Control>
  </Model>
  <Solve Iterations="3"/>
</CLBConfig>"""


def _solver(tmp_path, case=CASE):
    x = np.linspace(0, 1, 9)
    with open(tmp_path / "sin.csv", "w") as f:
        f.write("x,Sin,Cos\n")
        for v in x:
            f.write(f"{v},{np.sin(2 * np.pi * v)},{np.cos(2 * np.pi * v)}\n")
    root = ET.fromstring(case.format(out=tmp_path, csv=tmp_path / "sin.csv"))
    s = Solver("d2q9_plate", root, conffile=os.path.join(tmp_path, "c.xml"), device="cpu")
    s.run()
    return s, x


def test_csv_param_expressions(tmp_path):
    s, x = _solver(tmp_path)
    n = 100                                        # 2 s at 50 iterations per second
    py = s.lattice.zone_series("PY")
    pr = s.lattice.zone_series("PR")
    assert len(py) == n and len(pr) == n
    t = x * n                                      # Time = x * 2 s  (in iterations)
    it = np.arange(n)
    sin_i = np.interp(it, t, np.sin(2 * np.pi * x))
    cos_i = np.interp(it, t, np.cos(2 * np.pi * x))
    # lengths in lattice units: 1 x = 0.01 m
    np.testing.assert_allclose(py, sin_i * 3 + 8, rtol=1e-12)
    np.testing.assert_allclose(pr, cos_i * 2 + 1, rtol=1e-12)
    # the active value follows the iteration (iter % window)
    # the value of the last iteration run stays active (iter % window)
    assert s.lattice.get_setting("PY") == pytest.approx(py[(s.lattice.iter - 1) % n])


def test_unknown_variable_is_an_error(tmp_path):
    bad = CASE.replace("Sin*0.03m+0.08m", "Tan*0.03m")
    with pytest.raises(HandlerError):
        _solver(tmp_path, bad)
