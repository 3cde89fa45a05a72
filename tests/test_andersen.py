"""<Andersen> (reference acAndersen.cpp): Anderson acceleration of the steady state of a
force-driven channel approaches the Poiseuille solution much faster than the same number
of plain iterations (mixing of the stored input states, as the reference)."""
import os
import xml.etree.ElementTree as ET

import numpy as np

from tclb_amd import handlers  # noqa: F401
from tclb_amd.solver import Solver

CASE = """<?xml version="1.0"?>
<CLBConfig version="2.0" output="output/">
  <Geometry nx="4" ny="34">
    <MRT><Box/></MRT>
    <Wall mask="ALL"><Channel/></Wall>
  </Geometry>
  <Model>
    <Param name="Viscosity" value="0.02"/>
    <Param name="GravitationX" value="1e-7"/>
  </Model>
  {body}
</CLBConfig>"""


def _run(tmp_path, body):
    os.chdir(tmp_path)
    s = Solver("d2q9", ET.fromstring(CASE.format(body=body)), conffile=str(tmp_path / "c.xml"), device="cpu")
    s.run()
    return s


def _err(s):
    u = s.lattice.quantity("U").numpy()[0][0, :, 1]
    ny, g, nu = 34, 1e-7, 0.02
    y = np.arange(ny) - 0.5
    ana = g / (2 * nu) * y * (ny - 2 - y)
    return np.abs(u[1:-1] - ana[1:-1]).max() / ana.max()


def test_andersen_accelerates_steady_state(tmp_path):
    acc = _run(tmp_path, '<Andersen Directions="10" Times="24"><Solve Iterations="20"/></Andersen>')
    plain = _run(tmp_path, '<Solve Iterations="960"/>')      # same number of sweeps
    # (the viscous time of the channel is ~ny^2/nu = 58k sweeps; plain is still far off)
    assert _err(acc) < 0.3 * _err(plain), (_err(acc), _err(plain))
