"""Shan-Chen pseudopotential: a liquid drop in its vapour stays coexisting (density ratio
kept, mass conserved) — the reference's example/multiphase/SchanChen/d2q9_sc.xml case,
shrunk; and the two-stage Iteration action machinery (psi stage) runs on CPU."""
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from tclb_amd import handlers  # noqa: F401
from tclb_amd.solver import Solver

CASE = """<CLBConfig output="output/" permissive="true">
  <Geometry nx="48" ny="48">
    <MRT><Box/></MRT>
    <None name="blobb"><Sphere ny="20" nx="20" dx="14" dy="14"/></None>
  </Geometry>
  <Model>
    <Param name="Density" value="0.056"/>
    <Param name="Density" value="2.659" zone="blobb"/>
    <Param name="G_ff" value="-6.0"/>
    <Param name="viscosity" value="0.166"/>
  </Model>
  <Solve Iterations="600"/>
</CLBConfig>"""


def test_shanchen_drop(tmp_path):
    os.chdir(tmp_path)
    s = Solver("d2q9_ShanChen", ET.fromstring(CASE), conffile="sc.xml", device="cpu")
    s.read_units()
    s.set_size()
    from tclb_amd.handlers.base import make_handler
    lat = s.lattice
    root = make_handler(s.config_tree, s)
    rho = lat.quantity("Rho").numpy()[0, 0]
    assert np.isfinite(rho).all()
    assert rho[24, 24] > 1.5 and rho[2, 2] < 0.3      # liquid inside, vapour outside
    f = lat.fields_interior().numpy()
    mass = f[:9].sum()
    lat.iterate(50)
    assert abs(lat.fields_interior().numpy()[:9].sum() - mass) / mass < 1e-10
    psi = lat.quantity("Psi").numpy()[0, 0]
    assert np.isfinite(psi).all() and 0 < psi.min() and psi.max() < 1
