"""<Sample> probes (reference src/Handlers/cbSample.cpp, src/Sampler.cpp): one CSV row per
iteration and point, recorded on the device every iteration (native multi-step loop or
Python per-step path) and flushed at the callback."""
import csv
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from tclb_amd import handlers  # noqa: F401
from tclb_amd.lattice import Lattice
from tclb_amd.sampler import Sampler
from tclb_amd.solver import Solver

CASE = """<CLBConfig version="2.0" output="{out}/">
  <Geometry nx="32" ny="16"><MRT><Box/></MRT><Wall mask="ALL"><Channel/></Wall></Geometry>
  <Model><Param name="Viscosity" value="0.1"/><Param name="GravitationX" value="1e-5"/></Model>
  <Sample Iterations="10" what="U,Rho">
    <Point dx="5" dy="8"/>
    <Point dx="20" dy="3"/>
  </Sample>
  <Solve Iterations="25"/>
</CLBConfig>"""


def _run(tmp_path, native):
    os.environ["TCLB_NATIVE_LOOP"] = "1" if native else "0"
    try:
        root = ET.fromstring(CASE.format(out=tmp_path))
        s = Solver("d2q9", root, conffile=os.path.join(tmp_path, "c.xml"), device="cpu")
        s.run()
    finally:
        os.environ.pop("TCLB_NATIVE_LOOP", None)
    fn = [f for f in os.listdir(tmp_path) if "Sampler" in f and f.endswith(".csv")]
    assert len(fn) == 1
    with open(tmp_path / fn[0]) as f:
        rows = list(csv.reader(f))
    return s, rows


@pytest.mark.parametrize("native", [True, False])
def test_one_row_per_iteration_and_point(tmp_path, native):
    s, rows = _run(tmp_path, native)
    assert rows[0] == ["Iteration", "X", "Y", "Z", "Rho", "U.x", "U.y", "U.z"]
    body = rows[1:]
    assert len(body) == 25 * 2
    its = [int(r[0]) for r in body]
    assert its == sorted(its) and its[0] == 1 and its[-1] == 25
    # the last row of point 1 is the state at the end of the run
    last = [r for r in body if int(r[0]) == 25 and r[1:4] == ["20", "3", "0"]][0]
    u = s.lattice.quantity("U")[:, 0, 3, 20].numpy()
    np.testing.assert_allclose([float(v) for v in last[5:8]], u, rtol=1e-12, atol=1e-300)


def test_native_and_python_paths_agree(tmp_path):
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    _, ra = _run(tmp_path / "a", True)
    _, rb = _run(tmp_path / "b", False)
    assert ra == rb


def test_sampler_matches_full_quantity_each_step():
    lat = Lattice("d2q9", (24, 12, 1))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, 24), m.node_type("MRT").value, dtype=np.uint16)
    lat.set_flags(fl)
    lat.set_setting("Viscosity", 0.1)
    lat.set_setting("VelocityX", 0.02)
    lat.init()
    lat.snaps[lat.cur][:, 0, :, :24] += 1e-3 * __import__("torch").rand(lat.nf, lat.NY, 24, dtype=lat.sdtype)
    smp = Sampler(lat, [(3, 4, 0), (23, 11, 0)], ["Rho", "U"], rows=2)
    lat.samplers.append(smp)
    ref = []
    for _ in range(5):
        lat.iterate(1)
        ref.append((lat.quantity("Rho")[0, 0].numpy().copy(), lat.quantity("U")[:, 0].numpy().copy()))
    rows = smp.flush()
    assert len(rows) == 10 and smp.plan.rows >= 5      # the buffer grew past its 2 rows
    for it, i, (x, y, z), v in rows:
        rho, u = ref[it - 1]
        np.testing.assert_allclose(v, [rho[y, x], *u[:, y, x]], rtol=1e-13)
