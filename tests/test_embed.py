"""Embedded Python with the reference's ``Solver`` object model (handlers/embed.py;
reference src/Handlers/cbRunR.cpp:67-516 and its reticulate face :687-760):

* a Python port of example/runr/spheres.xml — geometry editing through
  ``Solver.Geometry.X/Y`` and ``Solver.Geometry.BOUNDARY/COLLISION`` assignment, then a
  per-node parameter field written through ``Solver.Fields`` — runs and changes the case;
* the ``Solver.*`` part of example/python/karman_vtk.xml (without vtk): the
  ``Solver.Geometry.X`` shape and ``for n, tab in Solver.Quantities`` give the lattice's
  quantities in the reference (nx, ny, nz) order, lattice and SI units;
* Settings / Globals / Actions / Info, one namespace shared by all blocks, and a clear
  error for names that do not exist."""
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from tclb_amd import handlers  # noqa: F401
from tclb_amd.solver import Solver

SPHERES = """<CLBConfig version="2.0" output="{out}/" permissive="true">
  <Geometry nx="96" ny="48"><MRT><Box/></MRT></Geometry>
  <RunPython>
    rad = 6
    tab = [(30.0, 20.0), (60.0, 30.0)]
    X = Solver.Geometry.X
    Y = Solver.Geometry.Y
    sel = np.zeros(X.shape, dtype=bool)
    for (cx, cy) in tab:
        R = np.sqrt((X - cx) ** 2 + (Y - cy) ** 2)
        sel |= rad > R
    b = Solver.Geometry.BOUNDARY
    b = np.where(sel, "Wall", np.array(Solver.Geometry.levels("BOUNDARY"))[b])
    Solver.Geometry.BOUNDARY = b
    c = Solver.Geometry.COLLISION
    c[sel] = 0
    Solver.Geometry.COLLISION = c
  </RunPython>
  <Model>
    <Param name="nu" value="0.05"/>
    <Param name="ForceX" value="1e-5"/>
  </Model>
  <RunPython>
    w = np.ones(X.shape)
    for (cx, cy) in tab:
        R = np.sqrt((X - cx) ** 2 + (Y - cy) ** 2)
        w = np.minimum(w, np.clip((R - rad) / 4.0, 0.0, 1.0))
    Solver.Fields.w = w
    seen = dict(Solver.Settings)
  </RunPython>
  <RunPython Iterations="10">
    hist.append((Solver.Globals.Iteration, Solver.Globals.Drag))
  </RunPython>
  <Solve Iterations="30"/>
</CLBConfig>"""


def _solver(tmp_path, xml, model):
    root = ET.fromstring(xml.format(out=tmp_path))
    return Solver(model, root, conffile=os.path.join(tmp_path, "case.xml"), device="cpu")


def test_spheres_port_edits_geometry_and_field(tmp_path):
    xml = SPHERES.replace("<RunPython Iterations=\"10\">", "<RunPython>hist = []</RunPython>\n  <RunPython Iterations=\"10\">")
    s = _solver(tmp_path, xml, "d2q9_adj")
    s.run()
    lat = s.lattice
    m = lat.model
    fl = lat.get_flags()[0]                      # (ny, nx)
    wall = m.node_type("Wall").value
    bmask, cmask = m.group_masks["BOUNDARY"], m.group_masks["COLLISION"]
    assert (fl[20, 30] & bmask) == wall and (fl[20, 30] & cmask) == 0
    assert (fl[30, 60] & bmask) == wall
    assert (fl[5, 5] & bmask) == 0 and (fl[5, 5] & cmask) == m.node_type("MRT").value
    w = lat.field("w").numpy()[0]
    assert w[20, 30] == 0.0 and w[5, 5] == 1.0 and 0.0 < w[20, 38] < 1.0
    ns = s._embed_ns
    assert ns["seen"]["nu"] == pytest.approx(0.05)
    assert [h[0] for h in ns["hist"]] == [10, 20, 30]
    assert all(np.isfinite(h[1]) for h in ns["hist"])


KARMAN = """<CLBConfig version="2.0" output="{out}/" permissive="true">
  <Units><Param value="0.001m" gauge="1"/></Units>
  <Geometry nx="64" ny="20">
    <MRT><Box/></MRT>
    <WVelocity name="Inlet"><Inlet/></WVelocity>
    <EPressure name="Outlet"><Outlet/></EPressure>
    <Wall mask="ALL"><Channel/><Wedge dx="20" nx="6" dy="8" ny="6" direction="LowerRight"/></Wall>
  </Geometry>
  <Model>
    <Param name="VelocityX" value="0.01"/>
    <Param name="Viscosity" value="0.02"/>
  </Model>
  <RunPython>
import json
  </RunPython>
  <RunPython Iterations="20">
tab = Solver.Geometry.X
shape = (tab.shape[0] + 1, tab.shape[1] + 1, tab.shape[2] + 1)
arrays = {{}}
for n, tab in Solver.Quantities:
    arrays[n] = tab
json.dumps(list(arrays))
  </RunPython>
  <Solve Iterations="40"/>
</CLBConfig>"""


def test_karman_vtk_solver_part(tmp_path):
    s = _solver(tmp_path, KARMAN, "d2q9")
    s.run()
    ns = s._embed_ns
    assert ns["shape"] == (65, 21, 2)
    arr = ns["arrays"]
    assert sorted(arr) == ["Rho", "Rho.si", "U", "U.si"]
    lat = s.lattice
    rho = lat.quantity("Rho")[0].numpy()          # (nz, ny, nx)
    u = lat.quantity("U").numpy()
    assert arr["Rho"].shape == (64, 20, 1) and arr["U"].shape == (3, 64, 20, 1)
    assert np.array_equal(arr["Rho"][:, :, 0], rho[0].T)
    assert np.array_equal(arr["U"][0, :, :, 0], u[0, 0].T)
    # SI: velocity scales with dx/dt, positions are cell centres in metres
    sc = 1.0 / s.units.unit_scale("m/s")
    np.testing.assert_allclose(arr["U.si"], arr["U"] * sc)
    api = ns["Solver"]
    X = api.Geometry.X
    np.testing.assert_allclose(X[:3, 0, 0], (np.arange(3) + 0.5) * 0.001)
    assert api.Geometry.dim.tolist() == [64, 20, 1] and api.Geometry.size == 64 * 20


def test_api_settings_actions_errors(tmp_path):
    s = _solver(tmp_path, KARMAN.replace("<Solve Iterations=\"40\"/>", ""), "d2q9")
    s.run()
    api = s._embed_ns["Solver"]
    api.Settings.Viscosity = 0.03
    assert s.lattice.get_setting("Viscosity") == pytest.approx(0.03)
    assert api.Settings.VelocityX.DefaultZone == pytest.approx(0.01)
    api.Settings.VelocityX.DefaultZone = 0.02
    assert s.lattice.get_setting("VelocityX") == pytest.approx(0.02)
    it = s.lattice.iter
    api.Actions.Iteration()
    assert s.lattice.cur in (0, 1) and "Iteration" in dir(api.Actions)
    assert api.Info.OutputPath == s.outpath
    assert sorted(dir(api)) == sorted(["Settings", "Fields", "Parameters", "Quantities", "Globals", "Actions",
                                       "Geometry", "Info"])
    with pytest.raises(AttributeError):
        api.Quantities.NotAQuantity
    from tclb_amd.handlers.base import HandlerError
    bad = KARMAN.replace("import json", "Solverr.Settings")
    with pytest.raises(HandlerError, match="Solverr"):
        _solver(tmp_path, bad, "d2q9").run()
    del it


def test_geometry_assignment_refreshes_ghost_flags(tmp_path):
    """with ghost planes (multi-rank path, this rank its own neighbour) the edited flags
    reach the ghosts: the run equals the plain single-rank run"""
    from tclb_amd.parallel.comm import LoopbackComm
    xml = SPHERES.replace("<RunPython Iterations=\"10\">", "<RunPython>hist = []</RunPython>\n  <RunPython Iterations=\"10\">")
    xml = xml.replace("(30.0, 20.0), (60.0, 30.0)", "(30.0, 3.0), (60.0, 45.0)")    # spheres across the y wrap
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    a = _solver(tmp_path / "a", xml, "d2q9_adj")
    a.run()
    root = ET.fromstring(xml.format(out=tmp_path / "b"))
    b = Solver("d2q9_adj", root, conffile=os.path.join(tmp_path, "b", "case.xml"), device="cpu",
               comm=LoopbackComm(exercise_dist_path=True))
    b.run()
    assert b.lattice.g > 0
    assert np.array_equal(a.lattice.get_flags(), b.lattice.get_flags())
    lb = b.lattice
    ghost = lb.flags[:, 0, :lb.shape[0]].numpy()          # lower ghost row = top row (periodic)
    top = lb.flags[:, lb.shape[1], :lb.shape[0]].numpy()
    assert np.array_equal(ghost, top)
    assert np.array_equal(a.lattice.fields_interior().numpy(), b.lattice.fields_interior().numpy())
