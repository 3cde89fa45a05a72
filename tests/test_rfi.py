"""Socket Remote Force Interface (tclb_amd/particles/rfi.py; reference
src/RemoteForceInterface.*, simplepart.cpp, empty.cpp): a lattice coupled to the
stand-alone integrator tools/rfi_simplepart.py in another process reproduces the
in-process SIMPLEPART run (to the rounding of the executor's atomic force sums, whose
order differs between two in-process runs as well); the XML handler spawns the integrator and stops it
at the end of the run (death protocol); the empty integrator exchanges zero particles."""
import json
import os
import subprocess
import sys
import threading
import xml.etree.ElementTree as ET

import numpy as np
import torch

from tclb_amd.lattice import Lattice
from tclb_amd.particles import SimplePart
from tclb_amd.particles.rfi import IntegratorClient, RemoteParticles

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "rfi_simplepart.py")
PART = {"x": [16.0, 12.0, 12.0], "r": 4.0, "v": [0.02, 0.0, 0.0], "m": 300.0}


def _lat():
    lat = Lattice("auto_d3q19_part", (32, 24, 24))
    lat.set_flags(np.full((lat.NZ, lat.NY, 32), lat.model.node_type("MRT").value, dtype=np.uint32))
    lat.set_setting("Viscosity", 0.1)
    return lat


def test_protocol_roundtrip():
    rp = RemoteParticles("127.0.0.1:0")
    got = {}

    def integrator():
        c = IntegratorClient(rp.address)
        got["peer"] = c.peer
        got["first"] = c.exchange(np.ones((2, 3)), np.zeros((2, 3)), np.zeros((2, 3)), np.array([1.0, 2.0]))
        got["stop"] = c.exchange(np.ones((2, 3)), np.zeros((2, 3)), np.zeros((2, 3)), np.array([1.0, 2.0]))
        c.close()
    t = threading.Thread(target=integrator)
    t.start()
    rp.accept()
    rec = rp.chan.expect(2)
    from tclb_amd.particles.rfi import pack_forces, unpack_particles
    assert unpack_particles(rec).shape == (2, 10)
    rp.force, rp.torque = np.full((2, 3), 0.5), np.zeros((2, 3))
    rp.chan.send(3, pack_forces(rp.force, rp.torque, True))
    rp.close()
    t.join(10)
    assert got["peer"]["role"] == "calculator"
    integrate, f = got["first"]
    assert integrate and f.shape == (2, 6) and (f[:, :3] == 0.5).all()
    assert got["stop"] is None


def test_remote_integrator_matches_in_process(tmp_path):
    steps = 12
    a = _lat()
    sp = SimplePart()
    sp.add(PART["x"], PART["r"], v=PART["v"], m=PART["m"])
    a.particles = sp
    a.init()
    a.iterate(steps)

    cfg = tmp_path / "parts.json"
    cfg.write_text(json.dumps({"particles": [PART]}))
    b = _lat()
    rp = RemoteParticles("127.0.0.1:0")
    proc = subprocess.Popen([sys.executable, TOOL, "--address", rp.address, "--config", str(cfg),
                             "--log", str(tmp_path / "log.csv")], cwd=ROOT)
    rp.accept()
    b.particles = rp
    b.init()
    b.iterate(steps)
    rp.close()
    assert proc.wait(60) == 0
    assert torch.allclose(a.fields_interior(), b.fields_interior(), rtol=0, atol=1e-13)
    np.testing.assert_allclose(sp.force, rp.forces_all[:, 0:3], rtol=1e-10, atol=1e-14)
    rows = open(tmp_path / "log.csv").read().splitlines()
    assert len(rows) == steps + 1                    # header + one row per integrated step
    x_remote = [float(v) for v in rows[-1].split(",")[1:4]]
    np.testing.assert_allclose(x_remote, sp.x[0], rtol=1e-10)
    assert sp.x[0, 0] > PART["x"][0]                 # the particle moved


CASE = """<CLBConfig version="2.0" output="{out}/" permissive="true">
  <Geometry nx="32" ny="24" nz="24"><MRT><Box/></MRT></Geometry>
  <Model><Param name="Viscosity" value="0.1"/></Model>
  <RemoteForceInterface integrator="{integ}" spawn="{spawn}"/>
  <Solve Iterations="6"/>
</CLBConfig>"""


def test_xml_handler_spawns_and_stops_integrator(tmp_path):
    from tclb_amd import handlers  # noqa: F401
    from tclb_amd.solver import Solver
    cfg = tmp_path / "parts.json"
    cfg.write_text(json.dumps({"particles": [PART]}))
    log = tmp_path / "log.csv"
    spawn = f"{sys.executable} {TOOL} --address {{address}} --config {cfg} --log {log}"
    root = ET.fromstring(CASE.format(out=tmp_path, integ="simplepart_remote", spawn=spawn))
    s = Solver("auto_d3q19_part", root, conffile=str(tmp_path / "case.xml"), device="cpu")
    s.run()
    assert s.iter == 6
    assert len(open(log).read().splitlines()) == 7
    assert s.particles.exchanges >= 6


def test_empty_integrator(tmp_path):
    from tclb_amd import handlers  # noqa: F401
    from tclb_amd.solver import Solver
    spawn = f"{sys.executable} {TOOL} --address {{address}} --empty"
    root = ET.fromstring(CASE.format(out=tmp_path, integ="empty", spawn=spawn))
    s = Solver("auto_d3q19_part", root, conffile=str(tmp_path / "case.xml"), device="cpu")
    s.run()
    assert s.iter == 6 and s.particles.n == 0


def test_vars_and_stats_negotiated(tmp_path):
    """reference Negotiate: named variables travel both ways (the peer's value wins a
    clash), statistics are collected when either side asks; the calculator and the
    integrator each append a line of mean particle counts and phase times every `iter`
    exchanges (reference enableStats / printStats)"""
    rp = RemoteParticles("127.0.0.1:0")
    rp.set_var("output", str(tmp_path / "run"))
    rp.set_var("content", json.dumps({"particles": [PART]}))
    rp.set_var("shared", "calc")
    rp.enable_stats(str(tmp_path / "rfi"), 2)
    got = {}

    def integrator():
        c = IntegratorClient(rp.address, vars={"code": "test", "shared": "integ"})
        got["vars"] = dict(c.vars)
        got["stats"] = c.stats is not None
        x = np.array([PART["x"]])
        for _ in range(5):
            if c.exchange(x, np.zeros((1, 3)), np.zeros((1, 3)), np.array([PART["r"]])) is None:
                break
        c.close()
    t = threading.Thread(target=integrator)
    t.start()
    lat = _lat()
    rp.accept()
    assert rp.vars["code"] == "test" and rp.vars["shared"] == "integ" and rp.vars["output"].endswith("run")
    lat.particles = rp
    lat.init()
    lat.iterate(4)
    rp.close()
    t.join(20)
    assert got["vars"]["content"] and got["vars"]["shared"] == "calc" and got["stats"]
    calc = (tmp_path / "rfi_calculator_P00.txt").read_text().splitlines()
    integ = (tmp_path / "rfi_integrator_P00.txt").read_text().splitlines()
    assert calc[0].startswith("size_iter, size_000, dt_wait_particles")
    assert len(calc) >= 3 and calc[1].split(", ")[0] == "2" and float(calc[1].split(", ")[1]) == 1.0
    assert integ[0].startswith("size_iter, size_000, dt_integrate") and len(integ) >= 2


def test_handler_sends_content_output_and_attributes(tmp_path):
    """<RemoteForceInterface> passes "output", its child as "content" and its other
    attributes as numbers (reference acRemoteForceInterface.cpp:26-82); the stand-alone
    simplepart takes its particles from "content" when no --config is given"""
    from tclb_amd.particles.rfi import negotiate
    mine = {"output": "o", "content": "{}", "Velocity": "0.01"}
    vars_, st = negotiate(mine, {"enabled": True, "prefix": "", "iter": 0}, {"vars": {"x": "1"},
                                                                          "stats": {"prefix": "p", "iter": 5}})
    assert vars_ == {"output": "o", "content": "{}", "Velocity": "0.01", "x": "1"}
    assert st == {"enabled": True, "prefix": "p", "iter": 5}
