"""Whole-stack multi-rank runs: ``python -m tclb_amd`` under ``torch.distributed.run``
with 2 and 4 gloo ranks must reproduce the single-rank run of the same XML case
(reference: mpirun -np N CLB/<model>/main case.xml).

* VTK output (.pvti assembled over the rank pieces) bit for bit,
* the Log CSV equal except the wall-clock columns,
* Sample CSV identical,
* a checkpoint written on 4 ranks restarts (its restart XML) on 2 ranks and on 1 rank
  with bitwise equal results,
* a moving SIMPLEPART particle: the particle log and fields equal to 1e-12 (the
  per-node force sums go through atomics, so their order is not fixed)."""
import csv
import glob
import os
import shutil
import socket
import subprocess
import sys

import numpy as np
import pytest

from tclb_amd.io.vtk import read_pvti

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = os.path.join(ROOT, "tests", "cases")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(workdir, model, case, nproc):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS=str(max(1, 8 // nproc)))
    env.pop("WORLD_SIZE", None)
    if nproc == 1:
        cmd = [sys.executable, "-m", "tclb_amd", model, case, "--device", "cpu"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m", "tclb_amd", model, case,
               "--device", "cpu"]
    r = subprocess.run(cmd, cwd=workdir, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        err = r.stderr
        k = max(err.find("Traceback"), err.find("terminate called"))
        raise AssertionError(f"rc={r.returncode}\n" + r.stdout[-1500:] + (err[k:k + 4000] if k >= 0 else err[-4000:]))


def _case_dir(tmp_path, tag, src):
    d = tmp_path / tag
    d.mkdir()
    shutil.copy(src, d / os.path.basename(src))
    return d


def _csv(path, drop=("walltime",)):
    rows = list(csv.reader(open(path)))
    keep = [i for i, h in enumerate(rows[0]) if not any(k in h.lower() for k in drop)]
    return [[r[i] for i in keep] for r in rows]


def _pvtis(d):
    return sorted(os.path.basename(p) for p in glob.glob(str(d / "output" / "*.pvti")))


def _assert_same_vtk(a, b, tol=0.0):
    names = _pvtis(a)
    assert names and names == _pvtis(b)
    for n in names:
        fa, fb = read_pvti(str(a / "output" / n)), read_pvti(str(b / "output" / n))
        assert fa.keys() == fb.keys()
        for k in fa:
            if tol == 0.0:
                assert np.array_equal(fa[k], fb[k]), (n, k)
            else:
                s = np.abs(fb[k]).max() + 1e-300
                assert np.allclose(fa[k], fb[k], rtol=0, atol=tol * s), (n, k, np.abs(fa[k] - fb[k]).max())


@pytest.mark.parametrize("nproc", [2, 4])
def test_channel_2d_xml_ranks_match_single(tmp_path, nproc):
    src = os.path.join(CASES, "d2q9", "channel.xml")
    one = _case_dir(tmp_path, "one", src)
    many = _case_dir(tmp_path, "many", src)
    _run(one, "d2q9", "channel.xml", 1)
    _run(many, "d2q9", "channel.xml", nproc)
    _assert_same_vtk(one, many)
    assert len(glob.glob(str(many / "output" / "*_VTK_P*.vti"))) == nproc
    la, lb = (_csv(d / "output" / "channel_Log_P00_00000000.csv") for d in (one, many))
    assert la == lb


def test_d3q27_xml_vtk_log_sample_checkpoint(tmp_path):
    src = os.path.join(CASES, "dist", "channel3d.xml")
    one = _case_dir(tmp_path, "one", src)
    four = _case_dir(tmp_path, "four", src)
    _run(one, "d3q27", "channel3d.xml", 1)
    _run(four, "d3q27", "channel3d.xml", 4)
    _assert_same_vtk(one, four)
    # globals are sums over ranks in a different order: equal to rounding (YFlux and ZFlux
    # are cancellations of O(1e-4) node sums)
    la, lb = (_csv(d / "output" / "channel3d_Log_P00_00000000.csv") for d in (one, four))
    assert la[0] == lb[0] and len(la) == len(lb) == 4
    np.testing.assert_allclose(np.array(lb[1:], float), np.array(la[1:], float), rtol=1e-10, atol=1e-15)
    # HDF5 written by 4 ranks into one file (each its own slab rows) equals the 1-rank file
    from tclb_amd.io.h5read import read_h5
    h1 = read_h5(str(one / "output" / "channel3d_HDF5_00000030.h5"))
    h4 = read_h5(str(four / "output" / "channel3d_HDF5_00000030.h5"))
    assert sorted(h1) == sorted(h4) and "U" in h1
    for k in h1:
        assert np.array_equal(h1[k], h4[k]), k
    sa = open(one / "output" / "channel3d_Sampler_P00_00000000.csv").read()
    assert sa == open(four / "output" / "channel3d_Sampler_P00_00000000.csv").read()
    assert len(sa.splitlines()) == 1 + 30 * 3
    # the 4-rank checkpoint restarts on 2 ranks and on 1 rank
    rx = "channel3d_restart_00000020.xml"
    assert (four / "output" / rx).exists()
    outs = []
    for tag, n in (("r2", 2), ("r1", 1)):
        d = tmp_path / tag
        shutil.copytree(four, d)
        for p in glob.glob(str(d / "output" / "*.pvti")) + glob.glob(str(d / "output" / "*.vti")):
            os.remove(p)
        _run(d, "d3q27", os.path.join("output", rx), n)
        outs.append(d)
    _assert_same_vtk(outs[0], outs[1])
    # and the restarted run continues the uninterrupted trajectory: iteration 45 of the
    # restart equals a 1-rank run of 45 iterations
    long = _case_dir(tmp_path, "long", src)
    xml = open(long / "channel3d.xml").read().replace('<Solve Iterations="30"/>', '<Solve Iterations="50"/>')
    open(long / "channel3d.xml", "w").write(xml)
    _run(long, "d3q27", "channel3d.xml", 1)
    n45 = "restart_VTK_P00_00000045.pvti"
    restart_45 = [p for p in _pvtis(outs[0]) if p.endswith("00000045.pvti")]
    assert restart_45, _pvtis(outs[0])
    fa = read_pvti(str(outs[0] / "output" / restart_45[0]))
    fb = read_pvti(str(long / "output" / "channel3d_VTK_P00_00000045.pvti"))
    for k in fb:
        assert np.array_equal(fa[k], fb[k]), (n45, k)


def test_particle_xml_ranks_match_single(tmp_path):
    src = os.path.join(CASES, "dist", "particle.xml")
    one = _case_dir(tmp_path, "one", src)
    two = _case_dir(tmp_path, "two", src)
    _run(one, "auto_d3q19_part", "particle.xml", 1)
    _run(two, "auto_d3q19_part", "particle.xml", 2)
    _assert_same_vtk(one, two, tol=1e-12)
    la = np.loadtxt(one / "output" / "particle_SP_Log.csv", delimiter=",", skiprows=1)
    lb = np.loadtxt(two / "output" / "particle_SP_Log.csv", delimiter=",", skiprows=1)
    assert la.shape == lb.shape and la.shape[0] == 12
    forces = la[:, 7:10]
    assert np.abs(forces).max() > 0
    np.testing.assert_allclose(lb, la, rtol=1e-12, atol=1e-12 * np.abs(forces).max())
    assert la[-1, 1] > 14.3 + 0.05                    # the particle moved in x


RFI_CASE = """<?xml version="1.0"?>
<CLBConfig version="2.0" output="output/">
  <Geometry nx="32" ny="24" nz="24"><MRT><Box/></MRT></Geometry>
  <Model><Param name="Viscosity" value="0.1"/></Model>
  <RemoteForceInterface integrator="simplepart_remote" spawn="{spawn}"/>
  <Solve Iterations="8"/>
</CLBConfig>"""


def test_socket_rfi_two_ranks_match_single(tmp_path):
    """the socket RFI on 2 ranks (rank 0 scatters each rank the particles of its box and
    sums the partial forces) drives the external integrator exactly like 1 rank: same
    trajectory in the integrator log to 1e-12; the particle near z = 0 reaches only the
    lower slab"""
    import json as _json
    tool = os.path.join(ROOT, "tools", "rfi_simplepart.py")
    parts = [{"x": [16.0, 12.0, 11.5], "r": 4.0, "v": [0.02, 0.0, 0.01], "m": 300.0},
             {"x": [8.0, 6.0, 3.0], "r": 2.0, "v": [0.0, 0.01, 0.0], "m": 40.0}]
    logs = []
    for tag, n in (("one", 1), ("two", 2)):
        d = tmp_path / tag
        d.mkdir()
        (d / "parts.json").write_text(_json.dumps({"particles": parts}))
        spawn = f"{sys.executable} {tool} --address {{address}} --config parts.json --log log.csv"
        (d / "rfi.xml").write_text(RFI_CASE.format(spawn=spawn))
        _run(d, "auto_d3q19_part", "rfi.xml", n)
        logs.append(np.loadtxt(d / "log.csv", delimiter=",", skiprows=1))
    a, b = logs
    assert a.shape == b.shape and a.shape[0] == 8
    # the per-node force sums go through atomics: components that cancel to ~1e-15 carry
    # the order noise of O(1) sums
    np.testing.assert_allclose(b, a, rtol=1e-12, atol=1e-12 * np.abs(a[:, 7:10]).max())
    from tclb_amd.particles.rfi import box_subset
    rec = np.zeros((2, 10))
    rec[:, 0:3] = [p["x"] for p in parts]
    rec[:, 9] = [p["r"] for p in parts]
    lower, upper = box_subset(rec, (0, 0, 0), (32, 24, 12)), box_subset(rec, (0, 0, 12), (32, 24, 12))
    assert lower.tolist() == [0, 1] and upper.tolist() == [0]
