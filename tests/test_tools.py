"""Auxiliary native tools: tclb-compare (reference src/compare.cpp) on .pvti datasets."""
import os
import subprocess

import numpy as np
import pytest

from tclb_amd.build import build_tools, tool_path
from tclb_amd.io.vtk import write_pvti, write_vti


def dataset(d, name, rho, u, flag):
    tot = (0, 0, 0, 8, 6, 4)
    pieces = []
    for k, (z0, nz) in enumerate([(0, 2), (2, 2)]):
        reg = (0, 0, z0, 8, 6, nz)
        src = f"{name}_P{k:02d}.vti"
        write_vti(os.path.join(d, src), tot, reg,
                  [("Rho", rho[z0:z0 + nz], 1), ("U", u[:, z0:z0 + nz], 3), ("BOUNDARY", flag[z0:z0 + nz], 1)])
        pieces.append((reg, src))
    write_pvti(os.path.join(d, name + ".pvti"), tot, pieces,
               [("Rho", "Float64", 1), ("U", "Float64", 3), ("BOUNDARY", "UInt8", 1)])
    return os.path.join(d, name + ".pvti")


def run(*args):
    build_tools()
    r = subprocess.run([tool_path("compare"), *map(str, args)], capture_output=True, text=True)
    return r.returncode, r.stdout


def test_compare(tmp_path):
    rng = np.random.default_rng(0)
    rho = 1 + 0.01 * rng.standard_normal((4, 6, 8))
    u = 0.01 * rng.standard_normal((3, 4, 6, 8))
    flag = (rng.random((4, 6, 8)) > 0.5).astype(np.uint8)
    a = dataset(tmp_path, "a", rho, u, flag)
    b = dataset(tmp_path, "b", rho, u, flag)
    rc, out = run(a, b)
    assert rc == 0 and "Rho: Max difference: 0" in out, out
    u2 = u.copy()
    u2[1, 3, 2, 5] += 1e-12                 # 4500 eps: fails at eps=1000, passes at eps=1e4
    c = dataset(tmp_path, "c", rho, u2, flag)
    assert run(a, c, 1000)[0] == 1
    assert run(a, c, 1e4)[0] == 0
    rho3 = np.roll(rho, 1, axis=2)          # shifted copy: agrees with delta_x = 1
    d = dataset(tmp_path, "d", rho3, np.roll(u, 1, axis=3), np.roll(flag, 1, axis=2))
    assert run(a, d)[0] == 1
    assert run(a, d, 1, 1, 0, 0)[0] == 0


def test_case_runner(tmp_path, monkeypatch):
    """tools/tests.sh equivalent: runs tests/cases/d2q9/channel.test (solver run, CSV log
    and VTK fields against stored outputs, expected failure)."""
    from tclb_amd.tools import testrun
    monkeypatch.chdir(tmp_path)
    assert testrun.main(["d2q9"]) == 0
    assert testrun.main(["no_such_model"]) == 0     # no tests -> no error, as the reference


def test_csvdiff(tmp_path):
    from tclb_amd.tools.csvdiff import csvdiff
    a, b, c = tmp_path / "a.csv", tmp_path / "b.csv", tmp_path / "c.csv"
    a.write_text('"Iteration","X","Walltime"\n1, 1.0, 5\n2, 2.0, 6\n')
    b.write_text('"Iteration","X","Walltime"\n1, 1.0, 7\n2, 2.0000000000001, 8\n')
    c.write_text('"Iteration","X","Walltime"\n1, 1.0, 7\n2, 2.1, 8\n')
    assert csvdiff(str(a), str(b), 1e-10, "Walltime") == 0
    assert csvdiff(str(a), str(b), 1e-10, "") == 3
    assert csvdiff(str(a), str(c), 1e-10, "Walltime") == 3
