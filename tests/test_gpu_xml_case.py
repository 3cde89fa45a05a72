"""End-to-end XML case on the GPU against the CPU executor: the karman vortex street
(d2q9 MRT, wedge obstacle, Zou/He inlet/outlet — the geometry of the reference's
example/flow/2d/karman.xml, written by tools/bench_karman.py) runs 200 iterations through
the full Solver/handler stack on cuda:0 and on the CPU; the two VTK outputs are compared
with the native tclb-compare (reference src/compare.cpp, tools/tests.sh pvtidiff)."""
import glob
import importlib.util
import io
import contextlib
import os
import subprocess
import xml.etree.ElementTree as ET

import pytest
import torch

from tclb_amd.build import build_tools, tool_path

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _case():
    spec = importlib.util.spec_from_file_location("bench_karman", os.path.join(ROOT, "tools", "bench_karman.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.CASE


def _run(out, device):
    from tclb_amd import handlers  # noqa: F401
    from tclb_amd.solver import Solver
    os.makedirs(out, exist_ok=True)
    root = ET.fromstring(_case().format(out=out, iters=200, vtk='<VTK Iterations="200"/>'))
    with contextlib.redirect_stdout(io.StringIO()):
        s = Solver("d2q9", root, conffile=os.path.join(out, "karman.xml"), device=device)
        s.run()
    if device == "cuda":
        torch.cuda.synchronize()
    files = sorted(glob.glob(os.path.join(out, "*_00000200.pvti")))
    assert files, os.listdir(out)
    return files[-1]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_karman_gpu_vtk_matches_cpu(tmp_path):
    build_tools()
    g = _run(str(tmp_path / "gpu"), "cuda")
    c = _run(str(tmp_path / "cpu"), "cpu")
    # eps is in units of the double epsilon: 1e5 ~ 2e-11 relative (FMA contraction and
    # summation order differ between hipcc and g++ builds of the same node code)
    r = subprocess.run([tool_path("compare"), g, c, "1e5"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Max difference" in r.stdout
