"""The benches' 'did the physics happen' guard (tclb_amd/utils/guard.py): a run whose
flags select no collision (the round-4 pf_velocity runs flagged BGK on a build that only
collides MRT nodes) is caught, and the perf tools exit non-zero on it."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice
from tclb_amd.utils.guard import collision_check

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from model_cases import case_settings  # noqa: E402


def _lat(name, flag, n=12):
    lat = Lattice(name, (n, n, n), device=torch.device("cpu"))
    lat.set_flags(np.full((lat.NZ, lat.NY, n), lat.model.node_type(flag).value, dtype=np.uint32))
    for k, v in case_settings(name).items():
        if not k.startswith("_") and lat.model.setting(k) is not None:
            lat.set_setting(k, v)
    lat.init()
    lat.iterate(2)
    return lat


@pytest.mark.parametrize("name,flag,collides", [("d3q27_pf_velocity", "BGK", False),
                                                ("d3q27_pf_velocity", "MRT", True),
                                                ("d3q27", "MRT", True), ("auto_d3q19_BGK", "MRT", True)])
def test_collision_check(name, flag, collides):
    lat = _lat(name, flag)
    before = lat.fields_interior().clone()
    it, cur = lat.iter, lat.cur
    g = collision_check(lat)
    assert g["collides"] is collides, g
    assert g["collision_nodes"] == 1.0
    # the lattice is left as it was
    assert torch.equal(before, lat.fields_interior()) and (lat.iter, lat.cur) == (it, cur)


def _perf(flag):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "tools", "perf_models.py"), "--device", "cpu", "--models",
           "d3q27_pf_velocity", "--n3", "12", "--steps", "2", "--flag", flag]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)


def test_perf_models_rejects_a_stream_only_run():
    """the r04r case: every node flagged BGK on the MRT build — the run exits non-zero and
    its line says it did not collide; flagged MRT it passes"""
    bad = _perf("BGK")
    assert bad.returncode == 3, bad.stderr[-2000:]
    rec = json.loads([l for l in bad.stdout.splitlines() if l.startswith("{")][0])
    assert rec["collides"] is False and rec["valid"] is False
    good = _perf("MRT")
    assert good.returncode == 0, good.stderr[-2000:]
    rec = json.loads([l for l in good.stdout.splitlines() if l.startswith("{")][0])
    assert rec["collides"] is True and rec["valid"] is True


def _lat2(name, flag=None, n=48):
    lat = Lattice(name, (n, n, 1), device=torch.device("cpu"))
    m = lat.model
    t = m.node_type(flag) if flag else next((x for x in m.node_types if x.group == "COLLISION"), None)
    lat.set_flags(np.full((lat.NZ, lat.NY, n), t.value if t else 0, dtype=np.uint32))
    for k, v in case_settings(name).items():
        if not k.startswith("_") and m.setting(k) is not None:
            lat.set_setting(k, v)
    lat.init()
    lat.iterate(2)
    return lat


@pytest.mark.parametrize("name,flag,collides,mode", [
    ("d2q9_reaction_diffusion_system_SIR_ModifiedPeng", "SRT_DF", True, "dynamics"),   # Run's default branch
    ("d2q9_reaction_diffusion_system_SimpleDiffusion", "TRT_M", True, None),
    ("diffusion2D", None, True, "dynamics"),               # no COLLISION group: a stencil update
    ("wave2D", None, True, "dynamics"),
    ("d2q9q9_cm_cht", "CM", False, "dynamics"),            # a type Run() has no case for: streaming only
    ("d2q9q9_cm_cht", "CM_HIGHER", True, "flags"),
])
def test_guard_models_without_flag_dispatch(name, flag, collides, mode):
    """models whose Run() does not select the collision by the COLLISION bits are judged
    by one step from a non-uniform state against pure streaming of its populations"""
    g = collision_check(_lat2(name, flag))
    assert g["collides"] is collides and mode in (None, g["mode"]), g
