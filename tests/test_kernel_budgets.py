"""Register budgets of the built gfx950 kernels, read from the code objects' metadata
(tools/isa_stats.py; runs on the build host, no GPU).

* The class-2 fence: every class-2 tile-list kernel of a split stage, and every
  deferred-node kernel, runs without AGPRs.  Without the 2-wave floor the tePSM class-2
  kernel (344 VGPRs + 88 AGPRs) was miscompiled by the GCN scheduler's high-pressure
  reschedule stage (profiles/README.md r05m, r06s-u).
* The budgets the round-6 measurements rest on: the headline collide fits 3 waves/SIMD
  (136 VGPRs today);
  the deferring tePSM class-1 collide stays within 256 VGPRs without AGPRs or scratch
  (2 waves/SIMD, r06k); the particle force stage of config 5 stays small (r06k-l)."""
import os
import re
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

LLVM = "/opt/rocm/lib/llvm/bin"
pytestmark = pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-readelf"), reason="no ROCm LLVM tools")


def _meta(model):
    import isa_stats
    from tclb_amd import build as B
    so = B.lib_path(model, "hip", "")
    if not os.path.exists(so):
        pytest.skip(f"{model}: HIP library not built")
    with tempfile.TemporaryDirectory() as tmp:
        meta = isa_stats.kernels(isa_stats.code_object(so, tmp))
    names = sorted(meta)
    return [(d, meta[n]) for n, d in zip(names, isa_stats.demangle(names))]


def _targs(name):
    """the template arguments of a demangled kernel name (top level only)"""
    s = name[name.index("<") + 1:]
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            if depth == 0:
                out.append(cur.strip())
                return out
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    return out


SPLIT_MODELS = ["d3q27_tePSM_per_NEBB", "d3q27_tePSM_per_SUP", "d3q27_pf_velocity", "d3q27_pf_velocity_thermo",
                "d2q9_pf_velocity", "auto_d3q19_part", "d3q27_PSM_NEBB"]


@pytest.mark.parametrize("model", SPLIT_MODELS)
def test_class2_and_deferred_kernels_use_no_agprs(model):
    seen = 0
    for name, m in _meta(model):
        if re.search(r"k_stage_list(_w)?<", name):
            if _targs(name)[-1] != "2":
                continue
        elif "k_stage_deferred<" not in name:
            continue
        seen += 1
        assert m["agpr"] == 0 and m["vgpr"] <= 256, (name[:160], m)
    if model.startswith("d3q27_tePSM"):
        assert seen > 0


def test_headline_collide_budget():
    rows = [(n, m) for n, m in _meta("d3q27") if n.startswith("void tclb::exec::k_stage<")
            and _targs(n)[1:3] == ["double", "double"] and _targs(n)[4] == "false"]
    assert rows
    for n, m in rows:
        assert m["vgpr"] <= 168 and m["agpr"] == 0 and m["scratch"] == 0, (n, m)


def test_tepsm_deferring_collide_budget():
    rows = [(n, m) for n, m in _meta("d3q27_tePSM_per_NEBB")
            if "k_stage_defer<" in n and _targs(n)[1:3] == ["double", "double"] and _targs(n)[3] == "1"
            and _targs(n)[4] == "false"]      # the plain step (the globals step is uncapped)
    assert rows
    for n, m in rows:
        assert m["vgpr"] <= 256 and m["agpr"] == 0 and m["scratch"] == 0, (n[:160], m)


def test_particle_force_stage_budget():
    rows = [(n, m) for n, m in _meta("auto_d3q19_part")
            if "k_stage_defer<" in n and _targs(n)[1:3] == ["double", "double"] and _targs(n)[4] == "false"]
    assert rows
    for n, m in rows:
        assert m["vgpr"] <= 64 and m["scratch"] == 0, (n[:160], m)
