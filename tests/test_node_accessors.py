"""Emitted node accessors (emit/emitter.py): the row form (uniform row base + lane x,
core.hpp row_at) with globals through glob_add/glob_max (LDS accumulators on the GPU
primal executor), and the flat form with per-thread globals that the GPU adjoint build
selects (TCLB_FLAT_NODE=1, build.py _adhip_source; profiles/README.md r03p)."""
import os

import pytest

from tclb_amd import build as B
from tclb_amd.emit.emitter import emit_header
from tclb_amd.models import registry


@pytest.mark.parametrize("name", ["d3q27", "d3q19_adj", "d3q27_pf_velocity"])
def test_both_accessor_forms_emitted(name):
    h = emit_header(registry.get(name))
    assert "#if TCLB_FLAT_NODE" in h
    flat, row = h.split("#if TCLB_FLAT_NODE", 1)[1].split("#else", 1)
    assert "row_at(" not in flat and "glob_add(" not in flat
    # every global accumulates through glob_add/glob_max in the row form, plainly in the flat one
    for g in registry.get(name).globals_:
        assert f"void AddTo{g.name}(R v)" in h
    assert h.count("glob_add(glob_") + h.count("glob_max(glob_") >= len(registry.get(name).globals_)
    assert "A.yzo(dy, dz)" in h and "A.off(dx, dy, dz)" in h


def test_gpu_adjoint_build_selects_flat_accessors(tmp_path):
    p = B._adhip_source(registry.get("d3q19_adj"), str(tmp_path))
    src = open(p).read()
    assert "#define TCLB_FLAT_NODE 1" in src
    assert src.index("TCLB_FLAT_NODE") < src.index('#include "model.hpp"')
    assert os.path.basename(p) == "kernels_adhip.hip"
