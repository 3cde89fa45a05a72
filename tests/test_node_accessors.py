"""Emitted node accessors (emit/emitter.py): one accessor set whose addressing form is a
compile-time choice per instantiation (Node::ROWA_): one 32-bit offset per access in the
plain kernels, a uniform row base + lane x (core.hpp row_at) in the globals kernels, the
flat form everywhere in the GPU adjoint build (TCLB_FLAT_NODE=1, build.py _adhip_source;
profiles/README.md r03p, r04b, r04c).  Globals go through glob_add/glob_max in every
form (LDS, register and dual-number accumulators alike)."""
import os

import pytest

from tclb_amd import build as B
from tclb_amd.emit.emitter import emit_header
from tclb_amd.models import registry


@pytest.mark.parametrize("name", ["d3q27", "d3q19_adj", "d3q27_pf_velocity"])
def test_one_accessor_set_with_compile_time_form(name):
    h = emit_header(registry.get(name))
    assert "#if TCLB_FLAT_NODE" not in h            # no preprocessor fork of the accessors
    assert "static constexpr bool ROWA_ = TCLB_ROW_ADDR && !TCLB_FLAT_NODE && (GLOB || TCLB_ROW_ADDR_PLAIN);" in h
    # both forms behind if constexpr in ld / ld_out / st / NodeType_at
    assert h.count("if constexpr (ROWA_)") >= 5
    assert h.count("row_at<true>(") >= 5 and "row_at(" not in h.replace("row_at<true>(", "")
    assert "A.yzo(dy, dz)" in h and "A.off(dx, dy, dz)" in h
    # every global accumulates through glob_add/glob_max
    m = registry.get(name)
    for g in m.globals_:
        assert f"void AddTo{g.name}(R v)" in h
    assert "glob_[" not in h.replace("glob_add(glob_", "").replace("glob_max(glob_", "")
    assert h.count("glob_add(glob_") + h.count("glob_max(glob_") >= len(m.globals_)


def test_gpu_adjoint_build_selects_flat_accessors(tmp_path):
    p = B._adhip_source(registry.get("d3q19_adj"), str(tmp_path))
    src = open(p).read()
    assert "#define TCLB_FLAT_NODE 1" in src
    assert src.index("TCLB_FLAT_NODE") < src.index('#include "model.hpp"')
    assert os.path.basename(p) == "kernels_adhip.hip"
