"""Occupancy floor of the globals-integrating kernels (Model.glob_waves ->
Model::GLOB_WAVES_, executor_hip.hpp k_stage_glob): 2 waves/SIMD by default, off for the
models whose GLOB kernels need 256 VGPRs or more (they spilled under the cap, r03s)."""
import pytest

from tclb_amd.emit.emitter import emit_header
from tclb_amd.models import registry


@pytest.mark.parametrize("name,waves", [("d3q27", 2), ("d3q27_pf_velocity", 0), ("d3q27_pf_velocity_thermo", 0),
                                        ("d3q27_pf_velocity_OutFlow", 0), ("d3q27_tePSM_per_NEBB", 0),
                                        ("d3q27q7_cm_cht_OutFlowConvective", 0), ("d3q27q7_cm_cht", 0),
                                        ("d3q27_PSM_NEBB_singlekernel", 0), ("d3q27_PSM_NEBB", 2)])
def test_glob_waves_emitted(name, waves):
    m = registry.get(name)
    assert m.glob_waves == waves
    assert f"static constexpr int GLOB_WAVES_ = {waves};" in emit_header(m)
