"""Every production kernel above 256 registers runs GPU-vs-CPU (verdict r05: a > 256-register
kernel can be silently wrong).  tools/isa_stats.py --scan lists them
(profiles/r06/r06f_isa_scan_over256.csv): the stage kernels (k_stage, k_stage_list) and the
quantity kernels are compared by tests/test_catalog.py test_model_hip_matches_cpu on a case
with the collision type on every node and a wall plane (the interior and boundary node
classes); the sampler kernels (k_sample: every quantity of the model at the probe points,
up to 394 registers) are compared here, at wall and interior points."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")]

SAMPLE_OVER_256 = ["d2q9_csf", "d2q9_csf_bc_weno_cumulant", "d2q9_csf_bcinit_viscstep", "d2q9_csf_noflow",
                   "d3q27_cumulant_AVG_IB_SMAG", "d3q27_cumulant_IB_SMAG", "d3q27_cumulant_part_AVG_IB_SMAG",
                   "d3q27q27_cm_cht", "d3q27q27_cm_cht_AVG", "d3q27q27_cm_cht_CHT", "d3q27q27_cm_cht_IBB",
                   "d3q27q27_cm_cht_OutFlowConvective", "d3q27q27_cm_cht_OutFlowNeumann",
                   "d3q27q27_cm_cht_OutFlowNeumann_AVG_IBB", "d3q27q27_cm_cht_SMAG", "d3q27q7_cm_cht_IBB",
                   "d3q27q7_cm_cht_OutFlowConvective", "d3q27q7_cm_cht_OutFlowNeumann",
                   "d3q27q7_cm_cht_OutFlowNeumann_AVG_IBB"]


def _sampled(name, device):
    from model_cases import make_case, perturb
    from tclb_amd.ops import abi
    from tclb_amd.sampler import Sampler
    lat = make_case(name, device)
    lat.init()
    perturb(lat)
    lat.iterate(2)
    nx, ny, nz = lat.gshape
    pts = [(0, ny // 2, nz // 2), (1, 1, 0), (nx // 2, ny // 3, nz - 1), (nx - 1, ny - 1, nz // 3)]
    qs = [q.name for q in lat.model.quantities if not q.adjoint][:abi.SAMPLE_MAXQ]
    s = Sampler(lat, pts, qs)
    s.sample_now()
    return s.columns, np.array([v for _, _, _, v in s.flush()])


@pytest.mark.parametrize("name", SAMPLE_OVER_256)
def test_sample_kernel_matches_cpu(name):
    cols, a = _sampled(name, "cuda")
    _, b = _sampled(name, "cpu")
    assert a.shape == b.shape and a.size > 0
    scale = np.abs(b).max(axis=0) + 1e-300
    err = (np.abs(a - b) / scale).max(axis=0)
    bad = [(c, float(e)) for c, e in zip(cols, err) if e > 1e-10]
    assert not bad, bad
