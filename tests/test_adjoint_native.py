"""The unsteady adjoint's reverse sweep runs each checkpoint segment in one native call
(tclb_rt/ad_loop.hpp ad_segment, adjoint.py _segment_native) and gives the adjoint state,
objective and design gradient of the per-step Python sweep — reverse sweeps
(Model.set_reverse) and dual-number passes, on the CPU and the GPU executors.  Reference:
Iteration_Adj / IterateTill run these steps in C++ (src/Lattice.cu.Rt:542-613,843-890)."""
import numpy as np
import pytest
import torch

import test_adjoint_reverse as R

CASES = {"d3q19_adj": R._case, "d2q9_adj": R._d2q9_case, "d3q19_heat_adj": R._heat_case}


def _pair(monkeypatch, case, device, reverse):
    out = []
    for native in ("1", "0"):
        monkeypatch.setenv("TCLB_AD_NATIVE", native)
        lat, ad = case(device, reverse)
        out.append(ad)
    return out


def _check(monkeypatch, name, device, reverse):
    n, p = _pair(monkeypatch, CASES[name], device, reverse)
    assert n.native_steps > 0 and p.native_steps == 0
    a, b = n.a0.cpu(), p.a0.cpu()
    scale = b.abs().max().item()
    assert scale > 0
    # the adjoint push accumulates with atomics (OpenMP threads / GPU waves): rounding
    assert torch.allclose(a, b, rtol=0, atol=1e-13 * scale), (a - b).abs().max().item() / scale
    assert abs(n.J - p.J) <= 1e-14 * abs(p.J)


@pytest.mark.parametrize("reverse", [True, False])
@pytest.mark.parametrize("name", list(CASES))
def test_native_segment_matches_python_cpu(monkeypatch, name, reverse):
    _check(monkeypatch, name, "cpu", reverse)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
@pytest.mark.parametrize("reverse", [True, False])
@pytest.mark.parametrize("name", list(CASES))
def test_native_segment_matches_python_gpu(monkeypatch, name, reverse):
    _check(monkeypatch, name, "cuda", reverse)
