import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(autouse=True)
def _restore_cwd():
    """tests that chdir into tmp_path must not leave later tests in a deleted directory"""
    cwd = os.getcwd()
    yield
    os.chdir(cwd)


def _devices():
    import torch
    return ["cpu", pytest.param("cuda", marks=[pytest.mark.gpu, pytest.mark.skipif(
        not torch.cuda.is_available(), reason="no GPU")])]


# analytic / physics checks that run on both executors: the CPU one here, the HIP kernels
# on a GPU box (pytest -m gpu) — independent oracles for the device code, not only
# HIP-vs-CPU comparisons of the same node source
DEVICES = _devices()
