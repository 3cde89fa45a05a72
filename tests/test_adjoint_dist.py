"""Multi-rank discrete adjoint (reference Iteration_Adj on every rank with the adjoint
margins exchanged in the opposite direction, src/Lattice.cu.Rt:542-613): the unsteady
adjoint of N gloo ranks (ghost-plane contributions returned to the owning neighbour by
Lattice.reverse_halo) equals the single-rank adjoint — adjoint state, objective and
setting gradient — for a 3-D design model on z slabs and on a Y x Z grid, and a
two-stage stencil model on y slabs; the loopback multi-rank path equals the plain one."""
import json
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import dist_worker
from tclb_amd.parallel.comm import LoopbackComm


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,world,grid", [("d3q19_adj", 2, None), ("d3q19_adj", 3, None),
                                              ("d3q19_adj", 4, (2, 2)), ("d2q9_kuper", 2, None)])
def test_adjoint_ranks_match_single(tmp_path, model, world, grid):
    lat, ad = dist_worker.adjoint_case(model)
    name = "Theta" if model == "d3q19_adj" else "GravitationX"
    nx, ny, nz = lat.shape
    ref = ad.a0[:, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx].numpy()
    out = str(tmp_path / "adj.npy")
    mp.start_processes(dist_worker.worker_adjoint, args=(world, _port(), model, out, grid),
                       nprocs=world, start_method="spawn", join=True)
    full = np.load(out)
    meta = json.load(open(out + ".json"))
    scale = np.abs(ref).max()
    assert scale > 0
    np.testing.assert_allclose(full, ref, rtol=0, atol=1e-12 * scale)
    assert abs(meta["J"] - ad.J) <= 1e-12 * abs(ad.J)
    g1 = ad.setting_gradient(name)
    assert g1 != 0 and abs(meta["grad"] - g1) <= 1e-10 * abs(g1), (meta["grad"], g1)


@pytest.mark.parametrize("model", ["d3q19_adj", "d2q9_kuper"])
def test_adjoint_loopback_dist_path(model):
    a_lat, a = dist_worker.adjoint_case(model, LoopbackComm(exercise_dist_path=True))
    b_lat, b = dist_worker.adjoint_case(model)
    nx, ny, nz = a_lat.shape
    sa = a.a0[:, a_lat.gz:a_lat.gz + nz, a_lat.gy:a_lat.gy + ny, :nx]
    sb = b.a0[:, :nz, :ny, :nx]
    assert torch.allclose(sa, sb, rtol=0, atol=1e-12 * sb.abs().max().item())


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
@pytest.mark.parametrize("model", ["d3q19_adj", "d2q9_kuper"])
def test_gpu_adjoint_loopback_dist_path(model):
    """the GPU adjoint executor through the multi-rank path (ghost planes, reverse halo)
    equals the CPU single-rank adjoint"""
    a_lat, a = dist_worker.adjoint_case(model, LoopbackComm(exercise_dist_path=True), device="cuda")
    assert a_lat.is_gpu and a.lib is not None
    b_lat, b = dist_worker.adjoint_case(model)
    nx, ny, nz = a_lat.shape
    sa = a.a0[:, a_lat.gz:a_lat.gz + nz, a_lat.gy:a_lat.gy + ny, :nx].cpu()
    sb = b.a0[:, :nz, :ny, :nx]
    assert torch.allclose(sa, sb, rtol=0, atol=1e-11 * sb.abs().max().item())
