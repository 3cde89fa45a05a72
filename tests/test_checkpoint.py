"""Portable checkpoints (tclb_amd/io/checkpoint.py; reference SaveCheckpoint/LoadBinary,
src/Lattice.cu.Rt:708-769): shifted reduced-precision storage round-trips bit for bit,
and a checkpoint written on N gloo ranks restarts on M ranks (M != N, M = 1 included)
bit for bit against an uninterrupted single-rank run."""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import dist_worker
from model_cases import make_case, perturb, run
from tclb_amd.io.checkpoint import load_state, save_state


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _solver(lat):
    from tclb_amd.parallel.comm import LoopbackComm
    return types.SimpleNamespace(lattice=lat, rank=0, comm=LoopbackComm(), iter=lat.iter)


@pytest.mark.parametrize("precision", ["float-shift", "mixed-shift", "half-shift", "float", "double"])
def test_checkpoint_roundtrip_is_bitwise(tmp_path, precision):
    a = run("d3q27", "cpu", steps=4, precision=precision)
    path = save_state(_solver(a), str(tmp_path / "ck"))
    b = make_case("d3q27", "cpu", precision=precision)
    b.init()
    s = _solver(b)
    load_state(s, path)
    assert s.iter == 4 and b.iter == 4
    assert torch.equal(a.snaps[a.cur][:, :, :, :a.shape[0]], b.snaps[b.cur][:, :, :, :b.shape[0]])


@pytest.mark.parametrize("model", ["d3q27", "d3q27_pf_velocity"])
def test_checkpoint_n_to_m_ranks(tmp_path, model):
    """written on 4 ranks, restarted on 2 ranks and on 1 rank: equal to 8 uninterrupted
    single-rank steps"""
    ref = run(model, "cpu", steps=8)
    path = str(tmp_path / "ck4.tclb")
    mp.start_processes(dist_worker.worker_checkpoint, args=(4, _port(), model, path, 5, 0, ""),
                       nprocs=4, start_method="spawn", join=True)
    assert os.path.exists(path)
    out = str(tmp_path / "r2.npy")
    mp.start_processes(dist_worker.worker_checkpoint, args=(2, _port(), model, path, 0, 3, out),
                       nprocs=2, start_method="spawn", join=True)
    assert open(out + ".iter").read() == "8"
    assert np.array_equal(np.load(out), ref.fields_interior().numpy())
    one = make_case(model, "cpu")
    one.init()
    load_state(_solver(one), path)
    one.iterate(3)
    assert torch.equal(one.fields_interior(), ref.fields_interior())
