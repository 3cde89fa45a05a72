"""Multi-process (gloo) decomposition tests: N ranks must reproduce 1 rank bit-for-bit
(halo exchange, border/interior overlap, periodic wrap, global all-reduce)."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_worker
from tclb_amd.parallel.comm import LoopbackComm


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,shape,world,overlap", [
    ("d3q27", (16, 8, 12), 2, True),
    ("d3q27", (16, 8, 10), 3, False),
    ("d2q9", (24, 18, 1), 2, True),
])
def test_ranks_match_single(tmp_path, model, shape, world, overlap):
    steps = 5
    ref = dist_worker.run_case(model, shape, steps, LoopbackComm())
    out = str(tmp_path / "full.npy")
    mp.start_processes(dist_worker.worker, args=(world, _port(), model, shape, steps, out, overlap),
                       nprocs=world, start_method="spawn", join=True)
    full = np.load(out)
    r = ref.fields_interior().numpy()
    assert full.shape == r.shape
    assert np.array_equal(full, r)
    g = json.load(open(out + ".json"))
    for k, v in ref.globals.items():
        assert abs(g[k] - v) <= 1e-11 * (1 + abs(v)), k
