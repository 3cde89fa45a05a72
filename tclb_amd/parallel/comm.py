"""Communication backends for the lattice runtime.

The reference moves halos as host-staged MPI Isend/Irecv of per-direction margin
buffers and reduces globals with MPI_Reduce (reference: src/Lattice.cu.Rt:327-389,
1279-1292; src/Solver.cpp.Rt:288-370).  Here one process drives one GPU and:

* :class:`LoopbackComm`  — single rank; the periodic wrap of the decomposed axis is
  a device-side plane copy (the reference's self-neighbour margin aliasing,
  src/Lattice.cu.Rt:439-456);
* :class:`TorchDistComm` — ``torch.distributed`` (backend ``nccl`` = RCCL over xGMI
  on MI355X, ``gloo`` on CPU for tests): halos are device-resident packed slabs sent
  with grouped P2P ops (``batch_isend_irecv``) to the two slab neighbours, globals
  are all-reduced (SUM, then MAX) on device.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np
import torch


class Comm:
    rank = 0
    size = 1
    distributed = False

    def barrier(self):
        pass

    def allreduce_globals(self, g: torch.Tensor, nsum: int):
        return g

    def bcast_object(self, obj, src: int = 0):
        return obj

    def allreduce_scalar(self, v: float, op: str = "sum") -> float:
        return v

    def gather_objects(self, obj) -> List:
        return [obj]

    def scatter_objects(self, objs: Optional[List], src: int = 0):
        """objs[r] (given on src) -> rank r"""
        return objs[0]

    def gather_to_root(self, obj, dst: int = 0) -> Optional[List]:
        """every rank's obj, on dst only (None elsewhere)"""
        return [obj]

    def start_halo(self, send_up: Optional[torch.Tensor], send_down: Optional[torch.Tensor],
                   recv_below: Optional[torch.Tensor], recv_above: Optional[torch.Tensor], nbr=None):
        """send_up -> next, send_down -> prev, recv_below <- prev, recv_above <- next;
        nbr = (prev, next) ranks (default: rank -+ 1, the slab neighbours)"""
        raise NotImplementedError

    def wait_halo(self, handle):
        pass


class LoopbackComm(Comm):
    """Single rank: neighbour below and above are this rank (periodic).

    ``exercise_dist_path=True`` routes the halo through the multi-rank code path
    (border/interior split, pack, exchange, unpack) with this rank as its own
    neighbour — used to test that path on a single GPU."""

    def __init__(self, exercise_dist_path: bool = False):
        self.distributed = exercise_dist_path

    def start_halo(self, send_up, send_down, recv_below, recv_above, nbr=None):
        if send_up is not None:
            recv_below.copy_(send_up)
        if send_down is not None:
            recv_above.copy_(send_down)
        return None


class TorchDistComm(Comm):
    distributed = True

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.prev = (self.rank - 1) % self.size
        self.next = (self.rank + 1) % self.size

    def _g(self, r: int) -> int:
        return self.dist.get_global_rank(self.group, r) if self.group is not None else r

    def barrier(self):
        self.dist.barrier(group=self.group)

    def allreduce_globals(self, g: torch.Tensor, nsum: int):
        d = self.dist
        if self.backend == "nccl" and not g.is_cuda:
            g = g.cuda()
        if nsum > 0:
            s = g[:nsum].clone()
            d.all_reduce(s, op=d.ReduceOp.SUM, group=self.group)
            g[:nsum] = s
        if g.numel() > nsum:
            m = g[nsum:].clone()
            d.all_reduce(m, op=d.ReduceOp.MAX, group=self.group)
            g[nsum:] = m
        return g

    def allreduce_scalar(self, v: float, op: str = "sum") -> float:
        d = self.dist
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        d.all_reduce(t, op={"sum": d.ReduceOp.SUM, "max": d.ReduceOp.MAX, "min": d.ReduceOp.MIN}[op],
                     group=self.group)
        return float(t.item())

    def bcast_object(self, obj, src: int = 0):
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=self._g(src), group=self.group)
        return lst[0]

    def gather_objects(self, obj) -> List:
        out = [None] * self.size
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def scatter_objects(self, objs, src: int = 0):
        out = [None]
        self.dist.scatter_object_list(out, objs if self.rank == src else None, src=self._g(src), group=self.group)
        return out[0]

    def gather_to_root(self, obj, dst: int = 0):
        out = [None] * self.size if self.rank == dst else None
        self.dist.gather_object(obj, out, dst=self._g(dst), group=self.group)
        return out

    def start_halo(self, send_up, send_down, recv_below, recv_above, nbr=None):
        d = self.dist
        prev, nxt = nbr if nbr is not None else (self.prev, self.next)
        ops = []
        # identical op order on every rank: [send up, send down, recv below, recv above];
        # tags keep the two streams apart when prev == next (2 ranks).
        if send_up is not None:
            ops.append(d.P2POp(d.isend, send_up, self._g(nxt), self.group, 1))
        if send_down is not None:
            ops.append(d.P2POp(d.isend, send_down, self._g(prev), self.group, 2))
        if recv_below is not None:
            ops.append(d.P2POp(d.irecv, recv_below, self._g(prev), self.group, 1))
        if recv_above is not None:
            ops.append(d.P2POp(d.irecv, recv_above, self._g(nxt), self.group, 2))
        if not ops:
            return None
        return d.batch_isend_irecv(ops)

    def wait_halo(self, handle):
        if handle is None:
            return
        for w in handle:
            w.wait()


def make_comm(kind: str = "auto") -> Comm:
    """auto: TorchDistComm if torch.distributed is initialised with >1 rank."""
    import torch.distributed as dist
    if kind in ("auto", "dist") and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return TorchDistComm()
    if kind == "dist":
        raise RuntimeError("torch.distributed is not initialised")
    return LoopbackComm()


def init_distributed_from_env(device: str = "auto") -> Optional[Comm]:
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* (torchrun) if present."""
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 or dist.is_initialized():
        return make_comm()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    use_gpu = device == "cuda" or (device == "auto" and torch.cuda.is_available())
    backend = "nccl" if use_gpu else "gloo"
    kw = {}
    if use_gpu:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        # halo P2P runs on RCCL's internal stream while the interior kernel fills the CUs:
        # a high-priority stream lets its work-groups dispatch as soon as CUs free up
        if os.environ.get("TCLB_RCCL_HIGH_PRIORITY", "1") != "0":
            try:
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
            except (AttributeError, RuntimeError):
                pass
    dist.init_process_group(backend=backend, **kw)
    return make_comm()
