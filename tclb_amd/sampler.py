"""Per-iteration probes (reference Sampler, src/Sampler.cpp:16-99, filled every iteration
by Lattice::updateAllSamples, src/Lattice.cu.Rt:531 and 1376-1389).

The probes of every step are written by a point-gather kernel (``tclb_<model>_sample``,
one launch per step for all points and quantities) into a device buffer
``double[rows][points][width]``; the host reads the buffer once per callback interval.
Inside the native multi-step loop (``Lattice.iterate`` -> ``tclb::iterate_action``) the
probe launch follows the last stage of every step, so sampling does not force the Python
per-step path.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from .ops import abi


class Sampler:
    """probes at global lattice points; quantities in model order (reference
    Sampler::Allocate lays them out the same way)"""

    def __init__(self, lat, points: Sequence[Tuple[int, int, int]], quantities: Sequence[str],
                 scales: Dict[str, float] = None, rows: int = 1):
        m = lat.model
        self.lat = lat
        scales = scales or {}
        qs = [q for q in m.quantities if q.name in set(quantities) and not q.adjoint]
        if len(qs) > abi.SAMPLE_MAXQ:
            raise ValueError(f"at most {abi.SAMPLE_MAXQ} sampled quantities")
        self.quantities = qs
        self.columns: List[str] = []
        plan = abi.SamplePlan()
        off = 0
        for i, q in enumerate(qs):
            nc = 3 if q.vector else 1
            plan.q[i] = m.quantities.index(q)
            plan.ncomp[i] = nc
            plan.offset[i] = off
            plan.scale[i] = float(scales.get(q.name, 1.0))
            self.columns += [f"{q.name}.{c}" for c in "xyz"] if q.vector else [q.name]
            off += nc
        plan.nq = len(qs)
        plan.width = off
        # points owned by this rank, in local coordinates
        ox, oy, oz = lat.slab.offset
        nx, ny, nz = lat.shape
        self.points = [tuple(int(v) for v in p) for p in points]
        self.mine = [i for i, (x, y, z) in enumerate(self.points)
                     if 0 <= x < nx and oy <= y < oy + ny and oz <= z < oz + nz]
        loc = np.array([[self.points[i][0], self.points[i][1] - oy, self.points[i][2] - oz] for i in self.mine],
                       dtype=np.int32).reshape(-1, 3)
        self._pts = torch.from_numpy(loc.copy()).to(lat.device)
        plan.points = self._pts.data_ptr() if len(self.mine) else None
        plan.np = len(self.mine)
        self.plan = plan
        self.row = 0
        self.start_iter = lat.iter
        self._alloc(max(1, int(rows)))

    def _alloc(self, rows: int):
        old = getattr(self, "buf", None)
        self.buf = torch.zeros((rows, max(1, self.plan.np), max(1, self.plan.width)), dtype=torch.float64,
                               device=self.lat.device)
        if old is not None and self.row:
            self.buf[:self.row].copy_(old[:self.row])
        self.plan.out = self.buf.data_ptr()
        self.plan.rows = rows

    def reserve(self, n: int):
        """room for n more steps (the buffer grows if a callback interval was longer)"""
        if self.row + n > self.plan.rows:
            self._alloc(max(self.row + n, 2 * self.plan.rows))

    def plan_for(self, n: int) -> abi.SamplePlan:
        self.reserve(n)
        self.plan.row = self.row
        return self.plan

    def advance(self, n: int):
        self.row += n

    def sample_now(self):
        """record the current state as the next row (Python per-step path)"""
        lat = self.lat
        self.reserve(1)
        self.plan.row = self.row
        if self.plan.np:
            L = lat._L
            L.in_ = lat.snaps[lat.cur].data_ptr()
            L.out = lat.snaps[1 - lat.cur].data_ptr()
            L.iter = lat.iter
            L.reserved1 = max(1, lat.iter - lat.average_start)
            L.glob = 0
            L.stream = lat._stream()
            lat.lib.sample(L, lat.prec, self.plan)
        self.row += 1

    def flush(self) -> List[Tuple[int, int, Tuple[int, int, int], np.ndarray]]:
        """rows recorded since the last flush as (iteration, point index, point, values),
        this rank's points only; resets the buffer"""
        n = self.row
        vals = self.buf[:n].cpu().numpy() if n and self.plan.np else np.zeros((n, 0, 0))
        out = []
        for r in range(n):
            it = self.start_iter + r + 1           # state after iteration start_iter + r + 1
            for k, i in enumerate(self.mine):
                out.append((it, i, self.points[i], vals[r, k, :self.plan.width].copy()))
        self.row = 0
        self.start_iter = self.lat.iter
        return out
