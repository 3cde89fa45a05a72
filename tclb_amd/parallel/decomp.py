"""Domain decomposition.

The reference searches a 2-D Y x Z process grid minimising the cut surface
(reference: src/Solver.cpp.Rt:288-370, MPIDivision) and never splits X.  On one
MI355X node the 8 GPUs are a fully connected xGMI mesh with one dedicated link per
GPU pair, so a 1-D slab split along the slowest axis (z in 3-D, y in 2-D) is the
natural choice: every rank talks to exactly two neighbours over two independent
links, each halo is one contiguous plane per field, and the packed halo of a field
group is a single contiguous message.  X is never split (as in the reference).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple


@dataclass
class Slab:
    gnx: int
    gny: int
    gnz: int
    axis: int          # 1 = y, 2 = z (decomposed axis)
    rank: int
    size: int
    lo: int            # global start along axis
    n: int             # local extent along axis

    @property
    def local_shape(self) -> Tuple[int, int, int]:
        if self.axis == 2:
            return self.gnx, self.gny, self.n
        return self.gnx, self.n, self.gnz

    @property
    def offset(self) -> Tuple[int, int, int]:
        return (0, self.lo, 0) if self.axis == 1 else (0, 0, self.lo)


def split(n: int, size: int) -> List[Tuple[int, int]]:
    base, rem = divmod(n, size)
    out, lo = [], 0
    for r in range(size):
        m = base + (1 if r < rem else 0)
        out.append((lo, m))
        lo += m
    return out


def decompose(gnx: int, gny: int, gnz: int, rank: int, size: int, halo: int = 1) -> Slab:
    axis = 2 if gnz > 1 else 1
    n = gnz if axis == 2 else gny
    if size > n // max(1, halo):
        raise ValueError(f"cannot split {n} planes over {size} ranks with halo {halo}")
    lo, m = split(n, size)[rank]
    return Slab(gnx, gny, gnz, axis, rank, size, lo, m)
