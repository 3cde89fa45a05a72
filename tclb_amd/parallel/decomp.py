"""Domain decomposition.

The reference searches a 2-D Y x Z process grid minimising the cut surface
(reference: src/Solver.cpp.Rt:288-370, MPIDivision) and never splits X.  On one
MI355X node the 8 GPUs are a fully connected xGMI mesh with one dedicated link per
GPU pair, so a 1-D slab split along the slowest axis (z in 3-D, y in 2-D) is the
default: every rank talks to exactly two neighbours over two independent links, each
halo is one contiguous plane per field, and the border/interior split overlaps the
exchange with the interior kernel.  X is never split (as in the reference).

When the slab axis is too thin for the rank count (size > n / halo, e.g. flat
1280x130x130 domains on many ranks), or when a grid is requested explicitly, a 3-D
lattice is split over a Y x Z grid (``axis == 3``) chosen like MPIDivision: the grid
with the smallest total cut surface whose blocks are at least one halo thick.  Its
halos are exchanged in two phases (z planes, then y rows including the z ghosts, which
fills the edge ghosts), without the overlap split.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple


@dataclass
class Slab:
    gnx: int
    gny: int
    gnz: int
    axis: int          # 1 = y slab, 2 = z slab, 3 = Y x Z grid
    rank: int
    size: int
    lo: int            # global start along the slab axis (axis 1/2)
    n: int             # local extent along the slab axis (axis 1/2)
    # Y x Z grid (axis 3): rank = ry + py * rz; local block [ylo, ylo+ny) x [zlo, zlo+nz)
    py: int = 1
    pz: int = 1
    ry: int = 0
    rz: int = 0
    ylo: int = 0
    ny: int = 0
    zlo: int = 0
    nz: int = 0

    @property
    def local_shape(self) -> Tuple[int, int, int]:
        if self.axis == 3:
            return self.gnx, self.ny, self.nz
        if self.axis == 2:
            return self.gnx, self.gny, self.n
        return self.gnx, self.n, self.gnz

    @property
    def offset(self) -> Tuple[int, int, int]:
        if self.axis == 3:
            return 0, self.ylo, self.zlo
        return (0, self.lo, 0) if self.axis == 1 else (0, 0, self.lo)

    def neighbours(self, axis: int) -> Tuple[int, int]:
        """(previous, next) rank along y (axis 1) or z (axis 2), periodic"""
        if self.axis != 3:
            return (self.rank - 1) % self.size, (self.rank + 1) % self.size
        if axis == 1:
            return ((self.ry - 1) % self.py) + self.py * self.rz, ((self.ry + 1) % self.py) + self.py * self.rz
        return self.ry + self.py * ((self.rz - 1) % self.pz), self.ry + self.py * ((self.rz + 1) % self.pz)


def split(n: int, size: int) -> List[Tuple[int, int]]:
    base, rem = divmod(n, size)
    out, lo = [], 0
    for r in range(size):
        m = base + (1 if r < rem else 0)
        out.append((lo, m))
        lo += m
    return out


def choose_grid(gnx: int, gny: int, gnz: int, size: int, hy: int = 1, hz: int = 1) -> Optional[Tuple[int, int]]:
    """(py, pz) with py * pz = size minimising the cut surface (py-1) nx nz + (pz-1) nx ny
    (reference MPIDivision), blocks at least one halo thick; None if no grid fits"""
    best = None
    for py in range(1, size + 1):
        if size % py:
            continue
        pz = size // py
        if gny // py < max(1, hy) or gnz // pz < max(1, hz):
            continue
        cut = (py - 1) * gnx * gnz + (pz - 1) * gnx * gny
        if best is None or cut < best[0]:
            best = (cut, py, pz)
    return None if best is None else (best[1], best[2])


def decompose(gnx: int, gny: int, gnz: int, rank: int, size: int, halo: int = 1,
              grid: Optional[Tuple[int, int]] = None, halo_y: Optional[int] = None) -> Slab:
    """1-D slab (default) or, for 3-D lattices, a Y x Z grid when ``grid=(py, pz)`` is
    given or the slab would be thinner than the halo"""
    axis = 2 if gnz > 1 else 1
    n = gnz if axis == 2 else gny
    hy = halo if halo_y is None else halo_y
    if grid is None and size <= n // max(1, halo):
        lo, m = split(n, size)[rank]
        return Slab(gnx, gny, gnz, axis, rank, size, lo, m)
    if gnz == 1:
        raise ValueError(f"cannot split {n} rows over {size} ranks with halo {halo}")
    if grid is None:
        grid = choose_grid(gnx, gny, gnz, size, hy, halo)
        if grid is None:
            raise ValueError(f"no Y x Z grid of {size} ranks fits {gny}x{gnz} with halo {halo}")
    py, pz = grid
    if py * pz != size:
        raise ValueError(f"grid {py}x{pz} does not match {size} ranks")
    if (pz == 1 or py == 1) and size > 1:   # degenerate grid: a slab along the split axis
        ax = 2 if py == 1 else 1
        nn = gnz if ax == 2 else gny
        lo, m = split(nn, size)[rank]
        return Slab(gnx, gny, gnz, ax, rank, size, lo, m)
    ry, rz = rank % py, rank // py
    ylo, ny = split(gny, py)[ry]
    zlo, nz = split(gnz, pz)[rz]
    if ny < max(1, hy) or nz < max(1, halo):
        raise ValueError(f"grid {py}x{pz} blocks thinner than the halo")
    return Slab(gnx, gny, gnz, 3, rank, size, 0, 0, py, pz, ry, rz, ylo, ny, zlo, nz)
