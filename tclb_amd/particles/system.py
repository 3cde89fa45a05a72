"""Particle system + built-in rigid-sphere integrator (reference simplepart.cpp)."""
from __future__ import annotations

import math
import os
from typing import List, Optional

import numpy as np
import torch

PART_STRIDE = 10


class ParticleSystem:
    """Particles in lattice units (positions in node coordinates)."""

    def __init__(self, n: int = 0):
        self.x = np.zeros((n, 3))
        self.v = np.zeros((n, 3))
        self.omega = np.zeros((n, 3))
        self.r = np.zeros(n)
        self.m = np.zeros(n)
        self.force = np.zeros((n, 3))
        self.torque = np.zeros((n, 3))
        self.fixed = np.zeros(n, dtype=bool)
        self._dev = None
        self._acc = None
        self._grid = None
        self.grid_min = 16          # particles; below this every node scans the full list

    @property
    def n(self) -> int:
        return len(self.r)

    def add(self, x, r, v=(0, 0, 0), omega=(0, 0, 0), m=None, fixed=False):
        self.x = np.vstack([self.x, np.asarray(x, float)[None]])
        self.v = np.vstack([self.v, np.asarray(v, float)[None]])
        self.omega = np.vstack([self.omega, np.asarray(omega, float)[None]])
        self.r = np.append(self.r, float(r))
        self.m = np.append(self.m, float(m) if m else 4.0 / 3.0 * math.pi * r ** 3)
        self.force = np.vstack([self.force, np.zeros((1, 3))])
        self.torque = np.vstack([self.torque, np.zeros((1, 3))])
        self.fixed = np.append(self.fixed, bool(fixed))

    # -- lattice hooks --------------------------------------------------------------
    def pre_stage(self, lat):
        rec = np.zeros((max(1, self.n), PART_STRIDE))
        if self.n:
            rec[:self.n, 0:3] = self.x
            rec[:self.n, 3:6] = self.v
            rec[:self.n, 6:9] = self.omega
            rec[:self.n, 9] = self.r
        self._dev = torch.as_tensor(rec).to(lat.device)
        self._acc = torch.zeros((max(1, self.n), 6), dtype=torch.float64, device=lat.device)
        L = lat._L
        L.ext[2] = self._dev.data_ptr()
        L.ext[3] = self._acc.data_ptr()
        L.next[2] = self.n
        # solid container: uniform grid (reference default SolidGrid) once the linear scan
        # over all particles per node stops being cheap
        self._grid = None
        if self.n >= self.grid_min:
            from ..ops.host import solid_grid
            cell = int(np.ceil(self.r[:self.n].max() + 2.0)) if self.n else 1
            g = solid_grid(rec[:self.n], lat.gshape, cell)
            self._grid = torch.as_tensor(g).to(lat.device)
            L.ext[4] = self._grid.data_ptr()
            L.next[4] = self._grid.numel()
        else:
            L.ext[4] = None
            L.next[4] = 0

    def post_stage(self, lat):
        acc = self._acc
        if lat.comm.distributed and lat.comm.size > 1:
            acc = lat.comm.allreduce_globals(acc.reshape(-1).clone(), acc.numel()).reshape(acc.shape)
        a = acc.cpu().numpy()[:self.n]
        self.force = a[:, 0:3].copy()
        self.torque = a[:, 3:6].copy()
        self.detach(lat)

    def detach(self, lat):
        """drop the particle records from the launch (after a stage or a quantity)"""
        lat._L.next[2] = 0
        lat._L.ext[4] = None
        lat._L.next[4] = 0

    def step(self, lat):
        """advance after the particle stage of one iteration"""


def integrate_rigid(x, v, omega, r, m, fixed, force, torque, acc, periodic, period):
    """one explicit step of free rigid spheres (reference simplepart.cpp), in place; shared
    by the in-process SimplePart and the remote integrator tools/rfi_simplepart.py"""
    for i in range(len(r)):
        if fixed[i]:
            continue
        I = 0.4 * m[i] * r[i] ** 2
        v[i] += force[i] / m[i] + acc
        x[i] += v[i]
        omega[i] += torque[i] / I
        for d in range(3):
            if periodic[d] and period[d] > 0:
                x[i, d] %= period[d]


class SimplePart(ParticleSystem):
    """Built-in rigid spheres (reference simplepart: explicit integration, optional
    periodicity, constant acceleration, logging)."""

    def __init__(self):
        super().__init__(0)
        self.acc = np.zeros(3)
        self.periodic = np.zeros(3, dtype=bool)
        self.period = np.zeros(3)
        self.log_path: Optional[str] = None
        self.log_every = 1
        self.log_rotation = False
        self.logged: List[int] = []
        self.iteration = 0

    def step(self, lat):
        self.iteration += 1
        integrate_rigid(self.x, self.v, self.omega, self.r, self.m, self.fixed, self.force, self.torque, self.acc,
                        self.periodic, self.period)
        if self.log_path and self.iteration % self.log_every == 0 and lat.comm.rank == 0:
            self._log()

    def _log(self):
        new = not os.path.exists(self.log_path)
        with open(self.log_path, "a") as f:
            if new:
                cols = ["Iteration"]
                for i in self.logged:
                    cols += [f"p{i}_{c}{a}" for c in ("", "v", "f") for a in "xyz"]
                    if self.log_rotation:
                        cols += [f"p{i}_{c}{a}" for c in ("o", "t") for a in "xyz"]
                f.write(",".join(cols) + "\n")
            row = [str(self.iteration)]
            for i in self.logged:
                for arr in (self.x, self.v, self.force):
                    row += [f"{v:.10e}" for v in arr[i]]
                if self.log_rotation:
                    for arr in (self.omega, self.torque):
                        row += [f"{v:.10e}" for v in arr[i]]
            f.write(",".join(row) + "\n")
