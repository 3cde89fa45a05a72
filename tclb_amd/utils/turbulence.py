"""Synthetic turbulence: random Fourier modes with a von Karman spectrum.

Host side of the reference SyntheticTurbulence (src/SyntheticTurbulence.cpp:7-133):
rank 0 draws the modes (wave vector direction, amplitude vector orthogonal to it,
wave number), broadcasts them, and the device evaluates
  u(x) = sum_i sin(k_i.x) a_i + cos(k_i.x) (k_i x a_i)
in every model's ``SyntheticTurbulence(x,y,z)`` (modes in Launch.ext[0])."""
from __future__ import annotations

import math

import numpy as np


class SyntheticTurbulence:
    def __init__(self, seed: int = 0):
        self.modes = np.zeros((0, 7))
        self.time_wn = 0.0
        self.rng = np.random.default_rng(seed)

    def _generate(self, amplitudes, wavenumbers, comm=None):
        n = len(amplitudes)
        data = np.zeros((n, 7))
        for j in range(n):
            t = self.rng.standard_normal(6)
            t[:3] /= np.linalg.norm(t[:3])
            t[3:] -= t[:3] * np.dot(t[:3], t[3:])
            t[3:] *= amplitudes[j] / np.linalg.norm(t[3:])
            data[j, :6] = t
            data[j, 6] = wavenumbers[j]
        if comm is not None:
            data = comm.bcast_object(data, 0)
        self.modes = data
        return data

    def set_von_karman(self, n: int, main_wn: float, diff_wn: float, min_wn: float, max_wn: float, comm=None):
        """reference setVonKarman (Le, Ld, Lmin, Lmax are wave numbers here)"""
        Le, Ld = main_wn, diff_wn
        dL = (max_wn - min_wn) / n
        L = np.arange(n) * dL + dL / 2 + min_wn
        c = 1.453
        E = c / Le * (L / Le) ** 4 / (1.0 + (L / Le) ** 2) ** (17. / 6.) * np.exp(-2.0 * (L / Ld) ** 2)
        amp = np.sqrt(E * dL)
        self.energy_fraction = float((amp ** 2).sum())
        return self._generate(amp, L, comm)

    def set_one_wave(self, wn: float, comm=None):
        return self._generate(np.array([1.0]), np.array([wn]), comm)

    def evaluate(self, x, y, z):
        """host evaluation (tests)"""
        r = np.zeros(3)
        for m in self.modes:
            w = (m[0] * x + m[1] * y + m[2] * z) * m[6]
            a, k = m[3:6], m[0:3]
            r += math.sin(w) * a + math.cos(w) * np.cross(k, a)
        return r
