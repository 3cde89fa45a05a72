"""MRT and cumulant collisions against independent NumPy oracles (no code shared with the emitter):

* d2q9 (reference models/flow/d2q9/Dynamics.c.Rt:8-24 weighted-orthogonal basis): the
  collision relaxes the Hermite subspaces of the non-equilibrium part — order 2 with S2,
  order 3 with S3, order 4 with S4 — around the standard second-order equilibrium;
* d3q19 (reference src/lib/d3q19.R:24-63, models/flow/d3q19/Dynamics.c.Rt:240-262):
  d'Humieres' orthogonal basis built here from its polynomials, the equilibrium moments
  from the reference's moment-matching definition (<c^p> = rho prod(u_d | u_d^2 + 1/3),
  truncated below third order in J) solved numerically, relaxation 1 - omega on the
  even moments and the "magic" 1 - 8(2 - omega)/(8 - omega) on q and m, body force
  added to J between the two equilibria;
* d3q27_cumulant (reference models/flow/d3q27_cumulant/Dynamics.c.Rt): cumulants of the
  normalised distribution from the Leonov-Shiryaev set-partition formulas (not the
  emitter's sympy log-expansion), second order relaxed with the Galilean correction,
  third order with 1 - Omega, higher orders dropped, body force on the first order.

One step on a periodic box of random non-equilibrium populations: pull streaming
(np.roll) then the oracle collision.  The CPU executor runs here; the same check on the
HIP kernels is marked gpu."""
import itertools

import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice


def _one_step(model, shape, device, settings, seed=0):
    lat = Lattice(model, shape, device=torch.device(device))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint32)
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    dens = [d for d in m.densities if d.field.group == "f"]
    C = np.array([[d.dx, d.dy, d.dz] for d in dens], dtype=float)
    idx = [m.fields.index(d.field) for d in dens]
    c2 = (C ** 2).sum(1)
    f0 = lat.fields_interior().clone()
    rng = np.random.default_rng(seed)
    pert = torch.as_tensor(rng.uniform(-1e-2, 1e-2, f0[idx].shape), dtype=f0.dtype, device=f0.device)
    f0[idx] = f0[idx] * (1 + pert)
    lat.set_fields_interior(f0)
    lat.iterate(1)
    f1 = lat.fields_interior()[idx].cpu().numpy()
    fin = f0[idx].cpu().numpy()
    pulled = np.stack([np.roll(fin[i], (int(C[i, 2]), int(C[i, 1]), int(C[i, 0])), axis=(0, 1, 2))
                       for i in range(len(idx))])
    return lat, C, c2, pulled, f1


# ---------------------------------------------------------------- d2q9
def _d2q9_oracle(C, pulled, s2, s3, s4, g):
    cx, cy = C[:, 0], C[:, 1]
    w = np.where((C ** 2).sum(1) == 0, 4 / 9, np.where((C ** 2).sum(1) == 1, 1 / 9, 1 / 36))
    rho = pulled.sum(0)
    j = np.stack([np.tensordot(cx, pulled, 1), np.tensordot(cy, pulled, 1)])

    def feq(rho, j):
        u = j / rho
        cu = cx[:, None, None, None] * u[0] + cy[:, None, None, None] * u[1]
        return w[:, None, None, None] * rho * (1 + 3 * cu + 4.5 * cu ** 2 - 1.5 * (u ** 2).sum(0))

    herm = {2: [cx * cx - 1 / 3, cy * cy - 1 / 3, cx * cy], 3: [cx * cx * cy - cy / 3, cx * cy * cy - cx / 3],
            4: [(cx * cx - 1 / 3) * (cy * cy - 1 / 3)]}
    neq = pulled - feq(rho, j)
    out = feq(rho, j + rho * np.asarray(g).reshape(2, 1, 1, 1))
    for order, s in ((2, s2), (3, s3), (4, s4)):
        for h in herm[order]:
            a = np.tensordot(h, neq, 1) / np.sum(w * h * h)
            out = out + s * w[:, None, None, None] * h[:, None, None, None] * a[None]
    return out


def _check_d2q9(device):
    nu = 0.05
    om = 1 / (3 * nu + 0.5)
    lat, C, c2, pulled, f1 = _one_step("d2q9", (10, 7, 1), device,
                                       dict(Viscosity=nu, S3=0.3, S4=-0.2, GravitationX=2e-5, GravitationY=-1e-5))
    ora = _d2q9_oracle(C, pulled, 1 - om, 0.3, -0.2, (2e-5, -1e-5))
    assert np.abs(ora - f1).max() < 1e-14, np.abs(ora - f1).max()


# ---------------------------------------------------------------- d3q19
def _d3q19_oracle(C, pulled, omega, force):
    c2 = (C ** 2).sum(1)
    cx, cy, cz = C.T
    rows = {"rho": c2 * 0 + 1, "e": 19 * c2 - 30, "eps": (21 * c2 ** 2 - 53 * c2 + 24) / 2,
            "jx": cx, "qx": (5 * c2 - 9) * cx, "jy": cy, "qy": (5 * c2 - 9) * cy, "jz": cz, "qz": (5 * c2 - 9) * cz,
            "pxx": 3 * cx ** 2 - c2, "Pxx": (3 * c2 - 5) * (3 * cx ** 2 - c2), "pww": cy ** 2 - cz ** 2,
            "Pww": (3 * c2 - 5) * (cy ** 2 - cz ** 2), "pxy": cx * cy, "pyz": cy * cz, "pxz": cx * cz,
            "mx": (cy ** 2 - cz ** 2) * cx, "my": (cz ** 2 - cx ** 2) * cy, "mz": (cx ** 2 - cy ** 2) * cz}
    names = list(rows)
    M = np.array([rows[n] for n in names])
    g1 = 1 - omega
    g2 = 1 - 8 * (2 - omega) / (8 - omega)
    G = np.array([0.0 if n in ("rho", "jx", "jy", "jz") else (g2 if n[0] in "qm" else g1) for n in names])
    P = np.where(C < 0, 2, C).astype(int)
    Wm = np.array([[np.prod([C[k, d] ** P[i, d] for d in range(3)]) for i in range(19)] for k in range(19)])
    Winv = np.linalg.inv(Wm.T)

    def feq(rho, j):
        u = j / rho
        H = []
        for i in range(19):
            ones = [d for d in range(3) if P[i, d] == 1]
            twos = [d for d in range(3) if P[i, d] == 2]
            base = rho * np.prod([u[d] for d in ones], axis=0) if ones else rho
            tot = np.zeros_like(rho)
            for k in range(len(twos) + 1):
                if len(ones) + 2 * k > 2:         # truncated below third order in J
                    break
                for sub in itertools.combinations(twos, k):
                    term = base * (1 / 3) ** (len(twos) - k)
                    for d in sub:
                        term = term * u[d] ** 2
                    tot = tot + term
            H.append(tot)
        return np.tensordot(Winv, np.stack(H), 1)

    rho = pulled.sum(0)
    j = np.tensordot(C.T, pulled, 1)
    mom = np.tensordot(M, pulled, 1)
    meq0 = np.tensordot(M, feq(rho, j), 1)
    meq1 = np.tensordot(M, feq(rho, j + rho * np.asarray(force).reshape(3, 1, 1, 1)), 1)
    post = meq1 + G.reshape(-1, 1, 1, 1) * (mom - meq0)
    return np.tensordot(np.linalg.inv(M), post, 1)


def _check_d3q19(device):
    nu = 0.07
    force = (1e-4, -2e-4, 3e-5)
    lat, C, c2, pulled, f1 = _one_step("d3q19", (6, 5, 4), device,
                                       dict(nu=nu, ForceX=force[0], ForceY=force[1], ForceZ=force[2]), seed=1)
    ora = _d3q19_oracle(C, pulled, 1 / (3 * nu + 0.5), force)
    assert np.abs(ora - f1).max() < 1e-14, np.abs(ora - f1).max()


def test_d2q9_mrt_hermite_oracle_cpu():
    _check_d2q9("cpu")


def test_d3q19_mrt_dhumieres_oracle_cpu():
    _check_d3q19("cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_d2q9_mrt_hermite_oracle_gpu():
    _check_d2q9("cuda")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_d3q19_mrt_dhumieres_oracle_gpu():
    _check_d3q19("cuda")


# ---------------------------------------------------------------- d3q27 cumulant
def _set_partitions(items):
    if not items:
        yield []
        return
    first, rest = items[0], items[1:]
    for part in _set_partitions(rest):
        for i in range(len(part)):
            yield part[:i] + [[first] + part[i]] + part[i + 1:]
        yield [[first]] + part


def _blocks(k):
    """set partitions of the multiset x^a y^b z^c, each block as its (a, b, c) counts"""
    labels = [0] * k[0] + [1] * k[1] + [2] * k[2]
    out = []
    for part in _set_partitions(list(range(len(labels)))):
        out.append([tuple(sum(1 for p in B if labels[p] == d) for d in range(3)) for B in part])
    return out


def _cumulant_oracle(C, pulled, nu, omega3, force):
    """Leonov-Shiryaev partition formulas between the moments and the cumulants of the
    normalised distribution (no shared code with emit/cumulants.py); the relaxation
    follows the reference models/flow/d3q27_cumulant/Dynamics.c.Rt (second order with
    Galilean correction, third order with 1 - Omega, higher orders dropped)."""
    from math import factorial
    keys = [(a, b, c) for c in range(3) for b in range(3) for a in range(3)]
    V = np.array([[np.prod([C[i, d] ** k[d] for d in range(3)]) for i in range(27)] for k in keys])
    m = np.tensordot(V, pulled, 1)
    rho = m[0]
    mu = {k: m[n] / rho for n, k in enumerate(keys)}
    kap = {}
    for k in keys[1:]:
        tot = 0
        for part in _blocks(k):
            n = len(part)
            term = (-1) ** (n - 1) * factorial(n - 1)
            for b in part:
                term = term * mu[b]
            tot = tot + term
        kap[k] = tot
    w0, w1 = 1 / (3 * nu + 0.5), 1.0
    fx, fy, fz = force
    ux, uy, uz = kap[(1, 0, 0)] + fx / (2 * rho), kap[(0, 1, 0)] + fy / (2 * rho), kap[(0, 0, 1)] + fz / (2 * rho)
    c200, c020, c002 = kap[(2, 0, 0)], kap[(0, 2, 0)], kap[(0, 0, 2)]
    dxu = -w0 / 2 * (2 * c200 - c020 - c002) - w1 / 2 * (c200 + c020 + c002 - 1)
    dyv = dxu + 3 * w0 / 2 * (c200 - c020)
    dzw = dxu + 3 * w0 / 2 * (c200 - c002)
    g1 = 3 * (1 - w0 / 2) * (ux * ux * dxu - uy * uy * dyv)
    g2 = 3 * (1 - w0 / 2) * (ux * ux * dxu - uz * uz * dzw)
    g3 = 3 * (1 - w1 / 2) * (ux * ux * dxu + uy * uy * dyv + uz * uz * dzw)
    a = (1 - w0) * (c200 - c020) - g1
    b = (1 - w0) * (c200 - c002) - g2
    cc = w1 + (1 - w1) * (c200 + c020 + c002) - g3
    new = {}
    for k in keys[1:]:
        o = sum(k)
        if o == 1:
            new[k] = kap[k] + {(1, 0, 0): fx, (0, 1, 0): fy, (0, 0, 1): fz}[k]
        elif o == 2 and max(k) == 1:
            new[k] = kap[k] * (1 - w0)
        elif o == 3:
            new[k] = kap[k] * (1 - omega3)
        elif o > 3:
            new[k] = np.zeros_like(rho)
    new[(2, 0, 0)] = (a + b + cc) / 3
    new[(0, 2, 0)] = (cc - 2 * a + b) / 3
    new[(0, 0, 2)] = (cc - 2 * b + a) / 3
    mpost = [rho]
    for k in keys[1:]:
        tot = 0
        for part in _blocks(k):
            term = 1
            for b_ in part:
                term = term * new[b_]
            tot = tot + term
        mpost.append(rho * tot)
    return np.tensordot(np.linalg.inv(V), np.stack(mpost), 1)


def _check_cumulant(device):
    nu, om3, force = 0.03, 0.7, (2e-5, -1e-5, 3e-5)
    lat, C, c2, pulled, f1 = _one_step("d3q27_cumulant", (6, 5, 4), device,
                                       dict(nu=nu, Omega=om3, ForceX=force[0], ForceY=force[1], ForceZ=force[2]), seed=2)
    ora = _cumulant_oracle(C, pulled, nu, om3, force)
    assert np.abs(ora - f1).max() < 1e-14, np.abs(ora - f1).max()


def test_d3q27_cumulant_partition_oracle_cpu():
    _check_cumulant("cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_d3q27_cumulant_partition_oracle_gpu():
    _check_cumulant("cuda")
