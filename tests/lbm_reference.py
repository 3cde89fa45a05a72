"""Plain-PyTorch reference implementations of the LBM operators (oracle for the
HIP/CPU kernels).  Independent of the emitter: velocity sets, weights, pull
streaming (torch.roll) and BGK/second-order equilibrium written directly."""
import numpy as np
import torch

U27 = np.array([[x, y, z] for z in (-1, 0, 1) for y in (-1, 0, 1) for x in (-1, 0, 1)])
W27 = np.array([{0: 8 / 27, 1: 2 / 27, 2: 1 / 54, 3: 1 / 216}[int(np.abs(a).sum())] for a in U27])
U9 = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [-1, 0, 0], [0, -1, 0], [1, 1, 0], [-1, 1, 0], [-1, -1, 0], [1, -1, 0]])
W9 = np.array([4 / 9] + [1 / 9] * 4 + [1 / 36] * 4)


def stream(f, U):
    out = torch.empty_like(f)
    for i, (cx, cy, cz) in enumerate(U):
        out[i] = torch.roll(f[i], shifts=(int(cz), int(cy), int(cx)), dims=(0, 1, 2))
    return out


def feq(rho, J, U, W):
    c = torch.tensor(U, dtype=rho.dtype)
    w = torch.tensor(W, dtype=rho.dtype)
    cj = torch.einsum("qd,dzyx->qzyx", c, J)
    jsq = (J * J).sum(0)
    return w[:, None, None, None] * (rho + 3 * cj + 4.5 * cj * cj / rho - 1.5 * jsq / rho)


def moments(f, U):
    c = torch.tensor(U, dtype=f.dtype)
    return f.sum(0), torch.einsum("qzyx,qd->dzyx", f, c)


def bgk_step(f, omega, U, W, force=(0.0, 0.0, 0.0)):
    fs = stream(f, U)
    rho, J = moments(fs, U)
    fe = feq(rho, J, U, W)
    post_neq = (1 - omega) * (fs - fe)
    F = torch.tensor(force, dtype=f.dtype)[:, None, None, None]
    return feq(rho, J + F, U, W) + post_neq


def bounce_back_mask(f, mask, U):
    """swap opposite populations where mask (z,y,x) is True"""
    idx = {tuple(u): i for i, u in enumerate(U.tolist())}
    opp = [idx[tuple((-np.array(u)).tolist())] for u in U.tolist()]
    g = f.clone()
    g[:, mask] = f[opp][:, mask]
    return g
