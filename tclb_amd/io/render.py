"""Colour frames of a lattice slice: the headless counterpart of the reference's GLUT
window (src/gpu_anim.h; Solver::RunMainLoop, src/Solver.cpp.Rt:404-427), which shows
LatticeContainer::Color — every node's ``Color()`` (value l, weight w) of the middle z
slice through a fixed colour map (NodeToColor, src/LatticeContainer.inc.cpp.Rt:350-402).

Here the node colour pair comes from the model's emitted ``color()`` member, evaluated by
the quantity kernel over one z slice (``Lattice.color``); the colour map runs as a few
tensor ops on the lattice's device, and the image is written as PNG by the native writer
(csrc/runtime/png.cpp).  The window's mouse editing (walls drawn where the pointer moves)
is ``Lattice.draw_wall``.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


def colormap(l: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """RGBA uint8 of node values l and weights w (the reference NodeToColor map): l is
    scaled by 111; blue shades below 0, red -> yellow -> white above, saturating at
    +-111 (white); the weight blends towards green (w = 0: solid); NaN/inf is magenta"""
    l = l.to(torch.float32)
    w = w.to(torch.float32)
    s = l * 111.0
    r = torch.zeros_like(s)
    g = torch.zeros_like(s)
    b = torch.zeros_like(s)

    def put(mask, rv, gv, bv):
        nonlocal r, g, b
        r = torch.where(mask, rv, r)
        g = torch.where(mask, gv, g)
        b = torch.where(mask, bv, b)

    full = torch.full_like(s, 255.0)
    zero = torch.zeros_like(s)
    # integer arithmetic of the reference (int r = 255*(...)/100): truncation
    put(s < -111, full, full, full)
    put((s >= -111) & (s < -11), torch.trunc(255 * (-s - 11) / 100), full, full)
    put((s >= -11) & (s < -1), zero, torch.trunc(255 * (-s - 1) / 10), full)
    put((s >= -1) & (s < 0), zero, zero, torch.trunc(255 * (-s)))
    put((s >= 0) & (s < 1), torch.trunc(255 * s), zero, zero)
    put((s >= 1) & (s < 11), full, torch.trunc(255 * (s - 1) / 10), zero)
    put((s >= 11) & (s < 111), full, full, torch.trunc(255 * (s - 11) / 100))
    put(s >= 111, full, full, full)
    r = torch.trunc(r * w)
    g = torch.trunc(g * w + (1 - w) * 255)
    b = torch.trunc(b * w)
    bad = ~torch.isfinite(s)
    r = torch.where(bad, full, r)
    g = torch.where(bad, zero, g)
    b = torch.where(bad, full, b)
    a = torch.full_like(s, 255.0)
    return torch.stack([r, g, b, a], dim=-1).clamp(0, 255).to(torch.uint8)


def frame(lat, z: Optional[int] = None) -> Optional[np.ndarray]:
    """(ny, nx, 4) uint8 image of global slice z (default: the middle one, as the
    reference), top row = largest y (the window's orientation); every rank calls it, the
    root gets the image (None on the others)"""
    lw = lat.color(z)                                  # (ny_local, nx, 2) or None
    img = None if lw is None else colormap(lw[..., 0], lw[..., 1]).cpu().numpy()
    y0 = lat.slab.offset[1] if img is not None else 0
    pieces = lat.comm.gather_to_root((y0, img))
    if lat.comm.rank != 0:
        return None
    gnx, gny = lat.gshape[0], lat.gshape[1]
    out = np.zeros((gny, gnx, 4), dtype=np.uint8)
    for y, p in pieces:
        if p is not None:
            out[y:y + p.shape[0], :p.shape[1]] = p
    return out[::-1].copy()


def write_png(lat, path: str, z: Optional[int] = None) -> Optional[np.ndarray]:
    """write the colour frame of slice z to `path` (root rank); returns the image"""
    from ..ops.host import png_write
    img = frame(lat, z)
    if img is not None:
        png_write(path, img)
    return img
