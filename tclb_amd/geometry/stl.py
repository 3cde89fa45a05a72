"""STL primitive (reference Geometry::loadSTL / transformSTL, src/Geometry.cpp.Rt:397-688).
Binary STL only; transforms Xrot/Yrot/Zrot, scale, x/y/z; sides in/out (ray parity,
native) and surface (sub-voxel cuts for interpolated bounce-back, native)."""
from __future__ import annotations

import math
import struct

import numpy as np

from ..ops import host


def read_stl(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        header = f.read(80)
        if header[:5] == b"solid":
            raise ValueError(f"'STL' element {path} is not in binary format!")
        (ntri,) = struct.unpack("<i", f.read(4))
        rec = np.dtype([("n", "<f4", 3), ("p", "<f4", (3, 3)), ("attr", "<u2")])
        data = np.frombuffer(f.read(ntri * 50), dtype=rec, count=ntri)
    return data["p"].astype(np.float64).reshape(ntri, 9)


def transform(tri: np.ndarray, node, units) -> np.ndarray:
    P = tri.reshape(-1, 3, 3).copy()
    for d, (a1, a2) in enumerate([(1, 2), (2, 0), (0, 1)]):
        a = node.get("XYZ"[d] + "rot")
        if a is not None:
            v = units.alt(a)
            y = P[:, :, a1].copy()
            z = P[:, :, a2].copy()
            P[:, :, a1] = math.cos(v) * y - math.sin(v) * z
            P[:, :, a2] = math.sin(v) * y + math.cos(v) * z
    if node.get("scale") is not None:
        P *= units.alt(node.get("scale"))
    for d, a in enumerate("xyz"):
        if node.get(a) is not None:
            P[:, :, d] += units.alt(node.get(a))
    sm = np.array([0.1403e-4, 0.1687e-4, 0.1987e-4])
    P = np.round(P * 1e5) * 1e-5 + sm - 0.5
    return P.reshape(-1, 9)


D3Q27_DIRS = np.array([[x, y, z] for z in (0, 1, -1) for y in (0, 1, -1) for x in (0, 1, -1)])[1:]


def draw_stl(geom, reg, node):
    fn = node.get("file")
    if fn is None:
        raise ValueError("No 'file' attribute in 'STL' element")
    side = node.get("side", "in")
    inside_out = {"in": 0, "out": 1, "surface": 2}[side]
    axis = {"x": 0, "y": 1, "z": 2}[node.get("ray_axis", "y")]
    tri = transform(read_stl(fn), node, geom.units)
    r = reg.intersect(geom.total)
    if r.size() == 0:
        return
    box = (r.dx, r.dy, r.dz, r.nx, r.ny, r.nz)
    if inside_out == 2:
        cuts, mask = host.stl_cuts(tri, box, D3Q27_DIRS)
        geom.record_cuts(r, cuts)
        sel = mask.astype(bool)
    else:
        lev = host.stl_fill(tri, box, axis, inside_out)
        sel = (lev % 2) == 1

    def pred(X, Y, Z):
        xi = (X - r.dx).astype(int)
        yi = (Y - r.dy).astype(int)
        zi = (Z - r.dz).astype(int)
        return sel[zi, yi, xi]
    geom.paint(r, pred)
