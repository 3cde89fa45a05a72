"""VTK ImageData output (.vti per rank + .pvti index on rank 0).

Same layout as the reference writer (reference: src/vtkOutput.cpp:54-200,
src/vtkLattice.cpp:9-54): CellData, inline base64 binary with a separately encoded
UInt32 byte-count header, one piece per rank, flag groups written as UInt8 fields
(value >> shift), quantities scaled back to SI units."""
from __future__ import annotations

import base64
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

_VTK_T = {np.dtype(np.float64): "Float64", np.dtype(np.float32): "Float32", np.dtype(np.uint8): "UInt8",
          np.dtype(np.uint16): "UInt16", np.dtype(np.uint32): "UInt32", np.dtype(np.int32): "Int32"}


def _b64(a: np.ndarray) -> str:
    data = np.ascontiguousarray(a).tobytes()
    return (base64.b64encode(np.uint32(len(data)).tobytes()) + base64.b64encode(data)).decode()


def extent(reg) -> str:
    x0, y0, z0, nx, ny, nz = reg
    return f"{x0} {x0 + nx} {y0} {y0 + ny} {z0} {z0 + nz}"


def write_vti(path: str, total_reg, reg, fields: List[Tuple[str, np.ndarray, int]], spacing: float = 1.0,
              origin=(0.0, 0.0, 0.0)):
    """fields: (name, array (nz,ny,nx) or (ncomp,nz,ny,nx), ncomp)"""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        f.write('<?xml version="1.0"?>\n<VTKFile type="ImageData" version="0.1" byte_order="LittleEndian">\n')
        f.write(f'<ImageData WholeExtent="{extent(reg)}" Origin="{origin[0]:g} {origin[1]:g} {origin[2]:g}" '
                f'Spacing="{spacing:g} {spacing:g} {spacing:g}">\n')
        f.write(f'<Piece Extent="{extent(reg)}">\n<CellData Scalars="rho" Vectors="velocity">\n')
        for name, arr, nc in fields:
            a = np.asarray(arr)
            if nc > 1:
                a = np.moveaxis(a, 0, -1)  # (nz,ny,nx,nc) interleaved components
            t = _VTK_T[a.dtype]
            f.write(f'<DataArray type="{t}" Name="{name}" format="binary" encoding="base64" '
                    f'NumberOfComponents="{nc}">\n')
            f.write(_b64(a))
            f.write("\n</DataArray>\n")
        f.write("</CellData>\n</Piece>\n</ImageData>\n</VTKFile>\n")


def write_pvti(path: str, total_reg, pieces: Sequence[Tuple[tuple, str]], fields: List[Tuple[str, str, int]],
               spacing: float = 1.0, origin=(0.0, 0.0, 0.0)):
    with open(path, "w") as f:
        f.write('<?xml version="1.0"?>\n<VTKFile type="PImageData" version="0.1" byte_order="LittleEndian">\n')
        f.write(f'<PImageData WholeExtent="{extent(total_reg)}" Origin="{origin[0]:g} {origin[1]:g} {origin[2]:g}" '
                f'Spacing="{spacing:g} {spacing:g} {spacing:g}">\n')
        for reg, src in pieces:
            f.write(f'<Piece Extent="{extent(reg)}" Source="{src}"/>\n')
        f.write('<PCellData Scalars="rho" Vectors="velocity">\n')
        for name, t, nc in fields:
            f.write(f'<PDataArray type="{t}" Name="{name}" NumberOfComponents="{nc}"/>\n')
        f.write("</PCellData>\n</PImageData>\n</VTKFile>\n")


def read_vti(path: str) -> Dict[str, np.ndarray]:
    """Minimal reader for our own .vti files (tests / compare tool)."""
    import xml.etree.ElementTree as ET
    root = ET.parse(path).getroot()
    piece = root.find("ImageData/Piece")
    e = [int(v) for v in piece.get("Extent").split()]
    nx, ny, nz = e[1] - e[0], e[3] - e[2], e[5] - e[4]
    out = {}
    inv = {v: k for k, v in _VTK_T.items()}
    for da in piece.find("CellData"):
        t = inv[da.get("type")]
        nc = int(da.get("NumberOfComponents", "1"))
        txt = da.text.strip()
        hdr = base64.b64decode(txt[:8])
        n = int(np.frombuffer(hdr, dtype=np.uint32)[0])
        data = base64.b64decode(txt[8:])[:n]
        a = np.frombuffer(data, dtype=t)
        a = a.reshape(nz, ny, nx, nc) if nc > 1 else a.reshape(nz, ny, nx)
        out[da.get("Name")] = a
    return out


def read_pvti(path: str) -> Dict[str, np.ndarray]:
    """assemble the pieces of a .pvti index into whole-extent arrays (tests, comparisons
    of runs on different rank counts)"""
    import xml.etree.ElementTree as ET
    root = ET.parse(path).getroot()
    img = root.find("PImageData")
    w = [int(v) for v in img.get("WholeExtent").split()]
    out: Dict[str, np.ndarray] = {}
    base = os.path.dirname(path)
    for piece in img.findall("Piece"):
        e = [int(v) for v in piece.get("Extent").split()]
        data = read_vti(os.path.join(base, piece.get("Source")))
        for name, a in data.items():
            if name not in out:
                shape = (w[5] - w[4], w[3] - w[2], w[1] - w[0]) + a.shape[3:]
                out[name] = np.zeros(shape, dtype=a.dtype)
            out[name][e[4] - w[4]:e[5] - w[4], e[2] - w[2]:e[3] - w[2], e[0] - w[0]:e[1] - w[0]] = a
    return out
