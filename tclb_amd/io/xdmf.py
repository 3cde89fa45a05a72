"""XDMF + raw binary field output (the HDF5 callback's container when libhdf5 is not
available).  One binary file per output step holds every field of the output region
back to back, each as a C-ordered (nz, ny, nx[, ncomp]) little-endian array; the .xmf
sidecar describes them as cell data on a 3DCoRectMesh."""
from __future__ import annotations

import os
from typing import List, Tuple

import numpy as np

_XT = {"f": "Float", "u": "UInt", "i": "Int"}


def layout(region, meta) -> List[Tuple[str, np.dtype, int, int]]:
    """[(name, dtype, ncomp, byte offset)] for the fields of `region`"""
    _, _, _, nx, ny, nz = region
    out, off = [], 0
    for name, dt, nc in meta:
        dt = np.dtype(dt)
        out.append((name, dt, nc, off))
        off += nx * ny * nz * nc * dt.itemsize
    return out


def total_bytes(region, lay) -> int:
    _, _, _, nx, ny, nz = region
    name, dt, nc, off = lay[-1]
    return off + nx * ny * nz * nc * dt.itemsize


def create(path: str, lay):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "wb"):
        pass


def write_piece(path: str, region, lreg, fields, lay):
    """pwrite this rank's sub-box `lreg` of every field into the shared file"""
    X0, Y0, Z0, NX, NY, NZ = region
    x0, y0, z0, nx, ny, nz = lreg
    fd = os.open(path, os.O_WRONLY)
    try:
        for (name, a, nc), (_, dt, _, off) in zip(fields, lay):
            a = np.asarray(a)
            if nc > 1:
                a = np.moveaxis(a, 0, -1)            # (nz, ny, nx, nc)
            a = np.ascontiguousarray(a.astype(dt.newbyteorder("<"), copy=False))
            for k in range(nz):
                for j in range(ny):
                    gi = ((z0 - Z0 + k) * NY + (y0 - Y0 + j)) * NX + (x0 - X0)
                    os.pwrite(fd, a[k, j].tobytes(), off + gi * nc * dt.itemsize)
    finally:
        os.close(fd)


def write_xmf(path: str, binname: str, region, lay, spacing: float = 1.0, time: float = 0.0, hdf5: bool = False,
              point_data: bool = False):
    """XDMF sidecar; hdf5=True: the DataItems point into an HDF5 file ("file.h5:/Name", as
    the reference's hdf5WriteLattice), else into the raw binary file at byte offsets.
    point_data: the values sit on the mesh points (a mesh of nz x ny x nx points,
    Center="Node"), else on the cells of an (nz+1) x (ny+1) x (nx+1) point mesh
    (reference HDF5_WRITE_POINT, src/hdf5Lattice.cpp:136-141)"""
    X0, Y0, Z0, nx, ny, nz = region
    pd = 0 if point_data else 1
    lines = ['<?xml version="1.0" ?>', '<!DOCTYPE Xdmf SYSTEM "Xdmf.dtd" []>', '<Xdmf Version="2.0">', '<Domain>',
             '<Grid Name="lattice" GridType="Uniform">', f'<Time Value="{time:g}"/>',
             f'<Topology TopologyType="3DCoRectMesh" Dimensions="{nz + pd} {ny + pd} {nx + pd}"/>',
             '<Geometry GeometryType="ORIGIN_DXDYDZ">',
             f'<DataItem Dimensions="3" NumberType="Float" Format="XML">{Z0 * spacing:g} {Y0 * spacing:g} {X0 * spacing:g}</DataItem>',
             f'<DataItem Dimensions="3" NumberType="Float" Format="XML">{spacing:g} {spacing:g} {spacing:g}</DataItem>',
             '</Geometry>']
    for name, dt, nc, off in lay:
        at = "Vector" if nc == 3 else "Scalar"
        dims = f"{nz} {ny} {nx}" + (f" {nc}" if nc > 1 else "")
        if hdf5:
            item = (f'<DataItem Dimensions="{dims}" NumberType="{_XT[dt.kind]}" Precision="{dt.itemsize}" '
                    f'Format="HDF">{binname}:/{name}</DataItem>')
        else:
            item = (f'<DataItem Dimensions="{dims}" NumberType="{_XT[dt.kind]}" Precision="{dt.itemsize}" '
                    f'Endian="Little" Format="Binary" Seek="{off}">{binname}</DataItem>')
        center = "Node" if point_data else "Cell"
        lines += [f'<Attribute Name="{name}" AttributeType="{at}" Center="{center}">', item, '</Attribute>']
    lines += ['</Grid>', '</Domain>', '</Xdmf>']
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def read_field(xmf_path: str, name: str) -> np.ndarray:
    """read one attribute back (tests)"""
    import xml.etree.ElementTree as ET
    root = ET.parse(xmf_path).getroot()
    for at in root.iter("Attribute"):
        if at.get("Name") == name:
            di = at.find("DataItem")
            dims = [int(v) for v in di.get("Dimensions").split()]
            if di.get("Format") == "HDF":
                from .h5read import read_h5
                fn, _, ds = di.text.strip().partition(":/")
                return read_h5(os.path.join(os.path.dirname(xmf_path), fn))[ds].reshape(dims)
            kind = {"Float": "f", "UInt": "u", "Int": "i"}[di.get("NumberType")]
            dt = np.dtype(f"<{kind}{di.get('Precision')}")
            with open(os.path.join(os.path.dirname(xmf_path), di.text.strip()), "rb") as f:
                f.seek(int(di.get("Seek")))
                return np.frombuffer(f.read(int(np.prod(dims)) * dt.itemsize), dtype=dt).reshape(dims)
    raise KeyError(name)
