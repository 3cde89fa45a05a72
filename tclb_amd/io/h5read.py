"""Minimal reader of classic-format HDF5 files (no libhdf5/h5py on the image): enough to
read back the contiguous datasets of the HDF5 output (csrc/runtime/h5.cpp) in tests and
tools.  It walks the structures the HDF5 file-format specification defines — superblock
version 0, the root group's symbol-table entry (v1 B-tree of group nodes + local heap of
names), symbol-table nodes, version-1 object headers with the dataspace (v1), datatype
(fixed/float), filter-pipeline (v1, deflate only) and data-layout (v3 contiguous or chunked,
with the v1 B-tree chunk index) messages — and rejects anything else.

    from tclb_amd.io.h5read import read_h5
    data = read_h5("out_HDF5_00000100.h5")     # {name: numpy array}
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"


class H5FormatError(ValueError):
    pass


def _u(b: bytes, off: int, n: int) -> int:
    return int.from_bytes(b[off:off + n], "little")


def _cstr(b: bytes, off: int) -> str:
    end = b.index(b"\0", off)
    return b[off:end].decode()


def _group_entries(b: bytes, btree: int, heap: int, so: int, sl: int, leaf_k: int) -> List[Tuple[str, int]]:
    if b[heap:heap + 4] != b"HEAP":
        raise H5FormatError("bad local heap signature")
    data = _u(b, heap + 8 + 2 * sl, so)
    out = []

    def node(addr):
        if b[addr:addr + 4] != b"TREE":
            raise H5FormatError("bad B-tree signature")
        ntype, level, used = b[addr + 4], b[addr + 5], _u(b, addr + 6, 2)
        if ntype != 0:
            raise H5FormatError("not a group B-tree")
        p = addr + 8 + 2 * so + sl               # first child pointer (after key 0)
        for i in range(used):
            child = _u(b, p + i * (so + sl), so)
            if level > 0:
                node(child)
                continue
            if b[child:child + 4] != b"SNOD":
                raise H5FormatError("bad symbol-table node signature")
            n = _u(b, child + 6, 2)
            for k in range(n):
                e = child + 8 + k * (2 * so + 24)
                out.append((_cstr(b, data + _u(b, e, so)), _u(b, e + so, so)))
    node(btree)
    return out


def _dataset(b: bytes, oh: int, so: int, sl: int) -> np.ndarray:
    if b[oh] != 1:
        raise H5FormatError("only version-1 object headers are read")
    nmsg, size = _u(b, oh + 2, 2), _u(b, oh + 8, 4)
    p, end = oh + 16, oh + 16 + size
    shape = dtype = layout = chunked = None
    filters: List[int] = []
    for _ in range(nmsg):
        if p >= end:
            break
        mtype, msize = _u(b, p, 2), _u(b, p + 2, 2)
        body = p + 8
        if mtype == 0x1:                           # dataspace
            if b[body] != 1:
                raise H5FormatError("dataspace version")
            rank = b[body + 1]
            shape = tuple(_u(b, body + 8 + k * sl, sl) for k in range(rank))
        elif mtype == 0x3:                         # datatype
            cls, size_b = b[body] & 0x0F, _u(b, body + 4, 4)
            bits0 = b[body + 1]
            if bits0 & 1:
                raise H5FormatError("big-endian data")
            if cls == 0:
                dtype = np.dtype(("<i" if bits0 & 0x08 else "<u") + str(size_b))
            elif cls == 1:
                dtype = np.dtype("<f" + str(size_b))
            else:
                raise H5FormatError(f"datatype class {cls}")
        elif mtype == 0xB:                         # filter pipeline
            if b[body] != 1:
                raise H5FormatError("filter pipeline version")
            q = body + 8
            for _ in range(b[body + 1]):
                fid, nlen, _flags, nval = (_u(b, q + 2 * k, 2) for k in range(4))
                if fid != 1:
                    raise H5FormatError(f"filter {fid} (only deflate is read)")
                q += 8 + ((nlen + 7) // 8) * 8 + 4 * nval + (4 if nval % 2 else 0)
                filters.append(fid)
        elif mtype == 0x8:                         # data layout
            if b[body] != 3 or b[body + 1] not in (1, 2):
                raise H5FormatError("only contiguous or chunked layout v3")
            if b[body + 1] == 1:
                layout = (_u(b, body + 2, so), _u(b, body + 2 + so, sl))
            else:
                nd = b[body + 2]
                chunked = (_u(b, body + 3, so), [_u(b, body + 3 + so + 4 * k, 4) for k in range(nd)])
        p = body + msize
    if chunked is not None and shape is not None and dtype is not None:
        return _chunked(b, shape, dtype, chunked[0], chunked[1], bool(filters), so)
    if shape is None or dtype is None or layout is None:
        raise H5FormatError("dataset without dataspace/datatype/layout")
    addr, nbytes = layout
    n = int(np.prod(shape)) if shape else 1
    if n * dtype.itemsize != nbytes:
        raise H5FormatError("layout size does not match the dataspace")
    return np.frombuffer(b, dtype=dtype, count=n, offset=addr).reshape(shape).copy()


def _chunked(b: bytes, shape, dtype, btree: int, cdims, deflate: bool, so: int) -> np.ndarray:
    """a chunked dataset: walk the raw-data-chunk B-tree (node type 1), inflate every
    chunk and place it at its element offsets (edge chunks cropped)"""
    import zlib
    rank = len(shape)
    out = np.zeros(shape, dtype=dtype)
    cd = cdims[:rank]
    keysz = 8 + 8 * (rank + 1)

    def node(addr):
        if b[addr:addr + 4] != b"TREE":
            raise H5FormatError("bad chunk B-tree signature")
        if b[addr + 4] != 1:
            raise H5FormatError("not a raw-data chunk B-tree")
        level, used = b[addr + 5], _u(b, addr + 6, 2)
        p = addr + 8 + 2 * so
        for i in range(used):
            k = p + i * (keysz + so)
            size = _u(b, k, 4)
            off = [_u(b, k + 8 + 8 * d, 8) for d in range(rank)]
            child = _u(b, k + keysz, so)
            if level > 0:
                node(child)
                continue
            raw = b[child:child + size]
            if deflate:
                raw = zlib.decompress(raw)
            blk = np.frombuffer(raw, dtype=dtype).reshape(cd)
            sl = tuple(slice(o, min(o + c, n)) for o, c, n in zip(off, cd, shape))
            out[sl] = blk[tuple(slice(0, s.stop - s.start) for s in sl)]
    node(btree)
    return out


def read_h5(path: str) -> Dict[str, np.ndarray]:
    with open(path, "rb") as f:
        b = f.read()
    if b[:8] != SIG:
        raise H5FormatError("not an HDF5 file")
    if b[8] != 0:
        raise H5FormatError(f"superblock version {b[8]} (only 0 is read)")
    so, sl = b[13], b[14]
    leaf_k = _u(b, 16, 2)
    eof = _u(b, 24 + 2 * so, so)
    if eof > len(b):
        raise H5FormatError("file shorter than its end-of-file address")
    root = 24 + 4 * so                              # root group symbol-table entry
    cache = _u(b, root + 2 * so, 4)
    if cache != 1:
        raise H5FormatError("root entry without a cached symbol table")
    btree, heap = _u(b, root + 2 * so + 8, so), _u(b, root + 2 * so + 8 + so, so)
    return {name: _dataset(b, oh, so, sl) for name, oh in _group_entries(b, btree, heap, so, sl, leaf_k)}
