"""ctypes bindings of the native host runtime library (libtclb_host.so)."""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    with _lock:
        if _lib is None:
            from .. import build as B
            path = os.path.join(B.LIB, "libtclb_host.so")
            stale = B.host_runtime_stale()
            if stale is not None:
                if os.environ.get("TCLB_NO_BUILD"):
                    raise RuntimeError(f"libtclb_host.so not usable ({stale}) and TCLB_NO_BUILD is set: {path}")
                B.build_host()
            L = ctypes.CDLL(path)
            P = ctypes.c_void_p
            i = ctypes.c_int
            L.tclb_stl_fill.argtypes = [P, i, i, i, i, i, i, i, i, P]
            L.tclb_stl_fill.restype = ctypes.c_longlong
            L.tclb_stl_cuts.argtypes = [P, i, i, i, i, i, i, i, P, P, P]
            L.tclb_stl_cuts.restype = ctypes.c_longlong
            L.tclb_h5_create.argtypes = [ctypes.c_char_p, i, ctypes.c_char_p, P, P, P, P]
            L.tclb_h5_create.restype = ctypes.c_longlong
            L.tclb_h5_create_chunked.argtypes = [ctypes.c_char_p, i, ctypes.c_char_p, P, P, P, P, i, P, P, P, P]
            L.tclb_h5_create_chunked.restype = ctypes.c_longlong
            L.tclb_h5_chunk_bound.argtypes = [i, i, P, P]
            L.tclb_h5_chunk_bound.restype = ctypes.c_longlong
            L.tclb_h5_chunk_pack.argtypes = [P, i, i, P, P, i, P, P]
            L.tclb_h5_chunk_pack.restype = ctypes.c_longlong
            L.tclb_solid_grid.argtypes = [P, i, i, i, i, i, i, P, ctypes.c_longlong]
            L.tclb_solid_grid.restype = ctypes.c_longlong
            L.tclb_nan_scan_f64.argtypes = [P, ctypes.c_longlong]
            L.tclb_nan_scan_f64.restype = ctypes.c_longlong
            L.tclb_nan_scan_f32.argtypes = [P, ctypes.c_longlong]
            L.tclb_nan_scan_f32.restype = ctypes.c_longlong
            L.tclb_png_write.argtypes = [ctypes.c_char_p, P, i, i]
            L.tclb_png_write.restype = i
            d = ctypes.c_double
            L.tclb_part_build_grid_cpu.argtypes = [P, i, P, i, i, i, i, i]
            L.tclb_part_build_grid_cpu.restype = i
            L.tclb_part_build_tree_cpu.argtypes = [P, i, P, i, d]
            L.tclb_part_build_tree_cpu.restype = i
            L.tclb_part_nan_to_zero_cpu.argtypes = [P, i]
            L.tclb_part_nan_to_zero_cpu.restype = None
            L.tclb_part_rigid_step_cpu.argtypes = [P, P, P, P, i, d, d, d, i, d, d, d]
            L.tclb_part_rigid_step_cpu.restype = None
            _lib = L
    return _lib


def stl_fill(tri: np.ndarray, region, axis: int, inside_out: int) -> np.ndarray:
    x0, y0, z0, nx, ny, nz = region
    lev = np.full((nz, ny, nx), inside_out, dtype=np.uint8)
    t = np.ascontiguousarray(tri, dtype=np.float64)
    lib().tclb_stl_fill(t.ctypes.data, len(t), x0, y0, z0, nx, ny, nz, axis, lev.ctypes.data)
    return lev


def stl_cuts(tri: np.ndarray, region, dirs: np.ndarray):
    x0, y0, z0, nx, ny, nz = region
    cuts = np.full((26, nz, ny, nx), 65535, dtype=np.uint16)
    mask = np.zeros((nz, ny, nx), dtype=np.uint8)
    t = np.ascontiguousarray(tri, dtype=np.float64)
    d = np.ascontiguousarray(dirs, dtype=np.int32)
    lib().tclb_stl_cuts(t.ctypes.data, len(t), x0, y0, z0, nx, ny, nz, d.ctypes.data, cuts.ctypes.data,
                        mask.ctypes.data)
    return cuts, mask


def nan_count(a: np.ndarray) -> int:
    a = np.ascontiguousarray(a)
    if a.dtype == np.float64:
        return int(lib().tclb_nan_scan_f64(a.ctypes.data, a.size))
    if a.dtype == np.float32:
        return int(lib().tclb_nan_scan_f32(a.ctypes.data, a.size))
    return int((~np.isfinite(a)).sum())


def solid_grid(rec: np.ndarray, shape, cell: int) -> np.ndarray:
    """uniform-grid solid container of particle records (n, stride) over a lattice of
    global shape (nx, ny, nz); see tclb_solid_grid in csrc/runtime/host.cpp"""
    rec = np.ascontiguousarray(rec, dtype=np.float64)
    n, stride = rec.shape
    nx, ny, nz = shape
    cell = max(1, int(cell))
    ncell = -(-nx // cell) * -(-ny // cell) * -(-nz // cell)
    out = np.zeros(9 + ncell + n, dtype=np.int32)
    r = lib().tclb_solid_grid(rec.ctypes.data, n, stride, nx, ny, nz, cell, out.ctypes.data, out.size)
    if r < 0:
        raise RuntimeError("solid grid buffer too small")
    return out[:r]


def h5_create(path: str, datasets) -> list:
    """write the metadata of an HDF5 file (csrc/runtime/h5.cpp) holding contiguous
    datasets [(name, numpy dtype, shape)], sized for their data; returns the file offset of
    each dataset's data block"""
    n = len(datasets)
    codes = {np.dtype(np.uint8): 0, np.dtype(np.float32): 1, np.dtype(np.float64): 2}
    names = b"".join(nm.encode() + b"\0" for nm, _, _ in datasets)
    dt = np.array([codes[np.dtype(t)] for _, t, _ in datasets], dtype=np.int32)
    rk = np.array([len(s) for _, _, s in datasets], dtype=np.int32)
    dims = np.zeros((max(1, n), 4), dtype=np.int64)
    for k, (_, _, s) in enumerate(datasets):
        dims[k, :len(s)] = s
    off = np.zeros(max(1, n), dtype=np.int64)
    r = lib().tclb_h5_create(path.encode(), n, names, dt.ctypes.data, rk.ctypes.data, dims.ctypes.data,
                              off.ctypes.data)
    if r < 0:
        raise OSError(f"cannot write {path}")
    return [int(v) for v in off[:n]]


def _h5_meta(datasets):
    codes = {np.dtype(np.uint8): 0, np.dtype(np.float32): 1, np.dtype(np.float64): 2}
    n = len(datasets)
    names = b"".join(nm.encode() + b"\0" for nm, _, _ in datasets)
    dt = np.array([codes[np.dtype(t)] for _, t, _ in datasets], dtype=np.int32)
    rk = np.array([len(s) for _, _, s in datasets], dtype=np.int32)
    dims = np.zeros((max(1, n), 4), dtype=np.int64)
    for k, (_, _, s) in enumerate(datasets):
        dims[k, :len(s)] = s
    return n, names, dt, rk, dims


def h5_chunk_pack(a: np.ndarray, cdims, level: int):
    """the chunks of one rank's local block `a` (chunk dims `cdims` dividing a.shape,
    row-major over the chunk grid), deflated (level >= 0, the HDF5 deflate filter's zlib
    format) or raw: returns (bytes as a uint8 array, per-chunk sizes)"""
    a = np.ascontiguousarray(a)
    ld = np.array(a.shape, dtype=np.int64)
    cd = np.array(cdims, dtype=np.int64)
    if len(ld) != len(cd) or np.any(ld % cd):
        raise ValueError(f"chunk dims {tuple(cd)} do not tile {tuple(ld)}")
    L = lib()
    bound = L.tclb_h5_chunk_bound(a.itemsize, a.ndim, ld.ctypes.data, cd.ctypes.data)
    out = np.empty(max(1, bound), dtype=np.uint8)
    sizes = np.zeros(int(np.prod(ld // cd)), dtype=np.int64)
    r = L.tclb_h5_chunk_pack(a.ctypes.data, a.itemsize, a.ndim, ld.ctypes.data, cd.ctypes.data, int(level),
                             out.ctypes.data, sizes.ctypes.data)
    if r < 0:
        raise RuntimeError("HDF5 chunk compression failed")
    return out[:r], sizes


def h5_create_chunked(path: str, datasets, cdims, level: int, chunks) -> list:
    """write the metadata and chunk indexes of an HDF5 file of chunked datasets
    [(name, dtype, shape)] with chunk dims cdims[i] and deflate `level` (< 0: none);
    chunks[i] = [(element offsets, stored size)] in the order the chunks are to be placed;
    returns each dataset's chunk addresses in that order"""
    n, names, dt, rk, dims = _h5_meta(datasets)
    cd = np.zeros((max(1, n), 4), dtype=np.int64)
    for k, c in enumerate(cdims):
        cd[k, :len(c)] = c
    nch = np.array([len(c) for c in chunks] or [0], dtype=np.int64)
    tot = int(nch.sum())
    coff = np.zeros((max(1, tot), 4), dtype=np.int64)
    csz = np.zeros(max(1, tot), dtype=np.int64)
    j = 0
    for lst in chunks:
        for off, sz in lst:
            coff[j, :len(off)] = off
            csz[j] = sz
            j += 1
    addr = np.zeros(max(1, tot), dtype=np.int64)
    r = lib().tclb_h5_create_chunked(path.encode(), n, names, dt.ctypes.data, rk.ctypes.data, dims.ctypes.data,
                                     cd.ctypes.data, int(level), nch.ctypes.data, coff.ctypes.data, csz.ctypes.data,
                                     addr.ctypes.data)
    if r < 0:
        raise OSError(f"cannot write {path}")
    out, j = [], 0
    for lst in chunks:
        out.append([int(v) for v in addr[j:j + len(lst)]])
        j += len(lst)
    return out


def png_write(path: str, rgba: np.ndarray):
    """write an (h, w, 4) uint8 RGBA image, top row first, as PNG (csrc/runtime/png.cpp)"""
    a = np.ascontiguousarray(rgba, dtype=np.uint8)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("png_write expects an (h, w, 4) uint8 array")
    if lib().tclb_png_write(path.encode(), a.ctypes.data, a.shape[1], a.shape[0]) != 0:
        raise OSError(f"cannot write {path}")
