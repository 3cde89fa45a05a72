"""Portable checkpoints.

The reference dumps raw per-rank margin blocks (`<out>_checkpoint_<iter>_<rank>.pri`,
src/Lattice.cu.Rt:708-769) which are layout- and rank-count-specific.  Here a
checkpoint is ONE file holding every stored field in global index order
[field][z][y][x] (storage dtype) plus a JSON header (model, precision, shape, iter,
settings, zones); every rank writes/reads its own slab through a memory map, so a
checkpoint written with N ranks restarts on M ranks (or on CPU)."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

MAGIC = "tclb_amd-checkpoint-1"


def _np_dtype(lat):
    """storage dtype, except that shifted (f - w) and fp16 storage are written as fp64
    true values so the file stays portable across precisions"""
    if lat.storage_shift or lat.sdtype == torch.float16:
        return np.float64
    return np.float32 if lat.sdtype == torch.float32 else np.float64


def save_state(solver, prefix: str) -> str:
    lat = solver.lattice
    path = prefix if prefix.endswith(".tclb") else prefix + ".tclb"
    gnx, gny, gnz = lat.gshape
    dt = _np_dtype(lat)
    shape = (lat.nf, gnz, gny, gnx)
    if solver.rank == 0:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        mm = np.lib.format.open_memmap(path, mode="w+", dtype=dt, shape=shape)
        del mm
        hdr = {"magic": MAGIC, "model": lat.model.name, "precision": lat.precision, "shape": list(lat.gshape),
               "iter": solver.iter, "settings": {n: float(lat.svals[i]) for i, n in enumerate(lat.gsettings)},
               "zonal": {n: lat.zvals[i].tolist() for i, n in enumerate(lat.zsettings)},
               "zones": lat.zone_names, "fields": [f.name for f in lat.model.fields]}
        with open(path + ".json", "w") as f:
            json.dump(hdr, f, indent=1)
    solver.comm.barrier()
    mm = np.load(path, mmap_mode="r+")
    # shifted storage: the shift is added in fp64 (a fp32 sum would round f - w around w)
    loc = lat.fields_interior(torch.float64 if dt == np.float64 else None).detach().cpu().numpy().astype(dt, copy=False)
    ox, oy, oz = lat.slab.offset
    nx, ny, nz = lat.shape
    mm[:, oz:oz + nz, oy:oy + ny, :] = loc
    mm.flush()
    del mm
    solver.comm.barrier()
    return path


def load_state(solver, path: str, comp=None):
    lat = solver.lattice
    if not os.path.exists(path) and os.path.exists(path + ".tclb"):
        path = path + ".tclb"
    hdr = {}
    if os.path.exists(path + ".json"):
        with open(path + ".json") as f:
            hdr = json.load(f)
        if hdr.get("model") != lat.model.name:
            raise ValueError(f"checkpoint is for model {hdr.get('model')}, not {lat.model.name}")
    mm = np.load(path, mmap_mode="r")
    ox, oy, oz = lat.slab.offset
    nx, ny, nz = lat.shape
    data = np.array(mm[:, oz:oz + nz, oy:oy + ny, :])
    t = torch.from_numpy(data).to(lat.device, dtype=torch.float64)
    if comp is not None:
        cur = lat.fields_interior().clone()
        idx = [i for i, f in enumerate(lat.model.fields) if f.group == comp or f.nicename == comp or f.name == comp]
        cur[idx] = t[idx]
        t = cur
    lat.set_fields_interior(t)
    if hdr and comp is None:
        for n, v in hdr.get("settings", {}).items():
            if n in lat.gsettings:
                lat.svals[lat.gsettings.index(n)] = v
        for z, zi in hdr.get("zones", {}).items():
            lat.add_zone(z)
        for n, vals in hdr.get("zonal", {}).items():
            if n in lat.zsettings:
                row = lat.zsettings.index(n)
                for z, zi in hdr.get("zones", {}).items():
                    if zi < len(vals):
                        lat.zvals[row, lat.zone_names[z]] = vals[zi]
        lat._settings_dirty = True
        solver.iter = int(hdr.get("iter", solver.iter))
        lat.iter = solver.iter
