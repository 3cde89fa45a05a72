"""'Did the physics happen' guard of the benchmarks.

A collide-stream step on nodes whose node type the model's Run() does not dispatch a
collision on still streams, and streaming alone keeps a uniform state uniform, conserves
mass and keeps every symmetry: the finite / mass / invariance checks of the benches all
pass on such a run.  Round 4 lost two rounds of pf_velocity figures to exactly that
(every node flagged BGK on a build that collides MRT nodes only, profiles/README.md r04r).

``collision_check(lat)`` runs one step of the configured lattice twice from the same
state — with its flags, and with the COLLISION-group bits cleared from every node — and
compares: if the two steps agree, the flags select no collision anywhere and the run is
not the model's physics.  Models whose Run() acts whatever the COLLISION bits (reaction /
diffusion systems, the finite-difference PDEs, models without a COLLISION group) are then
checked by ``dynamics_check``: one step from a smooth non-uniform state must differ from
pure streaming of that state.  The lattice's state, iteration and flags are restored.  The
reference has no such check; its meter (src/main.cpp:101-127) counts node updates
whatever they do.
"""
from __future__ import annotations

import math
from typing import Dict

import torch


def collision_check(lat, action: str = "Iteration", min_rel: float = 1e-12, _flags=None,
                    _fallback: bool = True) -> Dict[str, object]:
    """{'collides': bool, 'rel_diff': float, 'collision_nodes': fraction of interior nodes
    with a COLLISION-group bit, 'mode'}; one extra step each with and without the collision
    bits.  When clearing them changes nothing, the bits either select no collision (the
    r04r case: flagged BGK on an MRT build — not the physics) or do not matter to this
    model at all (its Run() acts on every node, e.g. a default collision branch); that is
    decided by dynamics_check: the step's streamed populations must differ from pure
    streaming of a non-uniform state."""
    m = lat.model
    mask = m.group_masks.get("COLLISION", 0)
    nx, ny, nz = lat.shape
    fl = lat.flags[lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx]
    coll_frac = float(((fl.to(torch.int64) & mask) != 0).double().mean().item()) if mask else 0.0
    if not mask:
        d = dynamics_check(lat, action, min_rel)
        return {"collides": d["acts"], "rel_diff": d["rel_diff"], "collision_nodes": 0.0, "mode": "dynamics"}
    keep = ((1 << m.flag_bits) - 1) & ~mask
    if lat.flags.dtype == torch.int16 and keep >= 0x8000:
        keep -= 0x10000                  # the same bits in the int16 flag tensor
    state = lat.snaps[lat.cur].clone()
    # the output snapshot's old values matter only to models with late reads
    other = lat.snaps[1 - lat.cur].clone() if m.late_reads(action) else None
    it, cur, glob = lat.iter, lat.cur, dict(lat.globals)
    orig_flags = lat.flags.clone()
    flags = orig_flags if _flags is None else _flags
    ps = lat.particles
    lat.particles = None                 # no particle integration in the probe steps
    # a state away from equilibrium: every stored field scaled by its own factor, the same
    # at every node (a uniform state stays uniform under streaming, while a collision
    # relaxes the non-equilibrium part; an equilibrium state would not tell them apart)
    probe = state.clone()
    for i in range(lat.nf):
        probe[i].mul_(1.0 + 1e-3 * math.sin(1.7 * i + 0.3))
    try:
        first = None
        rel = 0.0
        for clear in (False, True):
            lat.snaps[cur].copy_(probe)
            if other is not None:
                lat.snaps[1 - cur].copy_(other)
            lat.cur, lat.iter = cur, it
            lat.flags.copy_(flags & keep if clear else flags)
            lat.flags_changed()
            lat.iterate(1, glob_last=False, action=action)
            res = lat.snaps[lat.cur][:, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx]
            if first is None:
                first = res.clone()
            else:
                scale, diff = 0.0, 0.0
                for i in range(lat.nf):                 # field by field: no fp64 copy of it all
                    a, b = first[i].double(), res[i].double()
                    scale = max(scale, float(a.abs().max().item()))
                    diff = max(diff, float((a - b).abs().max().item()))
                rel = diff / (scale or 1.0)
    finally:
        lat.particles = ps
        lat.flags.copy_(orig_flags)
        lat.flags_changed()
        lat.snaps[cur].copy_(state)
        if other is not None:
            lat.snaps[1 - cur].copy_(other)
        lat.cur, lat.iter = cur, it
        lat.globals.update(glob)
        del probe
    out = {"collides": bool(rel > min_rel), "rel_diff": rel, "collision_nodes": coll_frac, "mode": "flags"}
    if not out["collides"] and _fallback:
        # no COLLISION group, or a Run() that collides whatever the bits say (reaction /
        # diffusion systems, cm_cht, the finite-difference PDEs): the step must not be
        # pure streaming of a NON-uniform state
        d = dynamics_check(lat, action, min_rel)
        out.update({"collides": d["acts"], "rel_diff": max(rel, d["rel_diff"]), "mode": "dynamics"})
    return out


def dynamics_check(lat, action: str = "Iteration", min_rel: float = 1e-12) -> Dict[str, object]:
    """one step from a smooth non-uniform state against pure streaming of it: every saved
    density field pulled along its velocity (periodic), every other saved field unchanged.
    A step that only streams (or only copies) matches; a collision, reaction, source or
    stencil update does not.  State, iteration, globals restored."""
    m = lat.model
    nx, ny, nz = lat.shape
    saved = sorted({i for s in m.action(action).stages for i in lat._saved_fields(m.stage(s))})
    if not saved:
        return {"acts": False, "rel_diff": 0.0}
    shift = {}
    for dn in m.densities:
        i = next((k for k, f in enumerate(m.fields) if f is dn.field or f.name == dn.field.name), None)
        if i is not None:
            shift[i] = (dn.dz, dn.dy, dn.dx)
    # the streamed populations only, where the model has any: a macroscopic field computed
    # by a later stage (a phase field summed from h) changes under pure streaming too, and
    # would pass a run whose flags select no collision (the r04r case)
    moving = [i for i in saved if i in shift and shift[i] != (0, 0, 0)]
    if moving:
        saved = moving
    state = lat.snaps[lat.cur].clone()
    other = lat.snaps[1 - lat.cur].clone() if m.late_reads(action) else None
    it, cur, glob = lat.iter, lat.cur, dict(lat.globals)
    ps = lat.particles
    lat.particles = None
    dev = state.device
    z = torch.arange(nz, device=dev, dtype=torch.float64)[:, None, None]
    y = torch.arange(ny, device=dev, dtype=torch.float64)[None, :, None]
    x = torch.arange(nx, device=dev, dtype=torch.float64)[None, None, :]
    try:
        interior = lat.snaps[cur][:, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx]
        probe = []
        for i in range(lat.nf):
            w = 1e-3 * torch.sin(2 * math.pi * (x / nx + 2 * y / max(ny, 1) + 3 * z / max(nz, 1)) + 0.7 * i)
            a = interior[i].double()
            # additive as well as relative: a field that is zero everywhere (an initial
            # concentration) must become non-uniform too
            v = (a * (1.0 + w) + w * (1.0 + float(a.abs().max().item()))).to(interior.dtype)
            interior[i].copy_(v)
            probe.append(v.clone())
        lat.exchange()
        lat.iterate(1, glob_last=False, action=action)
        res = lat.snaps[lat.cur][:, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx]
        scale, diff = 0.0, 0.0
        for i in saved:
            exp = probe[i]
            if i in shift:
                dz, dy, dx = shift[i]
                exp = torch.roll(exp, shifts=(dz, dy, dx), dims=(0, 1, 2))
            a, b = res[i].double(), exp.double()
            scale = max(scale, float(b.abs().max().item()))
            diff = max(diff, float((a - b).abs().max().item()))
        rel = diff / (scale or 1.0)
    finally:
        lat.particles = ps
        lat.snaps[cur].copy_(state)
        if other is not None:
            lat.snaps[1 - cur].copy_(other)
        lat.cur, lat.iter = cur, it
        lat.globals.update(glob)
    return {"acts": bool(rel > min_rel), "rel_diff": rel}
