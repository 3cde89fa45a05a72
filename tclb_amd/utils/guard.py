"""'Did the physics happen' guard of the benchmarks.

A collide-stream step on nodes whose node type the model's Run() does not dispatch a
collision on still streams, and streaming alone keeps a uniform state uniform, conserves
mass and keeps every symmetry: the finite / mass / invariance checks of the benches all
pass on such a run.  Round 4 lost two rounds of pf_velocity figures to exactly that
(every node flagged BGK on a build that collides MRT nodes only, profiles/README.md r04r).

``collision_check(lat)`` runs one step of the configured lattice twice from the same
state — with its flags, and with the COLLISION-group bits cleared from every node — and
compares: if the two steps agree, the flags select no collision anywhere and the run is
not the model's physics.  The lattice's state, iteration and flags are restored.  The
reference has no such check; its meter (src/main.cpp:101-127) counts node updates
whatever they do.
"""
from __future__ import annotations

import math
from typing import Dict

import torch


def collision_check(lat, action: str = "Iteration", min_rel: float = 1e-12) -> Dict[str, object]:
    """{'collides': bool, 'rel_diff': float, 'collision_nodes': fraction of interior nodes
    with a COLLISION-group bit}; one extra step each with and without the collision bits"""
    m = lat.model
    mask = m.group_masks.get("COLLISION", 0)
    nx, ny, nz = lat.shape
    fl = lat.flags[lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx]
    coll_frac = float(((fl.to(torch.int64) & mask) != 0).double().mean().item()) if mask else 0.0
    if not mask:
        return {"collides": False, "rel_diff": 0.0, "collision_nodes": 0.0}
    keep = ((1 << m.flag_bits) - 1) & ~mask
    if lat.flags.dtype == torch.int16 and keep >= 0x8000:
        keep -= 0x10000                  # the same bits in the int16 flag tensor
    state = lat.snaps[lat.cur].clone()
    # the output snapshot's old values matter only to models with late reads
    other = lat.snaps[1 - lat.cur].clone() if m.late_reads(action) else None
    it, cur, glob = lat.iter, lat.cur, dict(lat.globals)
    flags = lat.flags.clone()
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
        lat.flags.copy_(flags)
        lat.flags_changed()
        lat.snaps[cur].copy_(state)
        if other is not None:
            lat.snaps[1 - cur].copy_(other)
        lat.cur, lat.iter = cur, it
        lat.globals.update(glob)
        del probe
    return {"collides": bool(rel > min_rel), "rel_diff": rel, "collision_nodes": coll_frac}
