"""Particle system + built-in rigid-sphere integrator (reference simplepart.cpp,
src/RemoteForceInterface.*, src/SolidGrid.h).

Device-resident design: once attached to a lattice the particle records live on the
lattice's device — ``P`` (n, 10: position, velocity, angular velocity, radius), the
force/moment accumulator ``acc`` (n, 6) that the particle stage kernels add into, the
solid container (a uniform grid, a bounding-volume tree, or none: ``container``), and (SimplePart) the rigid-body integration.  A time step
therefore issues only device work: zero ``acc`` -> particle stage kernel -> all-reduce of
``acc`` over the ranks (RCCL: asynchronous, no host round trip) -> integration kernel.
The host copies (``x``, ``v``, ``omega``, ``force``, ``torque``) are refreshed lazily,
only when something reads them (a particle log, the socket RFI, a test): the reference's
per-iteration MPI exchange with the integrator is replaced by no synchronisation at all
on the steps without callbacks.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import numpy as np
import torch

PART_STRIDE = 10
_HOST = ("x", "v", "omega", "r", "m", "force", "torque", "fixed")


def _host_prop(name):
    def get(self):
        if name in self._host_stale:
            self._pull()
        # a read-only view: an in-place edit (ps.x[0] = ...) would never reach the device
        # copy, so it raises; assign a whole array (ps.x = a), which marks the device stale
        a = self._h[name].view()
        a.flags.writeable = False
        return a

    def set_(self, value):
        if self._host_stale:
            self._pull()
        self._h[name] = np.array(value, dtype=self._h[name].dtype)
        self._dev_stale = True
    return property(get, set_)


class ParticleSystem:
    """Particles in lattice units (positions in node coordinates)."""

    x = _host_prop("x")
    v = _host_prop("v")
    omega = _host_prop("omega")
    r = _host_prop("r")
    m = _host_prop("m")
    force = _host_prop("force")
    torque = _host_prop("torque")
    fixed = _host_prop("fixed")

    def __init__(self, n: int = 0):
        self._h = {"x": np.zeros((n, 3)), "v": np.zeros((n, 3)), "omega": np.zeros((n, 3)), "r": np.zeros(n),
                   "m": np.zeros(n), "force": np.zeros((n, 3)), "torque": np.zeros((n, 3)),
                   "fixed": np.zeros(n, dtype=bool)}
        self._host_stale = set()      # host arrays older than the device copy
        self._dev_stale = True        # device copy older than the host arrays
        self._d = None                # device tensors (P, acc, qacc, m, free, grid)
        self._dev_key = None
        self.grid_min = 16            # particles; below this the grid is skipped (full scan)
        # solid container (reference --with-solid-container=grid|tree|all,
        # src/configure.ac:92-716): chosen at run time here
        self.container = os.environ.get("TCLB_SOLID_CONTAINER", "grid")
        if self.container not in ("grid", "tree", "all"):
            raise ValueError(f"TCLB_SOLID_CONTAINER={self.container!r}: expected grid, tree or all")

    @property
    def n(self) -> int:
        return len(self._h["r"])

    def add(self, x, r, v=(0, 0, 0), omega=(0, 0, 0), m=None, fixed=False):
        if self._host_stale:
            self._pull()
        h = self._h
        h["x"] = np.vstack([h["x"], np.asarray(x, float)[None]])
        h["v"] = np.vstack([h["v"], np.asarray(v, float)[None]])
        h["omega"] = np.vstack([h["omega"], np.asarray(omega, float)[None]])
        h["r"] = np.append(h["r"], float(r))
        h["m"] = np.append(h["m"], float(m) if m else 4.0 / 3.0 * math.pi * r ** 3)
        h["force"] = np.vstack([h["force"], np.zeros((1, 3))])
        h["torque"] = np.vstack([h["torque"], np.zeros((1, 3))])
        h["fixed"] = np.append(h["fixed"], bool(fixed))
        self._dev_stale = True

    # -- host <-> device ------------------------------------------------------------
    def _push(self, lat):
        """upload the host arrays (after a host-side change or a device change)"""
        h, n, dev = self._h, self.n, lat.device
        rec = np.zeros((max(1, n), PART_STRIDE))
        if n:
            rec[:n, 0:3], rec[:n, 3:6], rec[:n, 6:9], rec[:n, 9] = h["x"], h["v"], h["omega"], h["r"]
        # GPU: nslots copies of the accumulator (core.hpp particle_acc), enough to spread
        # one particle's atomics over the work-groups, few when there are many particles
        nslots = max(1, min(64, 4096 // max(1, n))) if dev.type == "cuda" else 1
        acc = np.zeros((max(1, n) * nslots, 6))
        if n:
            acc[:n, 0:3], acc[:n, 3:6] = h["force"], h["torque"]
        d = {"P": torch.as_tensor(rec).to(dev), "acc": torch.as_tensor(acc).to(dev),
             "qacc": torch.zeros((max(1, n), 6), dtype=torch.float64, device=dev),
             "m": torch.as_tensor(np.where(h["m"] > 0, h["m"], 1.0) if n else np.ones(1)).to(dev),
             "free": torch.as_tensor(~h["fixed"] if n else np.zeros(1, dtype=bool)).to(dev)}
        d["grid"], d["cell"], d["kind"] = None, 1, None
        d["nslots"] = nslots
        if self.container == "tree" and n >= 1:
            nl = 1 << (n - 1).bit_length()
            d["kind"], d["nl"] = "tree", nl
            d["grid"] = torch.zeros(8 + nl + 6 * (2 * nl - 1), dtype=torch.int32, device=dev)
            d["grid"][:8] = torch.tensor([0, 0, 0, 0, 1, nl, 0, 0], dtype=torch.int32)
            d["mscale"] = 1023.0 / max(1, max(lat.gshape))
        elif self.container == "grid" and n >= self.grid_min:
            d["kind"] = "grid"
            d["cell"] = int(np.ceil(h["r"].max() + 2.0))
            gx, gy, gz = (-(-s // d["cell"]) for s in lat.gshape)
            d["ncell"] = gx * gy * gz
            d["grid"] = torch.zeros(9 + d["ncell"] + n, dtype=torch.int32, device=dev)
            d["grid"][:4] = torch.tensor([gx, gy, gz, d["cell"]], dtype=torch.int32)
            d["gdim"] = (gx, gy, gz)
        self._d = d
        self._dev_key = (str(dev), n)
        self._dev_stale = False
        self._host_stale = set()

    def _pull(self):
        """refresh the host arrays from the device (one synchronising copy)"""
        if self._d is None or not self._host_stale:
            self._host_stale = set()
            return
        n = self.n
        P = self._d["P"][:n].cpu().numpy()
        acc = self._d["acc"][:n].cpu().numpy()
        h = self._h
        h["x"], h["v"], h["omega"] = P[:, 0:3].copy(), P[:, 3:6].copy(), P[:, 6:9].copy()
        h["force"], h["torque"] = acc[:, 0:3].copy(), acc[:, 3:6].copy()
        self._host_stale = set()

    def _ensure(self, lat):
        if self._dev_stale or self._d is None or self._dev_key != (str(lat.device), self.n):
            self._push(lat)

    def _build_grid(self):
        """uniform-grid solid container on the device, the layout of tclb_solid_grid
        (csrc/runtime/host.cpp): header gx gy gz cell, cell starts, particle ids sorted by
        cell (stable: ascending id inside a cell); no host round trip"""
        d, n = self._d, self.n
        gx, gy, gz = d["gdim"]
        c = torch.floor(d["P"][:n, 0:3] / d["cell"]).to(torch.int64)
        c[:, 0].clamp_(0, gx - 1)
        c[:, 1].clamp_(0, gy - 1)
        c[:, 2].clamp_(0, gz - 1)
        cid = (c[:, 2] * gy + c[:, 1]) * gx + c[:, 0]
        cnt = torch.zeros(d["ncell"] + 1, dtype=torch.int64, device=cid.device)
        cnt.scatter_add_(0, cid + 1, torch.ones_like(cid))
        g = d["grid"]
        g[8:9 + d["ncell"]] = torch.cumsum(cnt, 0).to(torch.int32)
        g[9 + d["ncell"]:] = torch.sort(cid, stable=True).indices.to(torch.int32)

    @staticmethod
    def _spread10(v):
        """interleave the 10 low bits of v with two zero bits each (Morton code)"""
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        return (v | (v << 2)) & 0x09249249

    def _build_tree(self):
        """bounding-volume tree solid container on the device (the role of the reference
        SolidTree, src/SolidTree.hpp:11-120, a kd-tree built on the host): the particles
        sorted by the Morton code of their centre are the leaves of an implicit complete
        binary tree (node i has children 2i+1, 2i+2; nl leaves, a power of two, unused
        ones empty); every node holds the fp32 box of its cut-off spheres (rad + 2, widened
        by 0.05 so fp32 rounding never drops a candidate), reduced level by level.
        Layout: int header[8] (kind 1 in [4], nl in [5]), leaf ids[nl] (-1: empty), float
        boxes[2 nl - 1][6] (lo xyz, hi xyz).  No host round trip."""
        d, n, nl = self._d, self.n, self._d["nl"]
        g = d["grid"]
        P = d["P"][:n]
        q = (P[:, 0:3] * d["mscale"]).clamp(0, 1023).to(torch.int64)
        code = self._spread10(q[:, 0]) | (self._spread10(q[:, 1]) << 1) | (self._spread10(q[:, 2]) << 2)
        order = torch.argsort(code, stable=True)
        g[8:8 + nl] = -1
        g[8:8 + n] = order.to(torch.int32)
        B = g[8 + nl:].view(torch.float32).view(2 * nl - 1, 6)
        Ps = P[order]
        cut = (Ps[:, 9] + 2.05)[:, None]
        B[nl - 1:nl - 1 + n, 0:3] = (Ps[:, 0:3] - cut).to(torch.float32)
        B[nl - 1:nl - 1 + n, 3:6] = (Ps[:, 0:3] + cut).to(torch.float32)
        B[nl - 1 + n:, 0:3] = float("inf")
        B[nl - 1 + n:, 3:6] = float("-inf")
        lvl = nl.bit_length() - 2          # deepest internal level
        while lvl >= 0:
            st, cnt = (1 << lvl) - 1, 1 << lvl
            ch = B[2 * st + 1:2 * st + 1 + 2 * cnt].view(cnt, 2, 6)
            B[st:st + cnt, 0:3] = ch[:, :, 0:3].amin(1)
            B[st:st + cnt, 3:6] = ch[:, :, 3:6].amax(1)
            lvl -= 1

    def _build_native(self, lat):
        """the solid container built by the native code the action loop also calls
        (csrc/device/particles.hip on a GPU, csrc/runtime/particles_cpu.cpp on the CPU), so
        the Python step path and the native loop share one implementation; _build_grid /
        _build_tree above are the tensor-op statements of the same layouts (tests)"""
        d, n = self._d, self.n
        P, g = d["P"], d["grid"]
        if P.is_cuda:
            from ..ops import device as D
            from ..parallel.native import _dev_lib
            need = int(_dev_lib().tclb_part_tmp_bytes(n, d["ncell"] if d["kind"] == "grid" else 0))
            if d.get("tmp") is None or d["tmp"].numel() < need:
                d["tmp"] = torch.empty(need, dtype=torch.uint8, device=P.device)
            t = d["tmp"]
            if d["kind"] == "grid":
                gx, gy, gz = d["gdim"]
                r = D.lib().tclb_part_build_grid(P.data_ptr(), n, g.data_ptr(), gx, gy, gz, d["cell"], d["ncell"],
                                                 t.data_ptr(), t.numel(), lat._stream())
            else:
                r = D.lib().tclb_part_build_tree(P.data_ptr(), n, g.data_ptr(), d["nl"], d["mscale"], t.data_ptr(),
                                                 t.numel(), lat._stream())
            if r != 0:
                raise RuntimeError(f"solid container build failed ({r})")
            return
        from ..ops import host as H
        if d["kind"] == "grid":
            gx, gy, gz = d["gdim"]
            H.lib().tclb_part_build_grid_cpu(P.data_ptr(), n, g.data_ptr(), gx, gy, gz, d["cell"], d["ncell"])
        else:
            H.lib().tclb_part_build_tree_cpu(P.data_ptr(), n, g.data_ptr(), d["nl"], d["mscale"])

    # -- native action loop (parallel/native.py) ------------------------------------
    def native_ok(self) -> bool:
        """the native action loop can run this system's stage hooks itself (device-resident
        records; no per-step host exchange with another program)"""
        return True

    def native_integrator(self):
        """parameters of the rigid-body step the loop runs after each particle stage, or
        None (particles that do not move)"""
        return None

    def after_native(self, lat, n: int, action: str):
        """host bookkeeping after n native steps"""
        self._host_stale |= {"force", "torque"}

    def _attach(self, lat, acc, nslots: int = 1):
        d = self._d
        L = lat._L
        L.ext[2] = d["P"].data_ptr()
        L.ext[3] = acc.data_ptr()
        L.next[2] = self.n
        L.next[3] = nslots
        if d["grid"] is not None:
            self._build_native(lat)
            L.ext[4] = d["grid"].data_ptr()
            L.next[4] = d["grid"].numel()
        else:
            L.ext[4] = None
            L.next[4] = 0

    # -- lattice hooks --------------------------------------------------------------
    def pre_stage(self, lat):
        """before a particle stage: zero the accumulator, hand the records to the launch"""
        self._ensure(lat)
        self._d["acc"].zero_()
        self._attach(lat, self._d["acc"], self._d["nslots"])

    def attach_for_quantity(self, lat):
        """before a quantity launch (quantities may look at particles): the current
        records, and a scratch accumulator so the stage's forces are not disturbed"""
        self._ensure(lat)
        self._d["qacc"].zero_()
        self._attach(lat, self._d["qacc"])

    def post_stage(self, lat):
        d = self._d
        acc = d["acc"][:max(1, self.n)]
        if d["nslots"] > 1 and self.n:
            from ..ops import device as D
            D.acc_slots(d["acc"], 6 * self.n, d["nslots"], lat._stream())
        if lat.comm.distributed and lat.comm.size > 1:
            acc.copy_(lat.comm.allreduce_globals(acc.reshape(-1).clone(), acc.numel()).reshape(acc.shape))
        # a NaN force is dropped (reference Lattice.cu.Rt:420-435 zeroes it with a notice;
        # the check stays on the device, no host round trip): one HIP kernel on a GPU
        if acc.is_cuda:
            from ..ops import device as D
            D.nan_to_zero(acc, lat._stream())
        else:
            from ..ops import host as H
            H.lib().tclb_part_nan_to_zero_cpu(acc.data_ptr(), acc.numel())
        self._host_stale |= {"force", "torque"}
        self.detach(lat)

    def detach(self, lat):
        """drop the particle records from the launch (after a stage or a quantity)"""
        lat._L.next[2] = 0
        lat._L.next[3] = 0
        lat._L.ext[4] = None
        lat._L.next[4] = 0

    def step(self, lat):
        """advance after the particle stage of one iteration"""


def integrate_rigid(x, v, omega, r, m, fixed, force, torque, acc, periodic, period):
    """one explicit step of free rigid spheres (reference simplepart.cpp), in place, on
    host arrays; used by the stand-alone integrator tools/rfi_simplepart.py.  The
    in-process SimplePart runs the same update on the device (SimplePart._integrate)."""
    for i in range(len(r)):
        if fixed[i]:
            continue
        I = 0.4 * m[i] * r[i] ** 2
        v[i] += force[i] / m[i] + acc
        x[i] += v[i]
        omega[i] += torque[i] / I
        for d in range(3):
            if periodic[d] and period[d] > 0:
                x[i, d] %= period[d]


class SimplePart(ParticleSystem):
    """Built-in rigid spheres (reference simplepart: explicit integration, optional
    periodicity, constant acceleration, logging), integrated on the lattice's device."""

    def __init__(self):
        super().__init__(0)
        self.acc = np.zeros(3)
        self.periodic = np.zeros(3, dtype=bool)
        self.period = np.zeros(3)
        self.log_path: Optional[str] = None
        self.log_every = 1
        self.log_rotation = False
        self.logged: List[int] = []
        self.iteration = 0

    def _integrate(self, lat=None):
        """the update of integrate_rigid, vectorised over the particles on the device:
        v += F/m + a; x += v; omega += T/I (I = 2/5 m r^2); periodic wrap.  On a GPU one
        HIP kernel (csrc/device/particles.hip), else tensor ops"""
        d, n = self._d, self.n
        if n == 0:
            return
        if d["P"].is_cuda:
            from ..ops import device as D
            bits = sum(1 << k for k in range(3) if self.periodic[k])
            stream = lat._stream() if lat is not None else torch.cuda.current_stream(d["P"].device).cuda_stream
            D.rigid_step(d["P"], d["acc"], d["m"], d["free"], n, self.acc, bits, self.period, stream)
            self._host_stale |= {"x", "v", "omega"}
            return
        # the host runtime's step (csrc/runtime/particles_cpu.cpp), the one the native
        # action loop runs on the CPU
        from ..ops import host as H
        bits = sum(1 << k for k in range(3) if self.periodic[k])
        H.lib().tclb_part_rigid_step_cpu(d["P"].data_ptr(), d["acc"].data_ptr(), d["m"].data_ptr(),
                                         d["free"].data_ptr(), n, float(self.acc[0]), float(self.acc[1]),
                                         float(self.acc[2]), bits, float(self.period[0]), float(self.period[1]),
                                         float(self.period[2]))
        self._host_stale |= {"x", "v", "omega"}

    def native_ok(self) -> bool:
        return self.log_path is None          # the particle log is written from Python per step

    def native_integrator(self):
        return {"a": [float(v) for v in self.acc], "period": [float(v) for v in self.period],
                "periodic": sum(1 << k for k in range(3) if self.periodic[k])}

    def after_native(self, lat, n: int, action: str):
        """bookkeeping after n native steps of `action`: the Python step path calls step()
        once per particle stage per step (not in Init), so the iteration count advances by
        n times the action's particle stages (0 when it has none)"""
        self._host_stale |= {"force", "torque"}
        if action == "Init":
            return
        m = lat.model
        k = sum(1 for s in m.action(action).stages if m.stage(s).particle)
        self.iteration += n * k
        if k and self.n:
            self._host_stale |= {"x", "v", "omega"}

    def step(self, lat):
        self.iteration += 1
        self._integrate(lat)
        if self.log_path and self.iteration % self.log_every == 0 and lat.comm.rank == 0:
            self._log()

    def _log(self):
        new = not os.path.exists(self.log_path)
        with open(self.log_path, "a") as f:
            if new:
                cols = ["Iteration"]
                for i in self.logged:
                    cols += [f"p{i}_{c}{a}" for c in ("", "v", "f") for a in "xyz"]
                    if self.log_rotation:
                        cols += [f"p{i}_{c}{a}" for c in ("o", "t") for a in "xyz"]
                f.write(",".join(cols) + "\n")
            row = [str(self.iteration)]
            for i in self.logged:
                for arr in (self.x, self.v, self.force):
                    row += [f"{v:.10e}" for v in arr[i]]
                if self.log_rotation:
                    for arr in (self.omega, self.torque):
                        row += [f"{v:.10e}" for v in arr[i]]
            f.write(",".join(row) + "\n")
