"""Remote Force Interface over a socket: couple a lattice to a particle integrator that
runs as another program (a DEM code, or tools/rfi_simplepart.py).

The reference couples TCLB (the "ForceCalculator") to LAMMPS / LIGGGHTS / ESYS /
simplepart (the "ForceIntegrator") through MPI intercommunicators built by its MPMD
helper: sizes, then particles (16 reals each), then forces and torques (6 reals) per
particle stage, with a death protocol when either side ends
(src/RemoteForceInterface.h:52-178, src/RemoteForceInterface.hpp:23-748, src/MPMD.hpp).
Here one process per GPU has no MPI, so the same exchange runs over a TCP (or Unix)
stream socket between rank 0 of the lattice job and the integrator:

    integrator -> HELLO     {"role": "integrator", "version": 1}
    calculator -> HELLO     {"role": "calculator", "version": 1, "units": {...}, "box": [...]}
    per particle stage:
      integrator -> PARTICLES  n, float64[n][10]  x y z  vx vy vz  wx wy wz  r  (lattice units)
      calculator -> FORCES     integrate flag, float64[n][6]  fx fy fz  tx ty tz
    calculator -> STOP         (the lattice run ended; the integrator exits)

FORCES carries integrate = 0 after a particle stage of the Init action (no time step,
as the in-process SIMPLEPART does not step in Init) and 1 otherwise.

Multi-rank: like the reference RFI, each rank receives only the particles that can act
on its box (sphere of radius r + 2, the kernels' cut-off, overlapping the rank's nodes;
src/RemoteForceInterface.h:52-178): rank 0 scatters the per-rank subsets with their
global indices and gathers the per-rank partial forces back, summing them in rank order.
"""
from __future__ import annotations

import json
import socket
import struct
from typing import Optional, Tuple

import numpy as np

from .system import ParticleSystem

VERSION = 1
MAGIC = b"RFI1"
HELLO, PARTICLES, FORCES, STOP = 1, 2, 3, 4
_HDR = struct.Struct("<4sIQ")
PREC = 10                       # reals per particle record


class RFIError(RuntimeError):
    pass


def parse_address(addr: str) -> Tuple[str, int]:
    host, _, port = addr.rpartition(":")
    return (host or "127.0.0.1"), int(port)


class Channel:
    """length-prefixed binary messages over a stream socket"""

    def __init__(self, sock: socket.socket):
        self.sock = sock

    def send(self, kind: int, payload: bytes = b""):
        self.sock.sendall(_HDR.pack(MAGIC, kind, len(payload)) + payload)

    def _read(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise RFIError("RFI peer closed the connection")
            buf += chunk
        return bytes(buf)

    def recv(self) -> Tuple[int, bytes]:
        magic, kind, n = _HDR.unpack(self._read(_HDR.size))
        if magic != MAGIC:
            raise RFIError(f"bad RFI frame {magic!r}")
        return kind, self._read(n)

    def expect(self, kind: int) -> bytes:
        k, p = self.recv()
        if k != kind:
            raise RFIError(f"RFI: expected message {kind}, got {k}")
        return p

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


def pack_particles(x, v, omega, r) -> bytes:
    n = len(r)
    rec = np.zeros((n, PREC))
    if n:
        rec[:, 0:3], rec[:, 3:6], rec[:, 6:9], rec[:, 9] = x, v, omega, r
    return struct.pack("<q", n) + rec.astype("<f8").tobytes()


def unpack_particles(p: bytes) -> np.ndarray:
    (n,) = struct.unpack_from("<q", p)
    return np.frombuffer(p, dtype="<f8", count=n * PREC, offset=8).reshape(n, PREC).copy()


def pack_forces(force, torque, integrate: bool) -> bytes:
    f = np.concatenate([np.asarray(force, float).reshape(-1, 3), np.asarray(torque, float).reshape(-1, 3)], axis=1)
    return struct.pack("<qq", int(integrate), len(f)) + f.astype("<f8").tobytes()


def unpack_forces(p: bytes) -> Tuple[bool, np.ndarray]:
    integrate, n = struct.unpack_from("<qq", p)
    return bool(integrate), np.frombuffer(p, dtype="<f8", count=n * 6, offset=16).reshape(n, 6).copy()


def box_subset(rec: np.ndarray, offset, shape) -> np.ndarray:
    """indices of the particle records whose influence sphere (radius r + 2) overlaps the
    node box [offset, offset + shape) in every dimension"""
    if len(rec) == 0:
        return np.zeros(0, dtype=np.int64)
    c, reach = rec[:, 0:3], rec[:, 9:10] + 2.0
    lo = np.asarray(offset, float)[None]
    hi = lo + np.asarray(shape, float)[None] - 1.0
    ok = ((c + reach) >= lo) & ((c - reach) <= hi)
    return np.nonzero(ok.all(1))[0]


class RemoteParticles(ParticleSystem):
    """The lattice side (ForceCalculator).  Rank 0 listens on ``address`` (port 0: any
    free port, see ``.address``) and accepts one integrator; ``accept()`` completes the
    handshake."""

    def __init__(self, address: str = "127.0.0.1:0", comm=None, units: Optional[dict] = None, box=None,
                 timeout: float = 120.0):
        super().__init__(0)
        self.comm = comm
        self.units = units or {}
        self.box = list(box) if box is not None else []
        self.timeout = timeout
        self.chan: Optional[Channel] = None
        self._pending = False
        self.exchanges = 0
        self._srv = None
        self._boxes = None            # (offset, shape) of every rank
        self._idx = np.zeros(0, dtype=np.int64)
        self._full = np.zeros((0, 6))  # forces/torques of all particles (rank 0)
        self.n_total = 0
        if self._root:
            host, port = parse_address(address)
            self._srv = socket.create_server((host, port))
            self._srv.settimeout(timeout)
            self.address = f"{host}:{self._srv.getsockname()[1]}"
        else:
            self.address = address
        if comm is not None and comm.size > 1:
            self.address = comm.bcast_object(self.address)

    @property
    def _root(self) -> bool:
        return self.comm is None or self.comm.rank == 0

    def accept(self):
        if self._root:
            sock, _ = self._srv.accept()
            sock.settimeout(self.timeout)
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.chan = Channel(sock)
            hello = json.loads(self.chan.expect(HELLO))
            if hello.get("version") != VERSION or hello.get("role") != "integrator":
                raise RFIError(f"RFI: incompatible peer {hello}")
            self.chan.send(HELLO, json.dumps({"role": "calculator", "version": VERSION, "units": self.units,
                                              "box": self.box}).encode())
        return self

    @property
    def _multi(self) -> bool:
        return self.comm is not None and self.comm.distributed and self.comm.size > 1

    @property
    def forces_all(self) -> np.ndarray:
        """(n, 6) forces and torques of every particle of the last exchange (rank 0)"""
        return self._full

    def _send_forces(self, integrate: bool):
        if self._root:
            self.chan.send(FORCES, pack_forces(self._full[:, 0:3], self._full[:, 3:6], integrate))
        self._pending = False

    # -- lattice hooks --------------------------------------------------------------
    def pre_stage(self, lat):
        if self._pending:            # the last particle stage was not followed by a step (Init)
            self._send_forces(False)
        if self._boxes is None:
            box = (tuple(lat.slab.offset), tuple(lat.shape))
            self._boxes = self.comm.gather_objects(box) if self._multi else [box]
        parts = None
        if self._root:
            rec = unpack_particles(self.chan.expect(PARTICLES))
            self.n_total = len(rec)
            parts = []
            for off, shp in self._boxes:
                idx = box_subset(rec, off, shp)
                parts.append((idx, rec[idx]))
        idx, sub = self.comm.scatter_objects(parts) if self._multi else parts[0]
        self._idx = idx
        self.x, self.v, self.omega = sub[:, 0:3].copy(), sub[:, 3:6].copy(), sub[:, 6:9].copy()
        self.r = sub[:, 9].copy()
        n = len(sub)
        self.m = np.zeros(n)
        self.fixed = np.zeros(n, dtype=bool)
        self.force = np.zeros((n, 3))
        self.torque = np.zeros((n, 3))
        self.exchanges += 1
        ParticleSystem.pre_stage(self, lat)

    def post_stage(self, lat):
        # partial forces of this rank's subset; summed on rank 0 (no all-reduce of the
        # whole particle set)
        self._host_stale |= {"force", "torque"}
        self.detach(lat)
        f = np.concatenate([self.force, self.torque], axis=1) if len(self._idx) else np.zeros((0, 6))
        parts = self.comm.gather_to_root((self._idx, f)) if self._multi else [(self._idx, f)]
        if self._root:
            full = np.zeros((self.n_total, 6))
            for idx, fr in parts:
                full[idx] += fr
            self._full = full
        self._pending = True

    def step(self, lat):
        self._send_forces(True)

    def close(self):
        """end of the run: flush a pending exchange and tell the integrator to stop
        (reference death protocol)"""
        if self._root and self.chan is not None:
            try:
                if self._pending:
                    self._send_forces(False)
                self.chan.send(STOP)
            except (OSError, RFIError):
                pass
            self.chan.close()
        if self._srv is not None:
            self._srv.close()


class IntegratorClient:
    """The integrator side: connect, then ``exchange(x, v, omega, r)`` per particle stage
    returns (integrate, forces[n][6]) or None once the lattice sent STOP."""

    def __init__(self, address: str, timeout: float = 120.0):
        host, port = parse_address(address)
        sock = socket.create_connection((host, port), timeout=timeout)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.chan = Channel(sock)
        self.chan.send(HELLO, json.dumps({"role": "integrator", "version": VERSION}).encode())
        self.peer = json.loads(self.chan.expect(HELLO))

    def exchange(self, x, v, omega, r):
        self.chan.send(PARTICLES, pack_particles(x, v, omega, r))
        while True:
            kind, p = self.chan.recv()
            if kind == FORCES:
                return unpack_forces(p)
            if kind == STOP:
                return None
            raise RFIError(f"RFI: unexpected message {kind}")

    def close(self):
        self.chan.close()
