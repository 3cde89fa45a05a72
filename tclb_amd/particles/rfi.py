"""Remote Force Interface over a socket: couple a lattice to a particle integrator that
runs as another program (a DEM code, or tools/rfi_simplepart.py).

The reference couples TCLB (the "ForceCalculator") to LAMMPS / LIGGGHTS / ESYS /
simplepart (the "ForceIntegrator") through MPI intercommunicators built by its MPMD
helper: sizes, then particles (16 reals each), then forces and torques (6 reals) per
particle stage, with a death protocol when either side ends
(src/RemoteForceInterface.h:52-178, src/RemoteForceInterface.hpp:23-748, src/MPMD.hpp).
Here one process per GPU has no MPI, so the same exchange runs over a TCP (or Unix)
stream socket between rank 0 of the lattice job and the integrator:

    integrator -> HELLO     {"role": "integrator", "version": 1, "vars": {...}, "stats": {...}}
    calculator -> HELLO     {"role": "calculator", "version": 1, "units": {...}, "box": [...],
                             "vars": {...}, "stats": {...}}
    per particle stage:
      integrator -> PARTICLES  n, float64[n][10]  x y z  vx vy vz  wx wy wz  r  (lattice units)
      calculator -> FORCES     integrate flag, float64[n][6]  fx fy fz  tx ty tz
    calculator -> STOP         (the lattice run ended; the integrator exits)

FORCES carries integrate = 0 after a particle stage of the Init action (no time step,
as the in-process SIMPLEPART does not step in Init) and 1 otherwise.

Negotiation (reference RemoteForceInterface::Negotiate, src/RemoteForceInterface.hpp:
277-440): each side sends its named string variables (``vars``: the calculator's "output"
path, "content" = the configuration inside the <RemoteForceInterface> element, and its
other attributes as numbers in lattice units) and its statistics request; after the
handshake both sides hold the union of the variables (the peer's value wins a name
clash) and collect statistics if either asked, with the first non-empty prefix and
non-zero interval.  Statistics (reference enableStats / printStats): every ``iter``
exchanges a line of the mean particles per rank and the mean wall time of each phase of
the exchange is appended to ``<prefix>_<role>_P<rank>.txt``.

Multi-rank: like the reference RFI, each rank receives only the particles that can act
on its box (sphere of radius r + 2, the kernels' cut-off, overlapping the rank's nodes;
src/RemoteForceInterface.h:52-178): rank 0 scatters the per-rank subsets with their
global indices and gathers the per-rank partial forces back, summing them in rank order.
"""
from __future__ import annotations

import json
import socket
import struct
import time
from typing import Dict, List, Optional, Tuple

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


def negotiate(mine_vars: Dict[str, str], mine_stats: dict, hello: dict) -> Tuple[Dict[str, str], dict]:
    """the shared variables and statistics request after a handshake (reference
    Negotiate): the peer's variables override ours of the same name; statistics on if
    either side asked, with our prefix / interval unless we gave none"""
    vars_ = dict(mine_vars)
    vars_.update({str(k): str(v) for k, v in (hello.get("vars") or {}).items()})
    other = hello.get("stats") or {}
    stats = {"enabled": bool(mine_stats.get("enabled")) or bool(other.get("enabled")),
             "prefix": mine_stats.get("prefix") or other.get("prefix") or "RFI",
             "iter": int(mine_stats.get("iter") or other.get("iter") or 0) or 200}
    return vars_, stats


class Stats:
    """per-exchange statistics of one side (reference sizesStats / waitStats, printed every
    stats_iter exchanges): mean particles per rank and mean seconds per phase"""

    def __init__(self, path: str, every: int, nranks: int, phases: List[str]):
        self.path, self.every, self.nranks, self.phases = path, max(1, int(every)), nranks, phases
        self._sizes = np.zeros(nranks)
        self._dt = np.zeros(len(phases))
        self._n = 0
        self._t = None
        with open(path, "w") as f:
            f.write(", ".join(["size_iter"] + [f"size_{i:03d}" for i in range(nranks)] +
                              [f"dt_{p}" for p in phases]) + "\n")

    def mark(self):
        self._t = time.perf_counter()

    def phase(self, k: int):
        """time since the last mark / phase into phase k"""
        t = time.perf_counter()
        if self._t is not None:
            self._dt[k] += t - self._t
        self._t = t

    def exchange(self, sizes):
        self._sizes += np.asarray(sizes, float)[:self.nranks]
        self._n += 1
        if self._n >= self.every:
            with open(self.path, "a") as f:
                f.write(", ".join([str(self._n)] + [f"{v:.10g}" for v in self._sizes / self._n] +
                                  [f"{v:.10g}" for v in self._dt / self._n]) + "\n")
            self._sizes[:] = 0
            self._dt[:] = 0
            self._n = 0


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

    def native_ok(self) -> bool:
        return False        # every particle stage exchanges with the integrator over the socket

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
        self.vars: Dict[str, str] = {}
        self._stats_req: dict = {}
        self.stats: Optional[Stats] = None
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

    def set_var(self, name: str, value):
        """a named string variable sent to the integrator at the handshake (reference
        RFI.setVar: "output", "content", the element's other attributes)"""
        self.vars[str(name)] = str(value)

    def enable_stats(self, prefix: str = "", every: int = 200):
        """ask for exchange statistics (reference RFI.enableStats)"""
        self._stats_req = {"enabled": True, "prefix": prefix, "iter": int(every)}

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
                                              "box": self.box, "vars": self.vars,
                                              "stats": self._stats_req}).encode())
            agreed = negotiate(self.vars, self._stats_req, hello)
        else:
            agreed = None
        if self._multi:
            agreed = self.comm.bcast_object(agreed)
        self.vars, st = agreed
        if st["enabled"] and self._root:
            nr = self.comm.size if self._multi else 1
            self.stats = Stats(f"{st['prefix']}_calculator_P00.txt", st["iter"], nr,
                               ["wait_particles", "scatter", "stage", "gather", "send_forces"])
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
            if self.stats:
                self.stats.phase(4)
                self.stats.exchange(getattr(self, "_sizes", [0]))
        self._pending = False

    # -- lattice hooks --------------------------------------------------------------
    def pre_stage(self, lat):
        if self._pending:            # the last particle stage was not followed by a step (Init)
            self._send_forces(False)
        if self._boxes is None:
            box = (tuple(lat.slab.offset), tuple(lat.shape))
            self._boxes = self.comm.gather_objects(box) if self._multi else [box]
        parts = None
        st = self.stats
        if self._root:
            if st:
                st.mark()
            rec = unpack_particles(self.chan.expect(PARTICLES))
            if st:
                st.phase(0)
            self.n_total = len(rec)
            parts = []
            for off, shp in self._boxes:
                idx = box_subset(rec, off, shp)
                parts.append((idx, rec[idx]))
            self._sizes = [len(p[0]) for p in parts]
        idx, sub = self.comm.scatter_objects(parts) if self._multi else parts[0]
        if st:
            st.phase(1)
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
        if self.stats:
            self.stats.phase(2)
        parts = self.comm.gather_to_root((self._idx, f)) if self._multi else [(self._idx, f)]
        if self._root:
            full = np.zeros((self.n_total, 6))
            for idx, fr in parts:
                full[idx] += fr
            self._full = full
        if self.stats:
            self.stats.phase(3)
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

    def __init__(self, address: str, timeout: float = 120.0, vars: Optional[Dict[str, str]] = None,
                 stats: Optional[dict] = None):
        host, port = parse_address(address)
        sock = socket.create_connection((host, port), timeout=timeout)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.chan = Channel(sock)
        mine = {str(k): str(v) for k, v in (vars or {}).items()}
        self.chan.send(HELLO, json.dumps({"role": "integrator", "version": VERSION, "vars": mine,
                                          "stats": stats or {}}).encode())
        self.peer = json.loads(self.chan.expect(HELLO))
        self.vars, st = negotiate(mine, stats or {}, self.peer)
        self.stats = Stats(f"{st['prefix']}_integrator_P00.txt", st["iter"], 1,
                           ["integrate", "wait_forces"]) if st["enabled"] else None

    def has_var(self, name: str) -> bool:
        return name in self.vars

    def get_var(self, name: str, default: Optional[str] = None) -> Optional[str]:
        return self.vars.get(name, default)

    def exchange(self, x, v, omega, r):
        st = self.stats
        if st:
            st.phase(0)              # since the previous exchange returned: integration
        self.chan.send(PARTICLES, pack_particles(x, v, omega, r))
        while True:
            kind, p = self.chan.recv()
            if kind == FORCES:
                if st:
                    st.phase(1)
                    st.exchange([len(r)])
                return unpack_forces(p)
            if kind == STOP:
                return None
            raise RFIError(f"RFI: unexpected message {kind}")

    def close(self):
        self.chan.close()
