"""Geometry rasteriser: XML <Geometry> -> node-type flag array of one rank.

Semantics follow the reference Geometry class (reference: src/Geometry.cpp.Rt):
default zones Inlet/Outlet/Channel/Tunnel (src/def.cpp.Rt:10-33), ``setFlag`` /
``setMask`` / ``setMode`` (overwrite|fill|change) / ``setZone`` (src/Geometry.cpp.Rt:161-230),
region attributes dx/dy/dz (negative = from the end, ``<`` and ``+`` prefixes),
nx/ny/nz, fx/fy/fz (inclusive end) resolved recursively through the parent chain
(getRegion, src/Geometry.cpp.Rt:216-304), the ``Dot`` rule (src/Geometry.cpp.Rt:307-319),
and the primitives Box, HalfSphere, Sphere, OffgridSphere, OffgridPipe, XPipe,
YPipe, ZPipe, XAnnulus, Pipe, PipeY, PipeZ, Cylinder, Wedge, STL, Sweep, Text
(src/Geometry.cpp.Rt:758-1124).

Each primitive is evaluated vectorised over its bounding box only (numpy); the
STL voxeliser (ray parity + sub-voxel cuts) runs in the native host library.
The rank-local array covers the local slab plus its ghost planes (global
coordinates wrap periodically there), so ghost flags need no exchange.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..utils.log import log
from ..utils.units import UnitEnv

MODE_OVERWRITE, MODE_FILL, MODE_CHANGE = 0, 1, 2

DEFAULT_ZONES = """<Geometry>
  <Zone name='Inlet'><Box dx='0' dy='0' dz='0' fx='0' fy='-1' fz='-1'/></Zone>
  <Zone name='Outlet'><Box dx='-1' dy='0' dz='0' fx='-1' fy='-1' fz='-1'/></Zone>
  <Zone name='Channel'>
    <Box dx='0' dy='0' dz='0' fx='-1' fy='0' fz='-1'/>
    <Box dx='0' dy='-1' dz='0' fx='-1' fy='-1' fz='-1'/>
  </Zone>
  <Zone name='Tunnel'>
    <Box dx='0' dy='0' dz='0' fx='-1' fy='0' fz='-1'/>
    <Box dx='0' dy='-1' dz='0' fx='-1' fy='-1' fz='-1'/>
    <Box dx='0' dy='0' dz='0' fx='-1' fy='-1' fz='0'/>
    <Box dx='0' dy='0' dz='-1' fx='-1' fy='-1' fz='-1'/>
  </Zone>
</Geometry>"""


@dataclass
class Region:
    dx: int = 0
    dy: int = 0
    dz: int = 0
    nx: int = 1
    ny: int = 1
    nz: int = 1

    def copy(self):
        return Region(self.dx, self.dy, self.dz, self.nx, self.ny, self.nz)

    def intersect(self, o: "Region") -> "Region":
        x0, y0, z0 = max(self.dx, o.dx), max(self.dy, o.dy), max(self.dz, o.dz)
        x1 = min(self.dx + self.nx, o.dx + o.nx)
        y1 = min(self.dy + self.ny, o.dy + o.ny)
        z1 = min(self.dz + self.nz, o.dz + o.nz)
        return Region(x0, y0, z0, max(0, x1 - x0), max(0, y1 - y0), max(0, z1 - z0))

    def size(self) -> int:
        return max(0, self.nx) * max(0, self.ny) * max(0, self.nz)


class GeometryError(Exception):
    pass


class Geometry:
    """Flag rasteriser for one rank.

    ``flags``: uint32 array (NZ, NY, nx) = local slab incl. ghost planes; ``gz`` (or
    ``gy``) ghost planes on the decomposed axis; global coordinates of local index
    k along that axis are ``(lo - g + k) mod n_global``."""

    def __init__(self, model, gshape: Tuple[int, int, int], slab_lo: int, slab_n: int, axis: int, ghost: int,
                 units: Optional[UnitEnv] = None, permissive: bool = False, yz: Optional[Tuple[int, ...]] = None):
        self.model = model
        self.gnx, self.gny, self.gnz = gshape
        self.axis = axis
        self.units = units or UnitEnv()
        self.permissive = permissive
        self.total = Region(0, 0, 0, self.gnx, self.gny, self.gnz)
        g = ghost
        if axis == 3:               # Y x Z grid block: yz = (ylo, ny, gy, zlo, nz, gz)
            ylo, ny, gy, zlo, nz, gz = yz
            ys = (np.arange(ny + 2 * gy) + ylo - gy) % self.gny
            zs = (np.arange(nz + 2 * gz) + zlo - gz) % self.gnz
        elif axis == 2:
            zs = (np.arange(slab_n + 2 * g) + slab_lo - g) % self.gnz
            ys = np.arange(self.gny)
        else:
            ys = (np.arange(slab_n + 2 * g) + slab_lo - g) % self.gny
            zs = np.arange(self.gnz)
        self.xs = np.arange(self.gnx)
        self.ys = ys
        self.zs = zs
        self.flags = np.zeros((len(zs), len(ys), self.gnx), dtype=np.uint32)
        self.zones: Dict[str, int] = {"DefaultZone": 0}
        self.cuts: Optional[np.ndarray] = None
        self.fg = 0
        self.fg_mask = 0
        self.fg_mode = MODE_OVERWRITE
        self._xml = None
        # sorted coordinate -> local indices maps (for box queries)
        self._yidx = self._index_map(ys)
        self._zidx = self._index_map(zs)

    @staticmethod
    def _index_map(vals: np.ndarray) -> Dict[int, List[int]]:
        d: Dict[int, List[int]] = {}
        for i, v in enumerate(vals.tolist()):
            d.setdefault(v, []).append(i)
        return d

    # ------------------------------------------------------------------ values
    def val(self, attr: Optional[str], default=None, as_int=True):
        if attr is None:
            if default is None:
                raise GeometryError("Attribute without value and default")
            return default
        v = self.units.alt(attr)
        return int(round(v)) if as_int else v

    def val_p(self, attr: str) -> Tuple[int, str]:
        s = attr.strip()
        side = s[0] if s and s[0] in "<>" else "+"
        if side in "<>":
            s = s[1:]
        return int(round(self.units.alt(s))), side

    # ------------------------------------------------------------------ flags
    def node_type_value(self, name: str):
        nt = self.model.node_type(name)
        if nt is not None:
            return nt.value, self.model.group_masks[nt.group]
        if name == "None":
            return 0, 0
        if name == "Clear":
            return 0, self.model.group_masks["ALL"]
        return None

    def set_flag(self, name: str) -> bool:
        v = self.node_type_value(name)
        if v is None:
            if self.permissive:
                log.warning(f"Unknown node type (in xml): {name} — skipped")
                return False
            raise GeometryError(f"Unknown flag (in xml): {name}")
        self.fg, self.fg_mask = v
        self.fg_mode = MODE_OVERWRITE
        return True

    def set_mask(self, name: str):
        if name in self.model.group_masks:
            self.fg_mask = self.model.group_masks[name]
        else:
            raise GeometryError(f"Unknown mask (in xml): {name}")

    def set_mode(self, mode: str):
        m = {"overwrite": MODE_OVERWRITE, "fill": MODE_FILL, "change": MODE_CHANGE}.get(mode)
        if m is None:
            raise GeometryError(f"Unknown mode (in xml): {mode}")
        self.fg_mode = m

    def set_zone(self, name: str):
        if name not in self.zones:
            zi = len(self.zones)
            if zi > self.model.zone_max:
                raise GeometryError(f"too many zones (max {self.model.zone_max})")
            self.zones[name] = zi
        zi = self.zones[name]
        zmask = self.model.group_masks["SETTINGZONE"]
        self.fg = (self.fg & ~zmask) | (zi << self.model.zone_shift)
        self.fg_mask |= zmask

    # ------------------------------------------------------------------ regions
    def get_region(self, node: ET.Element) -> Region:
        chain = []
        n = node
        while n is not None and n.tag != "Geometry":
            chain.append(n)
            n = self._parent.get(n)
        ret = self.total.copy() if n is not None else Region()
        for e in reversed(chain):
            ret = self._apply_region(e, ret)
        return ret

    def _apply_region(self, node: ET.Element, ret: Region) -> Region:
        ret = ret.copy()
        a = node.attrib
        for ax in "xyz":
            d = a.get("d" + ax)
            if d is not None:
                w, side = self.val_p(d)
                n = getattr(ret, "n" + ax)
                if side == "<":
                    w = n + w
                elif side == "+" and w < 0:
                    w = n + w
                setattr(ret, "d" + ax, getattr(ret, "d" + ax) + w)
                setattr(ret, "n" + ax, n - w)
        for ax in "xyz":
            f = a.get("f" + ax)
            if f is not None:
                w = self.val(f)
                if w < 0:
                    w = getattr(ret, "n" + ax) + w + getattr(ret, "d" + ax)
                setattr(ret, "n" + ax, w - getattr(ret, "d" + ax) + 1)
        for ax in "xyz":
            nn = a.get("n" + ax)
            if nn is not None:
                setattr(ret, "n" + ax, self.val(nn))
        return ret

    # ------------------------------------------------------------------ painting
    def _local_box(self, r: Region):
        """local index arrays of the nodes inside region r (global coords)"""
        x0, x1 = max(r.dx, 0), min(r.dx + r.nx, self.gnx)
        if x1 <= x0:
            return None
        ys = [i for y in range(max(r.dy, 0), min(r.dy + r.ny, self.gny)) for i in self._yidx.get(y, [])]
        zs = [i for z in range(max(r.dz, 0), min(r.dz + r.nz, self.gnz)) for i in self._zidx.get(z, [])]
        if not ys or not zs:
            return None
        return np.array(zs), np.array(ys), slice(x0, x1)

    def dot_mask(self, zi: np.ndarray, yi: np.ndarray, xs: slice, mask: Optional[np.ndarray] = None):
        """apply the reference Dot() rule to the sub-block (zi x yi x xs) where mask"""
        sub = self.flags[np.ix_(zi, yi, np.arange(xs.start, xs.stop))]
        sel = np.ones(sub.shape, dtype=bool) if mask is None else mask
        if self.fg_mode == MODE_FILL:
            sel &= (sub & self.fg_mask) == 0
        elif self.fg_mode == MODE_CHANGE:
            sel &= (sub & self.fg_mask) != 0
        new = (sub & np.uint32(~self.fg_mask & 0xFFFFFFFF)) | np.uint32(self.fg)
        sub = np.where(sel, new, sub)
        self.flags[np.ix_(zi, yi, np.arange(xs.start, xs.stop))] = sub

    def _coords(self, zi, yi, xs):
        X = np.arange(xs.start, xs.stop, dtype=np.float64)[None, None, :]
        Y = self.ys[yi].astype(np.float64)[None, :, None]
        Z = self.zs[zi].astype(np.float64)[:, None, None]
        return X, Y, Z

    def paint(self, r: Region, pred=None):
        """paint nodes of region r (global coords, clipped) where pred(X,Y,Z) holds"""
        b = self._local_box(r)
        if b is None:
            return
        zi, yi, xs = b
        if pred is None:
            self.dot_mask(zi, yi, xs)
            return
        X, Y, Z = self._coords(zi, yi, xs)
        m = np.broadcast_to(pred(X, Y, Z), (len(zi), len(yi), xs.stop - xs.start))
        if m.any():
            self.dot_mask(zi, yi, xs, np.array(m))

    def record_cuts(self, r: Region, cuts: np.ndarray):
        """store STL surface cuts (26, r.nz, r.ny, r.nx) into the local cut array"""
        if self.cuts is None:
            self.cuts = np.full((26,) + self.flags.shape, 65535, dtype=np.uint16)
        for k, gz in enumerate(self.zs.tolist()):
            if not (r.dz <= gz < r.dz + r.nz):
                continue
            for j, gy in enumerate(self.ys.tolist()):
                if not (r.dy <= gy < r.dy + r.ny):
                    continue
                src = cuts[:, gz - r.dz, gy - r.dy, :]
                dst = self.cuts[:, k, j, r.dx:r.dx + r.nx]
                np.minimum(dst, src, out=dst)

    # ------------------------------------------------------------------ primitives
    def _attr_f(self, n: ET.Element, name: str, default=None):
        v = n.get(name)
        if v is None:
            if default is None:
                raise GeometryError(f"{n.tag}: missing attribute {name}")
            return default
        return self.units.alt(v)

    def draw(self, node: ET.Element):
        for n in list(node):
            reg = self.get_region(n)
            tag = n.tag
            if tag == "Box":
                self.paint(reg)
            elif tag == "HalfSphere":
                self.paint(reg, lambda X, Y, Z, r=reg: _in_sphere((.5 + X - r.dx) / r.nx, 0.5 - (.5 + Y - r.dy) / r.ny / 2.,
                                                                 (.5 + Z - r.dz) / r.nz))
            elif tag == "Sphere":
                self.paint(reg, lambda X, Y, Z, r=reg: _in_sphere((.5 + X - r.dx) / r.nx, (.5 + Y - r.dy) / r.ny,
                                                                 (.5 + Z - r.dz) / r.nz))
            elif tag == "OffgridSphere":
                x0, y0, z0 = (self._attr_f(n, a) for a in "xyz")
                if n.get("R") is None:
                    Rx, Ry, Rz = (self._attr_f(n, a) for a in ("Rx", "Ry", "Rz"))
                else:
                    Rx = Ry = Rz = self._attr_f(n, "R")
                r = Region(int(x0 - Rx - 5), int(y0 - Ry - 5), int(z0 - Rz - 5), int(2 * Rx + 10), int(2 * Ry + 10),
                           int(2 * Rz + 10))
                self.paint(r, lambda X, Y, Z: ((.5 + X - x0) ** 2 / Rx ** 2 + (.5 + Y - y0) ** 2 / Ry ** 2 +
                                               (.5 + Z - z0) ** 2 / Rz ** 2) < 1.)
            elif tag == "OffgridPipe":
                x0, y0, z0 = (self._attr_f(n, a) for a in "xyz")
                if n.get("R") is None:
                    Rx, Ry = self._attr_f(n, "Rx"), self._attr_f(n, "Ry")
                else:
                    Rx = Ry = self._attr_f(n, "R")
                r = reg.copy()
                r.dx, r.dy, r.nx, r.ny = int(x0 - Rx - 5), int(y0 - Ry - 5), int(2 * Rx + 10), int(2 * Ry + 10)
                self.paint(r, lambda X, Y, Z: ((.5 + X - x0) ** 2 / Rx ** 2 + (.5 + Y - y0) ** 2 / Ry ** 2) < 1.)
            elif tag in ("XPipe", "YPipe", "ZPipe"):
                self._axis_pipe(n, reg, tag[0])
            elif tag == "XAnnulus":
                x0, y0, z0 = (self._attr_f(n, a) for a in "xyz")
                if n.get("Ro") is None:
                    Ryi, Rzi, Ryo, Rzo = (self._attr_f(n, a) for a in ("Ry_i", "Rz_i", "Ry_o", "Rz_o"))
                else:
                    Ryo = Rzo = self._attr_f(n, "Ro")
                    Ryi = Rzi = self._attr_f(n, "Ri")
                r = reg.copy()
                r.dy, r.dz, r.ny, r.nz = int(y0 - Ryo - 5), int(z0 - Rzo - 5), int(2 * Ryo + 10), int(2 * Rzo + 10)
                self.paint(r, lambda X, Y, Z: ((.5 + Z - z0) ** 2 / Rzo ** 2 + (.5 + Y - y0) ** 2 / Ryo ** 2 < 1.) &
                           ((.5 + Z - z0) ** 2 / Rzi ** 2 + (.5 + Y - y0) ** 2 / Ryi ** 2 > 1.))
            elif tag == "Pipe":
                r = Region(reg.dx, reg.dy - 1, reg.dz - 1, reg.nx, reg.ny + 2, reg.nz + 2)
                self.paint(r, lambda X, Y, Z, q=reg: ~_in_sphere(0.5, (.5 + Y - q.dy) / q.ny, (.5 + Z - q.dz) / q.nz))
            elif tag == "PipeY":
                r = Region(reg.dx - 1, reg.dy, reg.dz - 1, reg.nx + 2, reg.ny, reg.nz + 2)
                self.paint(r, lambda X, Y, Z, q=reg: ~_in_sphere(0.5, (.5 + X - q.dx) / q.nx, (.5 + Z - q.dz) / q.nz))
            elif tag == "PipeZ":
                r = Region(reg.dx - 1, reg.dy - 1, reg.dz, reg.nx + 2, reg.ny + 2, reg.nz)
                self.paint(r, lambda X, Y, Z, q=reg: ~_in_sphere(0.5, (.5 + Y - q.dy) / q.ny, (.5 + X - q.dx) / q.nx))
            elif tag == "Cylinder":
                r = Region(reg.dx, reg.dy - 1, reg.dz - 1, reg.nx, reg.ny + 2, reg.nz + 2)
                self.paint(r, lambda X, Y, Z, q=reg: _in_sphere((.5 + X - q.dx) / q.nx, (.5 + Y - q.dy) / q.ny, 0.5 + 0 * Z))
            elif tag == "Wedge":
                typ = n.get("direction", "")
                self.paint(reg, lambda X, Y, Z, q=reg: _in_wedge((X - q.dx) / max(q.nx - 1., 1e-300),
                                                                 (Y - q.dy) / max(q.ny - 1., 1e-300),
                                                                 (Z - q.dz) / max(q.nz - 1., 1e-300), typ))
            elif tag == "STL":
                from .stl import draw_stl
                draw_stl(self, reg, n)
            elif tag == "Sweep":
                self._sweep(reg, n)
            elif tag == "Text":
                self._text(reg, n)
            else:
                z = self._find(self._xml, "Zone", n.tag)
                if z is not None:
                    self.draw(z)
                else:
                    raise GeometryError(f"Unknown geometry element: {tag}")

    def _axis_pipe(self, n, reg, ax):
        # the coordinate along the pipe axis is read but unused by the reference
        # (src/Geometry.cpp.Rt:872): cases omit it (annularTaylorBubble_DasC.xml XPipe)
        x0, y0, z0 = (self._attr_f(n, a, 0.0 if a == ax.lower() else None) for a in "xyz")
        other = {"X": ("y", "z"), "Y": ("x", "z"), "Z": ("x", "y")}[ax]
        if n.get("R") is None:
            Ra, Rb = self._attr_f(n, "R" + other[0]), self._attr_f(n, "R" + other[1])
        else:
            Ra = Rb = self._attr_f(n, "R")
        r = reg.copy()
        c = {"x": x0, "y": y0, "z": z0}
        for o, R in zip(other, (Ra, Rb)):
            setattr(r, "d" + o, int(c[o] - R - 5))
            setattr(r, "n" + o, int(2 * R + 10))
        # NB: the reference YPipe/ZPipe use (x - y0) for the x offset (src/Geometry.cpp.Rt:930,969);
        # we keep that quirk for parity of existing cases.
        if ax == "X":
            pred = lambda X, Y, Z: ((.5 + Z - z0) ** 2 / Rb ** 2 + (.5 + Y - y0) ** 2 / Ra ** 2) < 1.
        elif ax == "Y":
            pred = lambda X, Y, Z: ((.5 + Z - z0) ** 2 / Rb ** 2 + (.5 + X - y0) ** 2 / Ra ** 2) < 1.
        else:
            pred = lambda X, Y, Z: ((.5 + Y - y0) ** 2 / Rb ** 2 + (.5 + X - y0) ** 2 / Ra ** 2) < 1.
        self.paint(r, pred)

    def _sweep(self, reg, node):
        order = int(node.get("order", "1"))
        dl = float(node.get("step", "1e-4"))
        if node.get("steps") is not None:
            dl = 1.0 / self.units.alt(node.get("steps"))
        def_r = self.units.alt(node.get("r")) if node.get("r") is not None else 1.0
        pts = []
        for p in node:
            if p.tag == "Point":
                pts.append((self.units.alt(p.get("x")), self.units.alt(p.get("y")), self.units.alt(p.get("z")),
                            self.units.alt(p.get("r")) if p.get("r") is not None else def_r))
        if not pts:
            return
        order = min(order, len(pts) - 1)
        P = np.array(pts)
        prev = None
        l = 0.0
        while l < 1:
            x0, y0, z0, r = (_bspline(l, P[:, k], order) for k in range(4))
            if prev is None or max(abs(x0 - prev[0]), abs(y0 - prev[1]), abs(z0 - prev[2]), abs(r - prev[3])) >= 0.25:
                prev = (x0, y0, z0, r)
                rr = reg.intersect(Region(int(x0 - r - 1), int(y0 - r - 1), int(z0 - r - 1), int(2 * r + 2),
                                          int(2 * r + 2), int(2 * r + 2)))
                self.paint(rr, lambda X, Y, Z: (.5 + X - x0) ** 2 + (.5 + Y - y0) ** 2 + (.5 + Z - z0) ** 2 < r * r)
            l += dl

    def _text(self, reg, node):
        fn = node.get("file")
        if fn is None:
            raise GeometryError("No 'file' attribute in 'Text' element")
        vals = np.loadtxt(fn, dtype=np.int64).reshape(-1)
        need = reg.nx * reg.ny * reg.nz
        if vals.size < need:
            raise GeometryError(f"File ({fn}) ended while reading")
        # reference order: x outer, y, z inner
        v = vals[:need].reshape(reg.nx, reg.ny, reg.nz).transpose(2, 1, 0)  # -> z,y,x
        crop = self.get_region(self._parent[node]).intersect(self.total)

        def pred(X, Y, Z):
            xi = (X - reg.dx).astype(int)
            yi = (Y - reg.dy).astype(int)
            zi = (Z - reg.dz).astype(int)
            ok = (X >= crop.dx) & (X < crop.dx + crop.nx) & (Y >= crop.dy) & (Y < crop.dy + crop.ny) & \
                 (Z >= crop.dz) & (Z < crop.dz + crop.nz)
            return ok & (v[zi, yi, xi] != 0)
        self.paint(reg, pred)

    # ------------------------------------------------------------------ loading
    @staticmethod
    def _find(root, tag, name):
        if root is None:
            return None
        for c in root:
            if c.tag == tag and c.get("name") == name:
                return c
        return None

    def load(self, node: ET.Element):
        """reference Geometry::load (src/Geometry.cpp.Rt:1140-1184)"""
        defs = ET.fromstring(DEFAULT_ZONES)
        for z in reversed(list(defs)):
            if self._find(node, z.tag, z.get("name")) is None:
                node.insert(0, z)
        self._xml = node
        self._parent = {c: p for p in node.iter() for c in p}
        for n in list(node):
            if n.tag in ("Zone", "Type", "Mask"):
                continue
            if not self.set_flag(n.tag):
                continue
            for k, v in n.attrib.items():
                if k == "name":
                    self.set_zone(v)
                elif k == "mask":
                    self.set_mask(v)
                elif k == "mode":
                    self.set_mode(v)
            if n.get("zone") is not None:
                z = self._find(node, "Zone", n.get("zone"))
                if z is None:
                    raise GeometryError(f"Unknown zone (in xml): {n.get('zone')}")
                self.draw(z)
            self.draw(n)
        return self


def _in_sphere(x, y, z):
    x = 2 * x - 1
    y = 2 * y - 1
    z = 2 * z - 1
    return (x * x + y * y + z * z) < 1


def _in_wedge(x, y, z, typ):
    if typ == "":
        typ = "UpperLeft"
    if typ == "UpperLeft":
        d = x - y
    elif typ == "UpperRight":
        d = (1. - x) - y
    elif typ == "LowerLeft":
        d = x - (1. - y)
    elif typ == "LowerRight":
        d = (1. - x) - (1. - y)
    elif typ == "UpperLeftXZ":
        d = x - z
    elif typ == "UpperRightXZ":
        d = (1. - x) - z
    elif typ == "LowerLeftXZ":
        d = x - (1. - z)
    elif typ == "LowerRightXZ":
        d = (1. - x) - (1. - z)
    else:
        d = np.zeros_like(x)  # reference: unknown direction leaves delta = 0 (fills the region)
    return d < 1e-10


def _bspline(t: float, P: np.ndarray, order: int) -> float:
    """uniform clamped B-spline of given order through control points P (reference src/spline.h)"""
    n = len(P)
    k = order + 1
    m = n + k
    knots = np.concatenate([np.zeros(k), np.arange(1, n - order) / (n - order), np.ones(k)])
    if t >= 1:
        t = 1 - 1e-12
    N = np.array([1.0 if knots[i] <= t < knots[i + 1] else 0.0 for i in range(m - 1)])
    for d in range(1, k):
        Nn = np.zeros(m - 1 - d)
        for i in range(m - 1 - d):
            a = 0.0 if knots[i + d] == knots[i] else (t - knots[i]) / (knots[i + d] - knots[i]) * N[i]
            b = 0.0 if knots[i + d + 1] == knots[i + 1] else (knots[i + d + 1] - t) / (knots[i + d + 1] - knots[i + 1]) * N[i + 1]
            Nn[i] = a + b
        N = Nn
    return float(np.dot(N[:n], P))
