import xml.etree.ElementTree as ET

import numpy as np

from tclb_amd.geometry.geometry import Geometry
from tclb_amd.models import registry


def geom(xml, shape=(64, 32, 1), model="d2q9", lo=0, n=None, axis=None, g=1):
    m = registry.get(model)
    gnx, gny, gnz = shape
    axis = axis or (2 if gnz > 1 else 1)
    n = n if n is not None else (gnz if axis == 2 else gny)
    G = Geometry(m, shape, lo, n, axis, g, permissive=True)
    G.load(ET.fromstring(xml))
    return G, m


def interior(G, g=1, axis=1):
    return G.flags[:, g:-g, :] if axis == 1 else G.flags[g:-g]


def test_karman_like():
    xml = """<Geometry nx="64" ny="32"><MRT><Box/></MRT>
      <WVelocity name="Inlet"><Inlet/></WVelocity><EPressure name="Outlet"><Outlet/></EPressure>
      <Wall mask="ALL"><Channel/><Wedge dx="20" nx="8" dy="10" ny="8" direction="LowerRight"/></Wall></Geometry>"""
    G, m = geom(xml)
    f = interior(G)[0]
    wall = m.node_type("Wall").value
    mrt = m.node_type("MRT").value
    assert (f[0, :] == wall).all() and (f[-1, :] == wall).all()
    inner = f[5, 0]
    assert inner & m.group_masks["BOUNDARY"] == m.node_type("WVelocity").value
    assert (inner >> m.zone_shift) == G.zones["Inlet"]
    assert inner & mrt
    assert f[5, 63] & m.group_masks["BOUNDARY"] == m.node_type("EPressure").value
    assert f[12, 30] & m.group_masks["BOUNDARY"] in (0, wall)
    # wedge painted some walls in the box
    assert (f[10:18, 20:28] == wall).sum() > 10
    # ghost rows equal periodic images
    assert (G.flags[:, 0, :] == G.flags[:, -2, :]).all()
    assert (G.flags[:, -1, :] == G.flags[:, 1, :]).all()


def test_modes_fill_change():
    xml = """<Geometry nx="16" ny="16"><MRT><Box/></MRT>
      <Wall mode="fill"><Box dx="2" nx="4"/></Wall>
      <Wall><Box dx="8" nx="2"/></Wall>
      <Solid mode="change"><Box dx="7" nx="4"/></Solid></Geometry>"""
    G, m = geom(xml, shape=(16, 16, 1))
    f = interior(G)[0]
    B = m.group_masks["BOUNDARY"]
    assert ((f[:, 2:6] & B) == m.node_type("Wall").value).all()   # fill: boundary bits were empty
    assert ((f[:, 8:10] & B) == m.node_type("Solid").value).all()  # change: only where set
    assert ((f[:, 7] & B) == 0).all()


def test_region_attrs_negative_and_f():
    xml = """<Geometry nx="20" ny="10"><Wall><Box dx="-3" fx="-1"/></Wall></Geometry>"""
    G, m = geom(xml, shape=(20, 10, 1))
    f = interior(G)[0]
    w = m.node_type("Wall").value
    assert (f[:, 17:] == w).all() and (f[:, :17] == 0).all()


def test_sphere_3d_slab_split():
    xml = """<Geometry nx="16" ny="16" nz="16"><Wall><Sphere dx="4" nx="8" dy="4" ny="8" dz="4" nz="8"/></Wall></Geometry>"""
    full, m = geom(xml, shape=(16, 16, 16), model="d3q27")
    a, _ = geom(xml, shape=(16, 16, 16), model="d3q27", lo=0, n=8, axis=2)
    b, _ = geom(xml, shape=(16, 16, 16), model="d3q27", lo=8, n=8, axis=2)
    F = full.flags[1:-1]
    assert (np.concatenate([a.flags[1:-1], b.flags[1:-1]]) == F).all()
    assert 200 < (F > 0).sum() < 300  # ~ 4/3 pi 4^3 = 268
