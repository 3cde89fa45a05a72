"""Model documentation and XML schema generator.

The reference renders, per model, an XSD of the case file (src/schema.xsd.Rt from
doc/elements.yaml plus the model's node types, settings, globals and quantities), an
XML catalog mapping ``urn:tclb:<model>`` to the schemas (src/catalog.xml.Rt), a
Markdown page per model (src/Model.md.Rt), an index (src/Models.md.Rt) and a gitbook
SUMMARY (src/SUMMARY.Rt).  Here the same documents come from the registry's Model
objects, the handler registry (element names, and the attributes each handler reads,
found in its source) and the geometry primitives.

    python -m tclb_amd.tools.docgen --out docs [model ...]
"""
from __future__ import annotations

import argparse
import inspect
import os
import re
import xml.etree.ElementTree as ET
from typing import Dict, Iterable, List, Optional

from ..models import registry
from ..models.dsl import Model

XS = "http://www.w3.org/2001/XMLSchema"

# geometry primitives (geometry/geometry.py Geometry.draw) and the attributes each reads
# beyond the region box (dx dy dz nx ny nz fx fy fz)
REGION_ATTRS = ["dx", "dy", "dz", "nx", "ny", "nz", "fx", "fy", "fz", "mask", "name"]
PRIMITIVES: Dict[str, List[str]] = {
    "Box": [], "Sphere": [], "HalfSphere": [],
    "OffgridSphere": ["x", "y", "z", "R"], "OffgridPipe": ["x", "y", "z", "R", "direction"],
    "XPipe": ["x", "y", "z", "R"], "YPipe": ["x", "y", "z", "R"], "ZPipe": ["x", "y", "z", "R"],
    "XAnnulus": ["x", "y", "z", "R", "r"], "Pipe": [], "PipeY": [], "PipeZ": [], "Cylinder": [],
    "Wedge": ["direction"], "STL": ["file", "scale", "x", "y", "z", "Xrot", "Yrot", "Zrot", "side", "ray_type"],
    "Sweep": ["step", "steps"], "Text": ["file", "order"],
    # default zones usable as primitives (geometry.py DEFAULT_ZONES, reference src/def.cpp.Rt:10-33)
    "Inlet": [], "Outlet": [], "Channel": [], "Tunnel": [],
}

_ATTR_RE = re.compile(r"""(?:attr|context_attr|_attr_f|_attr_i|get)\(\s*["']([A-Za-z_][A-Za-z0-9_\-]*)["']""")


def handler_elements() -> Dict[str, List[str]]:
    """element name -> sorted attribute names its handler class reads"""
    from .. import handlers  # noqa: F401  (registers the handler classes)
    from ..handlers.base import REGISTRY
    out: Dict[str, List[str]] = {}
    for name, cls in sorted(REGISTRY.items()):
        attrs = set()
        for k in inspect.getmro(cls):
            if k.__module__.startswith("tclb_amd"):
                try:
                    attrs.update(_ATTR_RE.findall(inspect.getsource(k)))
                except (OSError, TypeError):
                    pass
        out[name] = sorted(attrs)
    return out


def _md_table(head: List[str], rows: Iterable[Iterable]) -> List[str]:
    out = ["| " + " | ".join(head) + " |", "|" + "---|" * len(head)]
    for r in rows:
        out.append("| " + " | ".join(str(c).replace("|", "\\|").replace("\n", " ") for c in r) + " |")
    return out


def model_md(m: Model) -> str:
    """one model page (reference src/Model.md.Rt)"""
    m = m.finalize() if not getattr(m, "_finalized", False) else m
    L = [f"# {m.name}", ""]
    if m.description:
        L += [m.description, ""]
    L += [f"* family: `{m.family}`, {m.dims}-D", f"* reference: `{m.reference}`"]
    opts = [k for k, v in m.options.items() if v]
    if opts:
        L.append("* options: " + ", ".join(f"`{o}`" for o in opts))
    L.append("")
    L += ["## Densities and fields", ""]
    dens = {d.field.name: d for d in m.densities}
    rows = []
    for f in m.fields:
        d = dens.get(f.name)
        st = " ".join(f"{a}:{lo}..{hi}" for a, (lo, hi) in zip("xyz", f.stencil) if (lo, hi) != (0, 0))
        rows.append([f"`{f.name}`", f.group, f"({d.dx},{d.dy},{d.dz})" if d else "",
                     "parameter" if f.parameter else "", st, f.comment])
    L += _md_table(["name", "group", "streaming", "", "stencil", "comment"], rows) + [""]
    L += ["## Settings", ""]
    rows = [[f"`{s.name}`", "zonal" if s.zonal else "global", s.default_str or s.default, s.unit,
             ", ".join(f"{k} = {v}" for k, v in s.derived.items()), s.comment] for s in m.settings]
    L += _md_table(["name", "kind", "default", "unit", "derived", "comment"], rows) + [""]
    if m.globals_:
        L += ["## Globals", ""]
        L += _md_table(["name", "op", "unit", "comment"], [[f"`{g.name}`", g.op, g.unit, g.comment] for g in m.globals_])
        L.append("")
    L += ["## Quantities", ""]
    L += _md_table(["name", "unit", "vector", "comment"],
                   [[f"`{q.name}`", q.unit, "yes" if q.vector else "", ("adjoint " if q.adjoint else "") + q.comment]
                    for q in m.quantities]) + [""]
    L += ["## Node types", ""]
    groups: Dict[str, List[str]] = {}
    for t in m.node_types:
        groups.setdefault(t.group, []).append(t.name)
    L += _md_table(["group", "types"], [[g, ", ".join(f"`{n}`" for n in ns)] for g, ns in groups.items()]) + [""]
    L += ["## Stages and actions", ""]
    L += _md_table(["stage", "function", "saves", "flags"],
                   [[f"`{s.name}`", s.main, ", ".join(s.save_fields) if s.save_fields else "all",
                     " ".join(k for k in ("fixed_point", "particle", "snapshot_reads", "init") if getattr(s, k))]
                    for s in m.stages])
    L += [""] + [f"* `{a.name}`: " + " → ".join(a.stages) for a in m.actions] + [""]
    return "\n".join(L)


def models_md(names: List[str]) -> str:
    """index page (reference src/Models.md.Rt)"""
    rows = []
    for n in names:
        m = registry.get(n)
        rows.append([f"[{n}]({n}.md)", m.family, m.dims, len(m.fields), len(m.settings), m.description])
    return "\n".join(["# Models", ""] + _md_table(["model", "family", "dims", "fields", "settings", "description"], rows)) + "\n"


def summary(names: List[str]) -> str:
    """gitbook SUMMARY (reference src/SUMMARY.Rt)"""
    L = ["# Summary", "", "* [Models](Models.md)"]
    L += [f"  * [{n}]({n}.md)" for n in names]
    return "\n".join(L) + "\n"


def catalog_xml(names: List[str]) -> str:
    """XML catalog: urn:tclb:<model> -> schema/<model>.xsd (reference src/catalog.xml.Rt)"""
    cat = ET.Element("catalog", {"xmlns": "urn:oasis:names:tc:entity:xmlns:xml:catalog"})
    for n in names:
        ET.SubElement(cat, "public", {"publicId": f"urn:tclb:{n}", "uri": f"schema/{n}.xsd"})
        ET.SubElement(cat, "uri", {"name": f"urn:tclb:{n}", "uri": f"schema/{n}.xsd"})
    ET.indent(cat)
    return '<?xml version="1.0"?>\n' + ET.tostring(cat, encoding="unicode") + "\n"


def _xs(parent, tag, **attrs):
    return ET.SubElement(parent, f"{{{XS}}}{tag}", {k: str(v) for k, v in attrs.items()})


def _doc(el, text: str):
    if text:
        a = _xs(el, "annotation")
        _xs(a, "documentation").text = text


def schema_xsd(m: Model, handlers: Optional[Dict[str, List[str]]] = None) -> str:
    """XSD of a case file for model m (reference src/schema.xsd.Rt): the handler elements
    with the attributes they read, <Param>/<Params> restricted to the model's settings,
    node-type elements inside <Geometry> holding the geometry primitives, and the model's
    quantities / globals / fields as enumerations for the attributes that name them"""
    handlers = handlers if handlers is not None else handler_elements()
    ET.register_namespace("xs", XS)
    root = ET.Element(f"{{{XS}}}schema", {"elementFormDefault": "qualified"})
    _doc(root, f"TCLB case file for model {m.name} ({m.description})")

    def enum_type(name, values):
        st = _xs(root, "simpleType", name=name)
        r = _xs(st, "restriction", base="xs:string")
        for v in values:
            _xs(r, "enumeration", value=v)

    enum_type("SettingName", [s.name for s in m.settings])
    enum_type("QuantityName", [q.name for q in m.quantities])
    enum_type("GlobalName", [g.name for g in m.globals_] or ["none"])
    enum_type("NodeTypeName", [t.name for t in m.node_types])
    # geometry primitives
    prim = _xs(root, "group", name="Primitives")
    ch = _xs(prim, "choice")
    for p, extra in PRIMITIVES.items():
        e = _xs(ch, "element", name=p)
        ct = _xs(e, "complexType")
        for a in REGION_ATTRS + extra:
            _xs(ct, "attribute", name=a, type="xs:string")
    # node-type elements (and Zone) inside Geometry
    gct = _xs(root, "complexType", name="NodeTypeElement")
    seq = _xs(gct, "sequence")
    _xs(seq, "group", ref="Primitives", minOccurs=0, maxOccurs="unbounded")
    for a in ("name", "mask"):
        _xs(gct, "attribute", name=a, type="xs:string")
    geom = _xs(root, "complexType", name="GeometryType")
    gch = _xs(_xs(geom, "sequence"), "choice", minOccurs=0, maxOccurs="unbounded")
    for t in m.node_types:
        _doc(_xs(gch, "element", name=t.name, type="NodeTypeElement"), f"node type of group {t.group}")
    _xs(gch, "element", name="Zone", type="NodeTypeElement")
    for a in ("nx", "ny", "nz", "predef", "model", "px", "py", "pz"):
        _xs(geom, "attribute", name=a, type="xs:string")
    # Model/Param
    par = _xs(root, "complexType", name="ParamType")
    _xs(par, "attribute", name="name", type="SettingName", use="required")
    for a in ("value", "zone", "gauge", "Time"):
        _xs(par, "attribute", name=a, type="xs:string")
    params = _xs(root, "complexType", name="ParamsType")
    for s in m.settings:
        _doc(_xs(params, "attribute", name=s.name, type="xs:string"), s.comment)
    _xs(params, "anyAttribute", processContents="lax")
    mod = _xs(root, "complexType", name="ModelType")
    mch = _xs(_xs(mod, "sequence"), "choice", minOccurs=0, maxOccurs="unbounded")
    _xs(mch, "element", name="Param", type="ParamType")
    _xs(mch, "element", name="Params", type="ParamsType")
    _xs(mch, "any", processContents="lax")
    # handler elements: open content (containers nest handlers; children are free-form)
    hct = _xs(root, "complexType", name="HandlerType", mixed="true")
    hch = _xs(_xs(hct, "sequence"), "choice", minOccurs=0, maxOccurs="unbounded")
    _xs(hch, "any", processContents="lax")
    _xs(hct, "anyAttribute", processContents="lax")
    cfg = _xs(root, "element", name="CLBConfig")
    cct = _xs(cfg, "complexType")
    cch = _xs(_xs(cct, "sequence"), "choice", minOccurs=0, maxOccurs="unbounded")
    _xs(cch, "element", name="Geometry", type="GeometryType")
    _xs(cch, "element", name="Model", type="ModelType")
    for h, attrs in handlers.items():
        if h in ("Geometry", "Model", "CLBConfig", "Param", "Params"):
            continue
        e = _xs(cch, "element", name=h, type="HandlerType")
        _doc(e, "attributes read: " + ", ".join(attrs) if attrs else "")
    for a in ("version", "output", "permissive"):
        _xs(cct, "attribute", name=a, type="xs:string")
    ET.indent(root)
    return '<?xml version="1.0"?>\n' + ET.tostring(root, encoding="unicode") + "\n"


def generate(out: str, names: Optional[List[str]] = None) -> List[str]:
    names = names or registry.names()
    os.makedirs(os.path.join(out, "schema"), exist_ok=True)
    hs = handler_elements()
    written = []

    def w(rel, text):
        p = os.path.join(out, rel)
        with open(p, "w") as f:
            f.write(text)
        written.append(p)

    for n in names:
        m = registry.get(n)
        w(f"{n}.md", model_md(m))
        w(os.path.join("schema", f"{n}.xsd"), schema_xsd(m, hs))
    w("Models.md", models_md(names))
    w("SUMMARY.md", summary(names))
    w("catalog.xml", catalog_xml(names))
    return written


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("models", nargs="*")
    ap.add_argument("--out", default="docs")
    a = ap.parse_args(argv)
    files = generate(a.out, a.models or None)
    print(f"wrote {len(files)} files under {a.out}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
