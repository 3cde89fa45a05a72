"""Model documentation and schema generator (reference src/schema.xsd.Rt, catalog.xml.Rt,
Model.md.Rt, Models.md.Rt, SUMMARY.Rt): per-model Markdown and XSD, catalog and index;
the XSD declares the elements and setting names a real case file uses."""
import os
import xml.etree.ElementTree as ET

from tclb_amd.tools import docgen

XS = "{http://www.w3.org/2001/XMLSchema}"


def test_generate_docs_and_schemas(tmp_path):
    files = docgen.generate(str(tmp_path), ["d2q9", "d3q27_cumulant"])
    assert len(files) == 7
    md = open(tmp_path / "d2q9.md").read()
    assert "`Viscosity`" in md and "`MRT`" in md and "BaseIteration" in md or "Iteration" in md
    cat = ET.parse(tmp_path / "catalog.xml").getroot()
    assert {e.get("uri") for e in cat} == {"schema/d2q9.xsd", "schema/d3q27_cumulant.xsd"}
    xsd = ET.parse(tmp_path / "schema" / "d2q9.xsd").getroot()
    enums = {st.get("name"): [e.get("value") for e in st.iter(XS + "enumeration")] for st in xsd.iter(XS + "simpleType")}
    assert "Viscosity" in enums["SettingName"] and "VelocityX" in enums["SettingName"]
    assert "U" in enums["QuantityName"] and "MRT" in enums["NodeTypeName"]
    declared = {e.get("name") for e in xsd.iter(XS + "element")}
    # every element of the karman case (tools/bench_karman.py) is declared
    import importlib.util
    spec = importlib.util.spec_from_file_location("bk", os.path.join(os.path.dirname(__file__), "..", "tools", "bench_karman.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    case = ET.fromstring(mod.CASE.format(out="o", iters=10, vtk='<VTK Iterations="5"/>'))
    used = {e.tag for e in case.iter()}
    assert used <= declared, used - declared
    assert {"Solve", "VTK", "Log", "Sample", "Control"} <= declared
    # handler attribute discovery reads the handler sources
    hs = docgen.handler_elements()
    assert "Iterations" in hs["Solve"]


def test_cli(tmp_path):
    assert docgen.main(["--out", str(tmp_path), "d2q9"]) == 0
    assert (tmp_path / "Models.md").exists() and (tmp_path / "SUMMARY.md").exists()
