"""tools/run_examples.py: model inference for cases that name no model (the simplest
catalog model accepting every node type and setting), RT-template detection, iteration
caps (Solve / RunAction / OptSolve)."""
import os
import sys
import xml.etree.ElementTree as ET

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import run_examples as rx  # noqa: E402

CASE2D = """<?xml version="1.0"?>
<CLBConfig version="2.0" output="output/">
  <Units><Param name="x" value="1m" gauge="10"/></Units>
  <Geometry nx="64" ny="32">
    <MRT><Box/></MRT>
    <WVelocity name="Inlet"><Box nx="1"/></WVelocity>
    <Wall mask="ALL"><Box ny="1"/></Wall>
  </Geometry>
  <Model><Param name="nu" value="0.02"/><Param name="Velocity" value="0.01"/></Model>
  <Solve Iterations="5000"/>
  <OptSolve Iterations="100000"/>
</CLBConfig>"""


def test_infer_2d_flow_case(tmp_path):
    p = tmp_path / "case.xml"
    p.write_text(CASE2D)
    dims, types, params = rx.case_requirements(str(p))
    assert dims == 2 and {"MRT", "WVelocity", "Wall"} <= types
    assert params == {"nu", "Velocity"}          # the <Units> gauge is not a setting
    ranked = rx.infer_models(str(p), with_missing=True)
    best = rx.infer_models(str(p))
    assert ranked[0][1] == [] and ranked[0][0] == best[0]      # accepts every name of the case
    assert all(f.startswith("d2q9") for f in best)
    assert len(best[0]) == min(len(f) for f in best)           # fewest options first


def test_infer_3d_case_by_nz(tmp_path):
    p = tmp_path / "case3d.xml"
    p.write_text(CASE2D.replace('ny="32"', 'ny="32" nz="16"'))
    fits = rx.infer_models(str(p), with_missing=True)
    assert fits and all(n.startswith(("d3q", "auto")) for n, _ in fits[:5])


def test_caps_iterations(tmp_path):
    p = tmp_path / "case.xml"
    p.write_text(CASE2D)
    out = rx.capped_case(str(p), 7, str(tmp_path / "out"))
    root = ET.parse(out).getroot()
    assert root.find("Solve").get("Iterations") == "7"
    assert root.find("OptSolve").get("Iterations") == "7"
    assert root.get("output") == str(tmp_path / "out") + "/"
