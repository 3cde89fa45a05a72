#!/usr/bin/env python3
"""Karman vortex street (d2q9 MRT, 1024 x 100, wedge obstacle, Zou/He inlet/outlet): the
small 2-D case most reference examples look like.  The case is written at run time (the
geometry of the reference's example/flow/2d/karman.xml) and run through the full XML
stack (Solver, handlers, VTK output); reports the whole-run MLUPS and the solver's own
MLBUps meter lines.

    python tools/bench_karman.py --iters 10000 [--device cuda]
"""
import argparse
import json
import os
import re
import sys
import tempfile
import time
import xml.etree.ElementTree as ET

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASE = """<CLBConfig version="2.0" output="{out}/" permissive="true">
 <Geometry nx="1024" ny="100">
  <MRT><Box/></MRT>
  <WVelocity name="Inlet"><Inlet/></WVelocity>
  <EPressure name="Outlet"><Outlet/></EPressure>
  <Inlet nx="1" dx="5"><Box/></Inlet>
  <Outlet nx="1" dx="-5"><Box/></Outlet>
  <Wall mask="ALL">
   <Channel/>
   <Wedge dx="120" nx="20" dy="50" ny="20" direction="LowerRight"/>
   <Wedge dx="120" nx="20" dy="30" ny="20" direction="UpperRight"/>
   <Wedge dx="140" nx="20" dy="50" ny="20" direction="LowerLeft"/>
   <Wedge dx="140" nx="20" dy="30" ny="20" direction="UpperLeft"/>
  </Wall>
 </Geometry>
 <Model>
  <Param name="VelocityX" value="0.01"/>
  <Param name="Viscosity" value="0.02"/>
 </Model>
 {vtk}
 <Solve Iterations="{iters}"/>
</CLBConfig>
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--vtk", type=int, default=1000)
    ap.add_argument("--device", default=None)
    ap.add_argument("--precision", default="double")
    a = ap.parse_args()
    import io
    import contextlib
    import torch
    from tclb_amd import handlers  # noqa: F401
    from tclb_amd.solver import Solver
    out = tempfile.mkdtemp(prefix="karman_")
    vtk = f'<VTK Iterations="{a.vtk}"/>' if a.vtk > 0 else ""      # --vtk 0: compute only
    root = ET.fromstring(CASE.format(out=out, iters=a.iters, vtk=vtk))
    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(buf):
        s = Solver("d2q9", root, conffile=os.path.join(out, "karman.xml"), device=dev, precision=a.precision)
        t0 = time.perf_counter()
        s.run()
        if dev == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    log = buf.getvalue()
    meter = [float(v) for v in re.findall(r"([0-9.]+) MLBUps", log)]
    nodes = 1024 * 100
    print(json.dumps({"case": "karman d2q9 1024x100", "device": dev, "precision": a.precision, "vtk_every": a.vtk, "iters": a.iters,
                      "wall_s": round(dt, 3), "MLUPS_whole_run": round(nodes * a.iters / dt / 1e6, 1),
                      "meter_MLBUps_max": max(meter) if meter else None,
                      "vtk_files": len([f for f in os.listdir(out) if f.endswith(".vti")])}), flush=True)


if __name__ == "__main__":
    main()
