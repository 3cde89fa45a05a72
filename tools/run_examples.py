#!/usr/bin/env python3
"""Run reference example cases unmodified except for an iteration cap.

    python tools/run_examples.py --iters 10 --device cpu /root/reference/example/article/ThermocapillaryFlow/*.xml

The model of a case is read from its header comment (``MODEL: <name>``, ``Model: <name>``,
``To be used with <name>``, ``Run with <name> model``) or given with ``--model``.  Every
``<Solve>`` / ``<RunAction>`` / ``<OptSolve>`` is capped to ``--iters`` iterations and ``<Repeat>`` to one
pass, so the case runs its geometry, initialisation, handlers and output once.  Each case
runs in a child process (``python -m tclb_amd <model> <case> <xpath edits>``) with the
case's directory as working directory and the output directory redirected to ``--out``;
a JSON line per case records status, wall time and the tail of the log.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time
import xml.etree.ElementTree as ET

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

HEADER_PATTERNS = [
    r"MODEL:\s*([A-Za-z0-9_]+)",
    r"[Mm]odel:\s*([A-Za-z0-9_]+)",
    r"[Tt]o be used with\s+([A-Za-z0-9_]+)",
    r"[Rr]un with\s+([A-Za-z0-9_]+)\s+model",
    r"\(([a-z0-9]+_[A-Za-z0-9_]+) model\)",
]


def model_from_header(path: str):
    from tclb_amd.models import registry
    with open(path, errors="replace") as f:
        head = f.read(4000)
    for pat in HEADER_PATTERNS:
        for m in re.finditer(pat, head):
            name = m.group(1)
            if registry.exists(name):
                return name
    # no header: cases kept in a directory named after their model
    # (example/multiphase/d3q27_pf_velocity/..., example/heat/d2q9q9_cm_cht/...)
    for part in reversed(os.path.normpath(os.path.dirname(os.path.abspath(path))).split(os.sep)):
        if registry.exists(part):
            return part
    return None


_GEOM_KEYWORDS = {"None", "Zone"}


def case_requirements(path: str):
    """(dims, node types drawn in <Geometry>, setting names set by <Param>/<Params>) of a case"""
    from tclb_amd.utils.xpath import load_case
    root = load_case(path)
    dims, types, params = 2, set(), set()
    for g in root.iter("Geometry"):
        nz = re.match(r"\s*([0-9.]+)", g.get("nz", "1"))
        if g.get("nz") is not None and not (nz and float(nz.group(1)) <= 1 and g.get("nz").strip() in ("1", "1.0")):
            dims = 3
        for ch in g:
            if isinstance(ch.tag, str) and ch.tag not in _GEOM_KEYWORDS:
                types.add(ch.tag)
    units = {id(p) for u in root.iter("Units") for p in u.iter("Param")}
    for p in root.iter("Param"):
        if p.get("name") and id(p) not in units:
            params.add(p.get("name"))
    for p in root.iter("Params"):
        for k in p.attrib:
            params.add(k.split("-")[0])
    return dims, types, params


def infer_models(path: str, candidates=None, with_missing=False):
    """reference-catalog models that accept the node types and settings the case uses, best
    first: fewest unknown names, then fewest options.  Cases without a MODEL header are
    run this way; the reference leaves the choice to the user (it builds every model and
    the case names none)."""
    from tclb_amd.models import registry
    dims, types, params = case_requirements(path)
    out = []
    for name in candidates or registry.names():
        try:
            m = registry.get(name)
        except Exception:  # noqa: BLE001 (a catalog entry that cannot be described)
            continue
        if m.dims != dims:
            continue
        nt = {n.name for n in m.node_types} | {n.group for n in m.node_types}
        st = {s.name for s in m.settings} | {g.name + "InObj" for g in m.globals_}
        missing = sorted((types - nt) | (params - st))
        out.append((len(missing), len(name), name, missing))
    out.sort()
    if with_missing:
        return [(n, miss) for _, _, n, miss in out]
    best = out[0][0] if out else 0
    return [n for k, _, n, _ in out if k == best]


OUTPUT_ELEMENTS = ("VTK", "TXT", "BIN", "HDF5", "Catalyst", "Log", "SaveCheckpoint", "SaveBinary", "Sample",
                   "Failcheck", "DumpSettings")


def capped_case(path: str, iters: int, outdir: str, no_output: bool = False) -> str:
    """the case with every Solve/RunAction/OptSolve capped to `iters` (shorter ones kept),
    Repeat to one pass, output redirected; no_output drops the output/check callbacks"""
    from tclb_amd.utils.xpath import load_case
    root = load_case(path)
    root.set("output", outdir.rstrip("/") + "/")
    for el in root.iter():
        if el.tag in ("Solve", "RunAction", "OptSolve") and "Iterations" in el.attrib:
            try:
                n = min(iters, int(float(el.get("Iterations"))))
            except ValueError:
                n = iters
            el.set("Iterations", str(n))
        if el.tag == "Repeat" and "Times" in el.attrib:
            el.set("Times", "1")
    if no_output:
        for parent in list(root.iter()):
            for ch in list(parent):
                if ch.tag in OUTPUT_ELEMENTS:
                    parent.remove(ch)
    d = tempfile.mkdtemp(prefix="tclb_case_")
    tmp = os.path.join(d, os.path.basename(path))
    ET.ElementTree(root).write(tmp)
    return tmp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="+")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--model", default=None)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--out", default="/tmp/tclb_examples")
    ap.add_argument("--timeout", type=int, default=1200)
    ap.add_argument("--infer", action="store_true",
                    help="cases naming no model: pick the simplest catalog model that accepts every node type "
                         "and setting the case uses")
    ap.add_argument("--no-output", action="store_true", help="drop VTK/Log/Failcheck/... (compute-only timing)")
    ap.add_argument("--cwd", default=None, help="working directory (default: the case's directory; the "
                                                 "reference resolves data paths like example/... from its root)")
    a = ap.parse_args()
    ok = 0
    for case in a.cases:
        model = a.model or model_from_header(case)
        rec = {"case": case, "model": model}
        with open(case, errors="replace") as f:
            text = f.read()
        if text.lstrip().startswith("<?R"):
            # R-templated case (<?R ... ?> blocks): the reference expands it with its RT tool first
            rec["status"] = "skipped: RT template, not a case"
            print(json.dumps(rec), flush=True)
            continue
        if model is None and a.infer:
            try:
                fits = infer_models(case)
            except Exception as e:  # noqa: BLE001 (an unparsable case is reported, not fatal)
                fits, rec["error"] = [], str(e)[-300:]
            model = fits[0] if fits else None
            rec.update(model=model, inferred=fits[:5])
        if model is None:
            rec["status"] = "no model in header"
            print(json.dumps(rec), flush=True)
            continue
        if re.search(r"<\s*RunR\b", text) and not re.search(r"<\s*RunR[^>]*python=", text):
            # cases embedding R code: no R interpreter (RunPython blocks do run)
            rec["status"] = "skipped: embedded R code"
            print(json.dumps(rec), flush=True)
            continue
        out = os.path.join(a.out, os.path.splitext(os.path.basename(case))[0])
        os.makedirs(out, exist_ok=True)
        tmp = capped_case(case, a.iters, out, a.no_output)
        t0 = time.time()
        try:
            r = subprocess.run([sys.executable, "-m", "tclb_amd", model, tmp, "--device", a.device],
                               cwd=a.cwd or os.path.dirname(os.path.abspath(case)), capture_output=True, text=True,
                               timeout=a.timeout, env={**os.environ, "PYTHONPATH": REPO})
            rec["status"] = "ok" if r.returncode == 0 else f"rc={r.returncode}"
            rec["tail"] = (r.stdout + r.stderr)[-600:]
            # the solver's speed meter lines: "<iter> it <MLBUps> MLBUps <GB/s> GB/s"
            rec["mlups"] = [float(v) for v in re.findall(r"it\s+([0-9.]+) MLBUps", r.stdout)]
        except subprocess.TimeoutExpired:
            rec["status"] = "timeout"
        finally:
            os.unlink(tmp)
            os.rmdir(os.path.dirname(tmp))
        rec["wall_s"] = round(time.time() - t0, 1)
        ok += rec["status"] == "ok"
        print(json.dumps(rec), flush=True)
    print(json.dumps({"summary": f"{ok}/{len(a.cases)} ok"}), flush=True)


if __name__ == "__main__":
    main()
