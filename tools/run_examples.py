#!/usr/bin/env python3
"""Run reference example cases unmodified except for an iteration cap.

    python tools/run_examples.py --iters 10 --device cpu /root/reference/example/article/ThermocapillaryFlow/*.xml

The model of a case is read from its header comment (``MODEL: <name>``, ``Model: <name>``,
``To be used with <name>``, ``Run with <name> model``) or given with ``--model``.  Every
``<Solve>`` / ``<RunAction>`` is capped to ``--iters`` iterations and ``<Repeat>`` to one
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
    return None


def capped_case(path: str, iters: int, outdir: str) -> str:
    from tclb_amd.utils.xpath import load_case
    root = load_case(path)
    root.set("output", outdir.rstrip("/") + "/")
    for el in root.iter():
        if el.tag in ("Solve", "RunAction") and "Iterations" in el.attrib:
            el.set("Iterations", str(iters))
        if el.tag == "Repeat" and "Times" in el.attrib:
            el.set("Times", "1")
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
    ap.add_argument("--cwd", default=None, help="working directory (default: the case's directory; the "
                                                 "reference resolves data paths like example/... from its root)")
    a = ap.parse_args()
    ok = 0
    for case in a.cases:
        model = a.model or model_from_header(case)
        rec = {"case": case, "model": model}
        if model is None:
            rec["status"] = "no model in header"
            print(json.dumps(rec), flush=True)
            continue
        with open(case, errors="replace") as f:
            text = f.read()
        if re.search(r"<\s*(RunR|RunPython)\b", text):
            # cases embedding R/Python code: the code in the case file is not executed here
            rec["status"] = "skipped: embedded RunR/RunPython code"
            print(json.dumps(rec), flush=True)
            continue
        out = os.path.join(a.out, os.path.splitext(os.path.basename(case))[0])
        os.makedirs(out, exist_ok=True)
        tmp = capped_case(case, a.iters, out)
        t0 = time.time()
        try:
            r = subprocess.run([sys.executable, "-m", "tclb_amd", model, tmp, "--device", a.device],
                               cwd=a.cwd or os.path.dirname(os.path.abspath(case)), capture_output=True, text=True,
                               timeout=a.timeout, env={**os.environ, "PYTHONPATH": REPO})
            rec["status"] = "ok" if r.returncode == 0 else f"rc={r.returncode}"
            rec["tail"] = (r.stdout + r.stderr)[-600:]
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
