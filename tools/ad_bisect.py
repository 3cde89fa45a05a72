#!/usr/bin/env python3
"""Pass search of the row-form GPU adjoint miscompile (profiles/README.md r03p-r05i).

The dual-number kernel k_ad built from the row-form node accessors at -O2 with >= 2
tangents per pass returns a wrong adjoint at every node (and faults at 3 tangents), while
the same source at -O1, at one tangent, or with the flat accessors is exact — with or
without AGPRs and with or without register spills (r05i).  LLVM's -opt-bisect-limit=N
runs only the first N optional passes of the compile; building the variant
"row_w2_bis<N>" for a grid of N and running the adjoint check on each narrows the first
pass after which the kernel is wrong.

    python tools/ad_bisect.py build --limits 2000,4000,...     # on the build host
    python tools/ad_bisect.py check --limits 2000,4000,...     # on the GPU box
Prints one JSON line per limit (check: max error of the dual-only adjoint step against
the CPU adjoint, tools/adjoint_diag.py's case).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["build", "check", "passes", "ir"])
    ap.add_argument("--out", default="gpurun_out/ad_ir", help="ir: directory of the IR files")
    ap.add_argument("--limits", default="")
    ap.add_argument("--model", default="d3q19_adj")
    ap.add_argument("--form", default="row_w2")
    a = ap.parse_args()
    from tclb_amd import build as B
    limits = [int(v) for v in a.limits.split(",") if v]
    if a.what == "build":
        for n in limits:
            B.build_model(a.model, kinds=("adhip",), variant=f"{a.form}_bis{n}")
            print(json.dumps({"built": f"{a.form}_bis{n}"}), flush=True)
        return
    if a.what == "ir":
        # the device IR of the AD library at each bisection limit (the change between
        # limits N-1 and N is exactly what pass N did; every later pass is skipped)
        from tclb_amd.models import registry
        m = registry.get(a.model)
        paths = B.emit_model(m)
        src = B._adhip_source(m, paths["dir"])
        os.makedirs(a.out, exist_ok=True)
        for n in limits:
            out = os.path.join(a.out, f"{a.model}_{a.form}_bis{n}.ll")
            cmd = B._cmd("adhip", src, out, paths["dir"], f"{a.form}_bis{n}")
            cmd = cmd[:cmd.index("-o")] + ["--offload-device-only", "-S", "-emit-llvm", "-o", out]
            r = subprocess.run(cmd, capture_output=True, text=True)
            print(json.dumps({"limit": n, "ir": out, "rc": r.returncode, "stderr": r.stderr[-300:] if r.returncode else ""}),
                  flush=True)
        return
    if a.what == "passes":
        # the device passes a limit corresponds to (device-only compile, stderr of the bisection)
        from tclb_amd.models import registry
        m = registry.get(a.model)
        paths = B.emit_model(m)
        src = B._adhip_source(m, paths["dir"])
        cmd = B._cmd("adhip", src, "/tmp/ad_bisect.o", paths["dir"], f"{a.form}_bis100000000")
        cmd = cmd[:cmd.index("-o")] + ["--offload-device-only", "-c", "-o", "/tmp/ad_bisect.o"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        lines = [ln for ln in r.stderr.splitlines() if ln.startswith("BISECT")]
        for n in limits:
            for ln in lines[max(0, n - 3):n + 2]:
                print(ln)
            print("--")
        return
    for n in limits:
        env = dict(os.environ, TCLB_AD_VARIANT=f"{a.form}_bis{n}", TCLB_NO_BUILD="1")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "adjoint_diag.py"), "--repeats", "1",
                            "--modes", "dual"], capture_output=True, text=True, env=env, timeout=300)
        rows = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
        err = max((row["max_err"] for row in rows), default=None)
        print(json.dumps({"limit": n, "max_err": err, "bad_nodes": max((row["bad_nodes"] for row in rows), default=None),
                          "rc": r.returncode, "stderr": r.stderr[-400:] if (r.returncode not in (0, 1) or not rows) else ""}),
              flush=True)
        if r.returncode not in (0, 1):
            break


if __name__ == "__main__":
    main()
