"""Regression-test runner for case scripts (reference tools/tests.sh:1-276).

    python -m tclb_amd.tools.testrun MODEL [TEST ...] [--tests-dir DIR] [--repeat N]

Tests live in ``DIR/<MODEL>/*.test`` (default ``tests/cases``).  A test is a line script
executed in a fresh directory ``test-<MODEL>-<TEST>-<repeat>``; the first word selects:

  run CMD...            run a command (must succeed)
  fail CMD...           run a command (must fail)
  need FILE [SRC]       copy a file from the test directory
  exists FILE           FILE must have been produced
  diff FILE [REF]       byte-identical to the reference copy
  sha1 FILE [REF]       sha1 equal to REF.sha1
  csvdiff FILE [REF] [EPS] [DISCARD]   numeric CSV comparison (tclb_amd.tools.csvdiff)
  pvtidiff FILE [REF] [EPS] [DX DY DZ] field comparison (native tclb-compare)
  csvconcatenate OUT IN...

Variables available in lines: $SOLVER (this framework's solver for MODEL), $MODEL,
$TCLB (repository root), $TOOLS, $TEST_DIR.  CSV comparisons discard the ``Walltime``
column by default, as the reference does."""
from __future__ import annotations

import argparse
import hashlib
import os
import shlex
import shutil
import subprocess
import sys
from typing import List

from . import csvconcatenate, csvdiff

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _say(ok: bool, msg: str):
    col = "\033[32m" if ok else "\033[31m"
    print(f"  {col}[{'  OK  ' if ok else 'FAILED'}]\033[0m {msg}", flush=True)


class Runner:
    def __init__(self, model: str, tests_dir: str):
        self.model = model
        self.tests_dir = os.path.abspath(tests_dir)
        self.env = dict(os.environ)
        self.env.update({
            "MODEL": model,
            "TCLB": REPO,
            "TOOLS": os.path.join(REPO, "tools"),
            "TEST_DIR": os.path.join(self.tests_dir, model),
            "SOLVER": f"{shlex.quote(sys.executable)} -m tclb_amd {model}",
        })
        self.env["PYTHONPATH"] = REPO + os.pathsep + self.env.get("PYTHONPATH", "")

    def _ref(self, args: List[str], name: str) -> (str, List[str]):
        tdir = self.env["TEST_DIR"]
        if args and os.path.isfile(os.path.join(tdir, args[0])):
            return os.path.join(tdir, args[0]), args[1:]
        return os.path.join(tdir, name), args

    def line(self, words: List[str], cwd: str) -> bool:
        cmd, args = words[0], words[1:]
        if cmd in ("run", "fail"):
            r = subprocess.run(" ".join(args), shell=True, cwd=cwd, env=self.env)
            ok = (r.returncode == 0) == (cmd == "run")
            _say(ok, f"{'running solver' if cmd == 'run' else 'running solver (should fail)'}: {' '.join(args)}")
            return ok
        if cmd == "csvconcatenate":
            ok = csvconcatenate.concatenate(os.path.join(cwd, args[0]), [os.path.join(cwd, a) for a in args[1:]]) == 0
            _say(ok, "concatenating csv files")
            return ok
        target = args[0]
        path = os.path.join(cwd, target)
        if cmd == "exists":
            ok = os.path.isfile(path)
            _say(ok, f"checking {target} (exists)")
            return ok
        ref, rest = self._ref(args[1:], target + (".sha1" if cmd == "sha1" else ""))
        if not os.path.isfile(ref):
            _say(False, f"Requested file not found: {ref}")
            return False
        if cmd == "need":
            shutil.copy(ref, path)
            _say(True, f"copy needed file {target}")
            return True
        if cmd == "diff":
            ok = open(path, "rb").read() == open(ref, "rb").read() if os.path.isfile(path) else False
        elif cmd == "sha1":
            want = open(ref).read().split()[0]
            ok = os.path.isfile(path) and hashlib.sha1(open(path, "rb").read()).hexdigest() == want
        elif cmd == "csvdiff":
            eps = float(rest[0]) if rest else 1e-10
            disc = rest[1] if len(rest) > 1 else "Walltime"
            ok = csvdiff.csvdiff(path, ref, eps, disc) == 0
        elif cmd == "pvtidiff":
            from ..build import build_tools, tool_path
            build_tools()
            extra = [rest[0] if rest else "8"] + rest[1:4]
            ok = subprocess.run([tool_path("compare"), path, ref, *extra], cwd=cwd).returncode == 0
        else:
            print(f"unknown: {cmd}")
            return False
        _say(ok, f"checking {target} ({cmd})")
        return ok

    def run_test(self, test: str, rep: int) -> bool:
        src = os.path.join(self.tests_dir, self.model, test)
        name = test[:-5].replace("/", "-")
        tdir = os.path.abspath(f"test-{self.model}-{name}-{rep}")
        if os.path.isdir(tdir):
            shutil.rmtree(tdir)
        os.makedirs(tdir)
        print(f"\n\033[1mRunning {name} test...\033[0m", flush=True)
        with open(src) as f:
            for raw in f:
                raw = raw.strip()
                if not raw or raw.startswith("#"):
                    continue
                words = shlex.split(_expand(raw, self.env))
                if not self.line(words, tdir):
                    return False
        return True

    def tests(self, names: List[str]) -> List[str]:
        base = os.path.join(self.tests_dir, self.model)
        if not os.path.isdir(base):
            return []
        out = []
        for t in names or ["."]:
            p = os.path.join(base, t)
            if os.path.isfile(p):
                out.append(t)
            elif os.path.isfile(p + ".test"):
                out.append(t + ".test")
            elif os.path.isdir(p):
                out += sorted(os.path.relpath(os.path.join(p, f), base) for f in os.listdir(p) if f.endswith(".test"))
            else:
                raise SystemExit(f"Test not found: {t}")
        return out


def _expand(line: str, env) -> str:
    old = os.environ.copy()
    try:
        os.environ.update(env)
        return os.path.expandvars(line)
    finally:
        os.environ.clear()
        os.environ.update(old)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="run case regression tests")
    ap.add_argument("model")
    ap.add_argument("tests", nargs="*")
    ap.add_argument("--tests-dir", default=os.path.join(REPO, "tests", "cases"))
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args(argv)
    r = Runner(a.model, a.tests_dir)
    tests = r.tests(a.tests)
    if not tests:
        print(f"No tests for model {a.model}.\nExiting with no error.")
        return 0
    ok_all = True
    for rep in range(1, a.repeat + 1):
        for t in tests:
            ok = r.run_test(t, rep)
            _say(ok, f"{t[:-5]} test finished -----")
            ok_all &= ok
    if not ok_all:
        print("Some tests failed")
    return 0 if ok_all else 1


if __name__ == "__main__":
    sys.exit(main())
