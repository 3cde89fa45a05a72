#!/usr/bin/env python3
"""Uninitialised-value check of one stage's node code on the host, in the form the GPU runs it.

The GPU runs a split stage as two kernels of the node code instantiated per node class
(Node<..., CLS_ = 1 / 2>, executor_hip.hpp launch_class); the CPU executor runs the
class-0 instantiation only, so UBSan on the CPU build (tests/test_ubsan.py) never executes
the class forms.  This tool takes the state of a small case after `--steps` iterations
(tests/model_cases.py make_case + perturb), dumps the launch and every buffer it points
to, and builds a host driver with clang++ -fsanitize=memory that runs one stage over the
whole box exactly as the GPU dispatch does: class 1 on every node, then class 3 (the nodes a
deferring stage's class 1 handed on), then class 2 (or the
plain node for an unsplit stage; --cls 0 forces that).  Memory Sanitizer aborts on a branch
on an uninitialised value, and after the stage every stored byte of the output snapshot is
checked with __msan_test_shadow: a node that stores a value computed from an uninitialised
variable (in the class form only, e.g. a variable set in the class-1 branch and read on the
common path) is reported with its field and node.

    python tools/msan_node.py d3q27_tePSM_per_NEBB --stage BaseIteration [--steps 2] [--glob]

Host-only: no GPU is used.  Parity note: the host compiler is not the GPU backend; a clean
run rules out source-level uninitialised reads of these instantiations, not a miscompile.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
CLANG = "/opt/rocm/llvm/bin/clang++"

DRIVER = r'''
#include "model.hpp"
#ifndef NO_MSAN
#include <sanitizer/msan_interface.h>
#endif
#include <stdio.h>
#include <stdlib.h>
using M = tclb::M_@MODEL@::Model;

static void* slurp(const char* dir, const char* name, long long* n) {
  char p[4096];
  snprintf(p, sizeof p, "%s/%s", dir, name);
  FILE* f = fopen(p, "rb");
  if (!f) { *n = 0; return nullptr; }
  fseek(f, 0, SEEK_END);
  const long long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* b = aligned_alloc(64, (size_t)((sz + 63) / 64 * 64 + 64));
  if (fread(b, 1, (size_t)sz, f) != (size_t)sz) { fclose(f); *n = 0; return nullptr; }
  fclose(f);
  *n = sz;
  return b;
}

template <int STG, int CLS, bool G>
static void run_cls(const tclb::Launch& L) {
  typedef typename M::template NodeCls<double, double, G, CLS> N;
  typename N::G_ g[M::NGLOBALS_ > 0 ? M::NGLOBALS_ : 1];
  for (int i = 0; i < (M::NGLOBALS_ > 0 ? M::NGLOBALS_ : 1); i++) g[i] = 0;
  for (int z = L.zlo; z < L.zhi; z++)
    for (int y = L.ylo; y < L.yhi; y++)
      for (int x = L.xlo; x < L.xhi; x++) {
        N n(L, x, y, z, g);
        n.template run_stage<STG>();
      }
}

int main(int argc, char** argv) {
  const char* dir = argv[1];
  const int cls = atoi(argv[2]);
  long long n;
  tclb::Launch L = *(tclb::Launch*)slurp(dir, "launch.bin", &n);
  long long nin, nout, nfl;
  L.in = slurp(dir, "in.bin", &nin);
  void* out = slurp(dir, "out.bin", &nout);
  L.out = out;
  L.flags = slurp(dir, "flags.bin", &nfl);
  L.settings = (const double*)slurp(dir, "settings.bin", &n);
  L.zonal = (const double*)slurp(dir, "zonal.bin", &n);
  L.globals = (double*)slurp(dir, "globals.bin", &n);
  L.aux = nullptr;
  L.stream = nullptr;
  L.mbase = nullptr;
  for (int k = 0; k < 6; k++) {
    char nm[32];
    snprintf(nm, sizeof nm, "ext%d.bin", k);
    long long ne;
    void* e = slurp(dir, nm, &ne);
    L.ext[k] = e;
    if (!e) L.next[k] = 0;
  }
@DISPATCH@
#ifndef NO_MSAN
  const long long bad = __msan_test_shadow(out, (size_t)nout);
#else
  const long long bad = -1;
#endif
  if (bad >= 0) {
    printf("UNINIT %lld\n", bad);
    return 3;
  }
  printf("CLEAN\n");
  return 0;
}
'''


def capture(lat, stage_index: int, glob: bool, out_dir: str):
    """the launch of stage `stage_index` over the whole box with every buffer it points to"""
    from tclb_amd.ops import abi
    lat._sync_settings()
    L = abi.Launch.from_buffer_copy(bytes(lat._L))
    nx, ny, nz = lat.shape
    L.xlo, L.xhi, L.ylo, L.yhi, L.zlo, L.zhi = 0, nx, 0, ny, 0, nz
    L.stage = stage_index
    L.glob = 1 if glob else 0
    L.iter = lat.iter
    L.mbase = None
    src, dst = lat.snaps[lat.cur], lat.snaps[1 - lat.cur]
    bufs = {"in": src, "out": dst, "flags": lat.flags, "settings": lat.settings_t, "zonal": lat.zonal_t,
            "globals": lat.globals_t}
    for name, t in bufs.items():
        a = t.detach().cpu()
        base = a.untyped_storage()
        raw = bytes(base)[a.storage_offset() * a.element_size():]
        with open(os.path.join(out_dir, name + ".bin"), "wb") as f:
            f.write(raw)
    for k in range(6):
        if L.ext[k] and L.next[k] > 0:
            raise SystemExit(f"ext[{k}] in use: add its dump to tools/msan_node.py")
    with open(os.path.join(out_dir, "launch.bin"), "wb") as f:
        f.write(bytes(L))
    return dst.numel() * dst.element_size()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("--stage", default=None, help="stage name (default: the first of Iteration)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--glob", action="store_true", help="the globals-integrating instantiation")
    ap.add_argument("--cls", type=int, default=-1, help="-1: as the GPU dispatches, 0: the plain node")
    ap.add_argument("--keep", default=None, help="keep the build/dump directory here")
    ap.add_argument("--san", default="memory", help="memory (default) or undefined,address")
    a = ap.parse_args()
    from model_cases import make_case, perturb
    from tclb_amd import build as B
    lat = make_case(a.model, "cpu")
    lat.init()
    perturb(lat)
    lat.iterate(a.steps)
    m = lat.model
    sname = a.stage or m.action("Iteration").stages[0]
    si = m.stage_index(sname)
    split = bool(m.stage(sname).split)
    # a deferring stage: class 1, its deferred nodes (CLS 3: executor_hip.hpp k_stage_deferred), class 2
    seq = [1, 3, 2] if getattr(m.stage(sname), "defer", False) else [1, 2]
    classes = seq if (split and a.cls < 0) else [max(0, a.cls)]
    tmp = a.keep or tempfile.mkdtemp(prefix="msan_")
    os.makedirs(tmp, exist_ok=True)
    capture(lat, si, a.glob, tmp)
    gen = os.path.join(B.BUILD, "gen", a.model)
    G = "true" if a.glob else "false"
    disp = "\n".join(f"  run_cls<{si}, {c}, {G}>(L);" for c in classes)
    src = DRIVER.replace("@MODEL@", a.model).replace("@DISPATCH@", disp)
    cpp = os.path.join(tmp, "driver.cpp")
    with open(cpp, "w") as f:
        f.write(src)
    exe = os.path.join(tmp, "driver")
    san = ["-fsanitize=memory", "-fsanitize-memory-track-origins", "-O1"] if a.san == "memory" else \
        [f"-fsanitize={a.san}", "-fno-sanitize-recover=all", "-O2", "-DNO_MSAN"]
    cmd = [CLANG, "-g", "-std=c++17", *san, "-fno-omit-frame-pointer", "-fno-math-errno",
           "-I", os.path.join(B.CSRC, "include"),
           "-I", os.path.join(B.CSRC, "models"), "-I", gen, cpp, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit("driver build failed:\n" + r.stderr[-4000:])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")     # the driver's own buffers
    r = subprocess.run([exe, tmp, "0"], capture_output=True, text=True, env=env)
    res = {"model": a.model, "stage": sname, "classes": classes, "glob": a.glob, "san": a.san, "rc": r.returncode}
    out = r.stdout.strip().splitlines()
    if r.returncode == 3 and out and out[-1].startswith("UNINIT"):
        off = int(out[-1].split()[1])
        es = lat.snaps[0].element_size()
        e = off // es
        f, rest = divmod(e, lat.fs)
        z, rest = divmod(rest, lat.NY * lat.px)
        y, x = divmod(rest, lat.px)
        res["uninit_store"] = {"field": m.fields[f].name, "x": x, "y": y - lat.gy, "z": z - lat.gz}
    elif r.returncode != 0:
        res["report"] = r.stderr[-3000:]
    print(json.dumps(res))
    sys.exit(0 if r.returncode == 0 else 1)


if __name__ == "__main__":
    main()
