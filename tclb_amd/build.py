"""In-tree build driver: emit + compile every model for gfx950 (hipcc) and for the
host (g++/OpenMP).  Replaces the reference's autoconf + generated makefiles
(reference: makefile:1-20, src/makefile.main.Rt, src/makefile.Rt:56-118).

Outputs go to ``tclb_amd/_build/lib/libtclb_<model>_{hip,cpu}.so`` (git-ignored but
shipped to GPU boxes with the repo snapshot).  Rebuilds are skipped when the
source hash of a target is unchanged.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterable, List, Optional

from .emit.emitter import BUILD, CSRC, emit_model
from .models import registry

LIB = os.path.join(BUILD, "lib")
HIPCC = os.environ.get("TCLB_HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("TCLB_CXX", "g++")
ARCH = os.environ.get("TCLB_OFFLOAD_ARCH", "gfx950")


# build variants (extra compile definitions), used for on-device A/B tuning
VARIANTS = {
    "": ["-DTCLB_NT_STORE=1"],          # default: non-temporal stores (A/B on MI355X: +2..7 %)
    "plain": [],
    "nt": ["-DTCLB_NT_LOAD=1", "-DTCLB_NT_STORE=1"],
    "ntld": ["-DTCLB_NT_LOAD=1"],
    "noxs": ["-DTCLB_DEBUG_NO_XSHIFT", "-DTCLB_NT_STORE=1"],   # diagnostic: aligned-x ceiling
    # occupancy floor for the fp32/fp16-storage kernels (executor_hip.hpp k_stage_narrow)
    "nw3": ["-DTCLB_NT_STORE=1", "-DTCLB_NARROW_WAVES=3"],
    "nw4": ["-DTCLB_NT_STORE=1", "-DTCLB_NARROW_WAVES=4"],
    # zonal settings read by scalar loads for the wave's first zone (core.hpp zonal_read A/B)
    "zscal": ["-DTCLB_NT_STORE=1", "-DTCLB_ZONAL_SCALAR=1"],
    # globals-integrating stage kernels: 2 waves/SIMD for every model / no cap for any
    # (executor_hip.hpp k_stage_glob; the default follows Model.glob_waves)
    "gw2": ["-DTCLB_NT_STORE=1", "-DTCLB_GLOB_WAVES=2"],
    "gw0": ["-DTCLB_NT_STORE=1", "-DTCLB_GLOB_WAVES=0"],
    # A/B of the round-3 defaults: per-thread register globals accumulators reduced at the
    # end of the block (executor_hip.hpp TCLB_GLOB_LDS=0); one 64-bit flat address per
    # access instead of SGPR row base + 32-bit lane offset (core.hpp TCLB_ROW_ADDR=0)
    "gregs": ["-DTCLB_NT_STORE=1", "-DTCLB_GLOB_LDS=0"],
    "flataddr": ["-DTCLB_NT_STORE=1", "-DTCLB_ROW_ADDR=0"],
    # the round-3 default: row addressing in the plain (globals-free) kernels too
    "rowplain": ["-DTCLB_NT_STORE=1", "-DTCLB_ROW_ADDR_PLAIN=1"],
    # A/B of the LDS-staged stencil tiles (executor_hip.hpp k_tile): global loads instead
    "nolds": ["-DTCLB_NT_STORE=1", "-DTCLB_LDS_TILES=0"],
    # A/B of a 2-waves/SIMD floor on every stage kernel (executor_hip.hpp TCLB_STAGE_WAVES)
    "sw2": ["-DTCLB_NT_STORE=1", "-DTCLB_STAGE_WAVES=2"],
    "sw3": ["-DTCLB_NT_STORE=1", "-DTCLB_STAGE_WAVES=3"],
    # node-class split stages (DSL add_stage(split=True)) as one kernel; a 2 / 3-waves/SIMD
    # floor on the class-1 kernel of split stages only
    "nosplit": ["-DTCLB_NT_STORE=1", "-DTCLB_NO_SPLIT=1"],
    # occupancy floors of the LDS tile kernels (k_tile.hpp TCLB_TILE_WAVES)
    "tw6": ["-DTCLB_NT_STORE=1", "-DTCLB_TILE_WAVES=6"],
    "tw8": ["-DTCLB_NT_STORE=1", "-DTCLB_TILE_WAVES=8"],
    # class-2 kernels without their 2-wave floor (reproduces the r05m tePSM fault)
    "c2w0": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES2=0"],
    # the same form with one backend stage changed at a time (which stage the fault needs):
    # VGPR->AGPR spill copies off, machine schedulers off, the high-pressure reschedule off,
    # -O1, and the machine verifier after every codegen pass
    "c2w0_noagpr": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES2=0", "-mllvm", "-amdgpu-spill-vgpr-to-agpr=0"],
    "c2w0_nomisched": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES2=0", "-mllvm", "-enable-misched=0"],
    "c2w0_nopostra": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES2=0", "-mllvm", "-enable-post-misched=0"],
    "c2w0_nohrp": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES2=0", "-mllvm",
                   "-amdgpu-disable-unclustered-high-rp-reschedule"],
    "c2w0_o1": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES2=0", "-O1"],
    "c2w0_verify": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES2=0", "-mllvm", "-verify-machineinstrs"],
    # the default build with the scheduler's high-pressure reschedule stage off (perf A/B)
    "nohrp": ["-DTCLB_NT_STORE=1", "-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule"],
    "cw2": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES=2"],
    "cw3": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES=3"],
    "cw4": ["-DTCLB_NT_STORE=1", "-DTCLB_SPLIT_WAVES=4"],
    # the round-2 form everywhere: flat accessors, register globals, no uniform-y hint
    # scheduler A/B: memory clauses grouped by the AMDGPU machine scheduler
    "mclause": ["-DTCLB_NT_STORE=1", "-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    "r02like": ["-DTCLB_NT_STORE=1", "-DTCLB_FLAT_NODE=1", "-DTCLB_GLOB_LDS=0", "-DTCLB_UNIFORM_Y=0"],
}
DEFAULT_VARIANT = os.environ.get("TCLB_VARIANT", "")
# CPU executor variants: "ubsan" builds the node code with UndefinedBehaviorSanitizer
# (host code only; the runtime is a plain shared dependency, no preload needed)
CPU_VARIANTS = {
    "ubsan": ["-fsanitize=undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g1"],
}


# GPU adjoint executor variants: tangents per pass (tclb_ad/executor_ad_hip.hpp TCLB_AD_WINDOW)
AD_VARIANTS = {f"w{w}": [f"-DTCLB_AD_WINDOW={w}"] for w in (1, 2, 3, 5)}
# diagnostics of the row-accessor adjoint fault (round-3 verdict, What's weak #3): the row
# accessors of the primal build, at -O2 / -O1 / one tangent per pass
AD_VARIANTS.update({"row": ["-DTCLB_FLAT_NODE=0"], "row_o1": ["-DTCLB_FLAT_NODE=0", "-O1"],
                    "row_w1": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WINDOW=1"],
                    "row_w2": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WINDOW=2"],
                    "row_w3": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WINDOW=3"],
                    # round-5 diagnosis: the same row-form builds with VGPR->AGPR spilling off
                    # (the failing builds are the ones whose k_ad runs past 256 VGPRs into AGPRs)
                    # (the flag leaves the code unchanged: the AGPRs are allocated as ordinary
                    # registers, not spill slots, profiles/README.md r05i) and with a 2-wave
                    # floor that keeps k_ad within 256 VGPRs (no AGPRs at all)
                    "row_noagpr": ["-DTCLB_FLAT_NODE=0", "-mllvm", "-amdgpu-spill-vgpr-to-agpr=0"],
                    "row_w2_noagpr": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WINDOW=2", "-mllvm",
                                      "-amdgpu-spill-vgpr-to-agpr=0"],
                    "row_w2_wpe2": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WINDOW=2", "-DTCLB_AD_WAVES=2"],
                    "row_wpe2": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WAVES=2"],
                    "flat_wpe2": ["-DTCLB_AD_WAVES=2"],
                    # round 6: the primal class-2 fault needs the scheduler's unclustered
                    # high-pressure reschedule stage (profiles/README.md r06s-t); the same
                    # two switches on the failing row form
                    "row_w2_nohrp": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WINDOW=2", "-mllvm",
                                     "-amdgpu-disable-unclustered-high-rp-reschedule"],
                    "row_w2_nomisched": ["-DTCLB_FLAT_NODE=0", "-DTCLB_AD_WINDOW=2", "-mllvm", "-enable-misched=0"]})


def ad_variant_flags(variant: str) -> Optional[List[str]]:
    """compile flags of an adjoint-executor variant: the named ones above, or
    "<row|flat>_w<W>_bis<N>" — W tangents per pass and LLVM's optimisation bisection
    stopped after pass N (-opt-bisect-limit, the pass search of the row-form k_ad
    miscompile, tools/ad_bisect.py)"""
    if variant in AD_VARIANTS:
        return AD_VARIANTS[variant]
    import re
    m = re.fullmatch(r"(row|flat)_w(\d)_bis(\d+)", variant or "")
    if not m:
        return None
    return ([] if m.group(1) == "flat" else ["-DTCLB_FLAT_NODE=0"]) + \
        [f"-DTCLB_AD_WINDOW={m.group(2)}", "-mllvm", f"-opt-bisect-limit={m.group(3)}"]


def _variant_of(kind: str, variant: str) -> str:
    """the variant a library of this kind is built in ("" for kinds without variants)"""
    if kind == "hip" or (kind == "cpu" and variant in CPU_VARIANTS) or (kind == "adhip" and ad_variant_flags(variant) is not None):
        return variant
    return ""


def lib_path(model: str, kind: str, variant: str = "") -> str:
    suffix = f"_{variant}" if variant else ""
    return os.path.join(LIB, f"libtclb_{model}_{kind}{suffix}.so")


def _hash_inputs(paths: Iterable[str], extra: str = "") -> str:
    h = hashlib.sha1(extra.encode())
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    return h.hexdigest()


# executor headers: each is included by the instantiation of one library kind only
# (kernels_<kind> of the emitted model), so an edit of one rebuilds that kind alone
_EXECUTOR_OF = {"executor_hip.hpp": ("hip",), "executor_cpu.hpp": ("cpu",), "executor_ad.hpp": ("ad",)}


def _tclb_headers(kind: Optional[str]) -> List[str]:
    inc = os.path.join(CSRC, "include", "tclb")
    return [os.path.join(inc, f) for f in sorted(os.listdir(inc)) if f.endswith((".hpp", ".h"))
            and (kind is None or kind in _EXECUTOR_OF.get(f, (kind,)))]


def _deps(model_dir: str, dynamics: Optional[str], kind: Optional[str] = None) -> List[str]:
    deps = _tclb_headers(kind)
    deps += [os.path.join(model_dir, f) for f in os.listdir(model_dir)
             if f.endswith((".hpp", ".hip", ".cpp")) and f != "kernels_adhip.hip"]
    # the dynamics include and everything it includes from csrc/models (transitively)
    todo = [dynamics] if dynamics else []
    seen = set()
    while todo:
        rel = todo.pop()
        p = os.path.join(CSRC, "models", rel)
        if rel in seen or not os.path.exists(p):
            continue
        seen.add(rel)
        deps.append(p)
        with open(p) as f:
            for line in f:
                s = line.strip()
                if s.startswith("#include \""):
                    todo.append(s.split('"')[1])
    return deps


AD_HIP_DIR = os.path.join(CSRC, "include", "tclb_ad")
TILE_DIR = os.path.join(CSRC, "include", "tclb_tile")


def _tile_deps(model, kind: str) -> List[str]:
    """the LDS-tile kernel headers (csrc/include/tclb_tile, included by executor_hip.hpp):
    a dependency of the HIP libraries of models with LDS-staged stages only, so an edit of
    the tile kernel rebuilds those and not the whole catalog"""
    if kind != "hip" or not any(getattr(st, "lds", None) for st in model.stages):
        return []
    return [os.path.join(TILE_DIR, f) for f in sorted(os.listdir(TILE_DIR)) if f.endswith(".hpp")]


def _adhip_source(model, gen_dir: str) -> str:
    """GPU adjoint executor instantiation (csrc/include/tclb_ad/executor_ad_hip.hpp),
    written next to the emitted model header"""
    from .emit.emitter import ad_tangents
    m = model.finalize()
    src = (f"// AUTO-GENERATED: GPU adjoint (AD) executor for model {m.name}\n"
           f"#define TCLB_AD_K {ad_tangents(m)}\n"
           f"#ifndef TCLB_FLAT_NODE\n#define TCLB_FLAT_NODE 1\n#endif\n"
           f'#include "model.hpp"\n'
           f'#include "tclb_ad/executor_ad_hip.hpp"\n'
           f"TCLB_EXPORT_AD_HIP({m.name}, tclb::M_{m.name}::Model)\n")
    p = os.path.join(gen_dir, "kernels_adhip.hip")
    if not os.path.exists(p) or open(p).read() != src:
        with open(p, "w") as f:
            f.write(src)
    return p


def _cmd(kind: str, src: str, out: str, gen_dir: str, variant: str = "", model_flags=()) -> List[str]:
    """the compile command of one library; model_flags: the model's own HIP defines
    (Model.hip_flags, e.g. the addressing form its collide measured faster with)"""
    incs = ["-I", os.path.join(CSRC, "include"), "-I", os.path.join(CSRC, "models"), "-I", gen_dir]
    if kind == "adhip":
        return [HIPCC, f"--offload-arch={ARCH}", "-O2", "-std=c++17", "-fPIC", "-shared", "-munsafe-fp-atomics",
                "-Wno-unused-result", "-Wno-pass-failed", *(ad_variant_flags(variant) or []), *incs, src, "-o", out]
    if kind == "hip":
        # simplifycfg-sink-common=false: boundary-condition switch cases that permute
        # the population array differ only in constant indices; sinking them into one
        # block turns the indices into PHIs and demotes f[] to scratch (seen as 152 B/lane
        # of scratch in the d3q27_cumulant fp64 kernel).
        return [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
                "-munsafe-fp-atomics", "-mllvm", "-simplifycfg-sink-common=false",
                # AddTo<global> into LDS (core.hpp glob_add): a DPP wave reduction + one
                # LDS atomic per wave instead of the default lane-by-lane loop
                "-mllvm", "-amdgpu-atomic-optimizer-strategy=DPP",
                "-Wno-unused-result", "-Wno-pass-failed", *model_flags, *VARIANTS[variant], *incs,
                src, "-o", out]
    opt = "-O2" if kind == "ad" else "-O3"
    extra = CPU_VARIANTS.get(variant, []) if kind == "cpu" else []
    return [CXX, opt, "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-fno-strict-aliasing",
            "-Wno-unused-variable", *extra, *incs, src, "-o", out]


_PKG = os.path.dirname(os.path.abspath(__file__))


def _rel_hash(paths: Iterable[str], extra: str = "") -> str:
    """like _hash_inputs but independent of where the tree lives (the snapshot a GPU box
    runs sits at another path than the tree the libraries were built in)"""
    h = hashlib.sha1(extra.replace(_PKG, "<pkg>").encode())
    for p in sorted(paths, key=lambda q: os.path.relpath(q, _PKG)):
        with open(p, "rb") as f:
            h.update(os.path.relpath(p, _PKG).encode())
            h.update(f.read())
    return h.hexdigest()


_STAMP_CACHE: Dict[str, str] = {}


def _module_file(mod: str, pkg: str) -> Optional[str]:
    """file of a (possibly relative) module name imported from package `pkg`"""
    if mod.startswith("."):
        lvl = len(mod) - len(mod.lstrip("."))
        parts = pkg.split(".")[:len(pkg.split(".")) - (lvl - 1)]
        mod = ".".join(parts + ([mod.lstrip(".")] if mod.lstrip(".") else []))
    if not mod.startswith("tclb_amd."):
        return None
    base = os.path.join(os.path.dirname(_PKG), *mod.split("."))
    for cand in (base + ".py", os.path.join(base, "__init__.py")):
        if os.path.exists(cand):
            return cand
    return None


def _import_closure(path: str, pkg: str, seen: set):
    """the package-local Python files a model module imports, transitively"""
    import re
    if path in seen:
        return
    seen.add(path)
    with open(path) as f:
        src = f.read()
    for m in re.finditer(r"^\s*from\s+(\.+[\w.]*|tclb_amd[\w.]*)\s+import\s+([\w, ()]+)", src, re.M):
        mod = m.group(1)
        fp = _module_file(mod, pkg)
        names = [n.strip() for n in m.group(2).strip("() ").split(",") if n.strip()]
        if fp is None or fp.endswith("__init__.py"):
            # "from .. import x": x may be a submodule
            for n in names:
                sub = _module_file(mod + ("." if not mod.endswith(".") else "") + n, pkg)
                if sub:
                    sp = ".".join(sub[len(os.path.dirname(_PKG)) + 1:-3].split(os.sep)[:-1])
                    _import_closure(sub, sp, seen)
        if fp:
            sp = ".".join(fp[len(os.path.dirname(_PKG)) + 1:-3].split(os.sep)[:-1])
            _import_closure(fp, sp, seen)


def _python_stamp(name: str) -> str:
    """hash of what a model's generated header depends on besides csrc: the emitter, the
    DSL, the model's module and the package modules it imports, and the registry entry
    (module, builder, options) — an edit elsewhere in models/ leaves the stamp alone"""
    if name not in _STAMP_CACHE:
        files = [os.path.join(d, f) for d, _, fs in os.walk(os.path.join(_PKG, "emit")) for f in fs
                 if f.endswith(".py")]
        files += [os.path.join(_PKG, "models", "dsl.py"), os.path.join(_PKG, "models", "options.py")]
        entry = registry._MODELS.get(name) or registry._resolve(name)
        seen: set = set()
        if entry is not None:
            mod = entry[0]
            fp = _module_file(mod, "tclb_amd.models")
            if fp:
                _import_closure(fp, ".".join(fp[len(os.path.dirname(_PKG)) + 1:-3].split(os.sep)[:-1]), seen)
        files = sorted(set(files) | seen)
        key = repr((entry[0], entry[1], sorted(entry[2].items()))) if entry else name
        _STAMP_CACHE[name] = _rel_hash(files, key)
    return _STAMP_CACHE[name]


def source_stamp(name: str, kind: str, variant: str = "") -> str:
    """cheap fingerprint of everything a model library is built from (the Python model
    definition and emitter, the csrc headers and dynamics includes, the compile command),
    stored next to the library as <lib>.src and checked by ops.abi.load without emitting"""
    model = registry.get(name)
    gdir = os.path.join(BUILD, "gen", name)
    v = _variant_of(kind, variant)
    cmd = _cmd(kind, os.path.join(gdir, "kernels_" + kind), lib_path(name, kind, v), gdir, v,
               getattr(model, "hip_flags", ()))
    deps = _deps_no_gen(model.dynamics, kind) + (_ad_hip_deps() if kind == "adhip" else []) + _tile_deps(model, kind)
    return _rel_hash(deps, " ".join(cmd) + _python_stamp(name))


def _ad_hip_deps() -> List[str]:
    return [os.path.join(AD_HIP_DIR, f) for f in sorted(os.listdir(AD_HIP_DIR)) if f.endswith(".hpp")]


def _deps_no_gen(dynamics: Optional[str], kind: Optional[str] = None) -> List[str]:
    deps = _tclb_headers(kind)
    todo, seen = ([dynamics] if dynamics else []), set()
    while todo:
        rel = todo.pop()
        p = os.path.join(CSRC, "models", rel)
        if rel in seen or not os.path.exists(p):
            continue
        seen.add(rel)
        deps.append(p)
        with open(p) as f:
            todo += [ln.strip().split('"')[1] for ln in f if ln.strip().startswith("#include \"")]
    return deps


def stale_reason(name: str, kind: str, variant: str = "") -> Optional[str]:
    """None when the library exists and was built from the current sources"""
    v = _variant_of(kind, variant)
    target = lib_path(name, kind, v)
    if not os.path.exists(target):
        return "missing"
    stamp = target + ".src"
    if not os.path.exists(stamp):
        return "no source stamp"
    with open(stamp) as f:
        if f.read() != source_stamp(name, kind, variant):
            return "sources changed since it was built"
    return None


def build_model(name: str, kinds=("cpu", "hip"), force: bool = False, verbose: bool = False,
                variant: str = "", paths: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    """compile one model's libraries of the given kinds (skipped when the stamped inputs
    are unchanged); paths: the model's emit_model result, when the caller emitted it
    already (build_all emits every model once, then compiles its kinds in parallel)"""
    model = registry.get(name)
    paths = paths or emit_model(model)
    os.makedirs(LIB, exist_ok=True)
    out = {}
    for kind in kinds:
        if kind in ("hip", "adhip") and not os.path.exists(HIPCC):
            continue
        v = _variant_of(kind, variant)
        target = lib_path(name, kind, v)
        src = _adhip_source(model, paths["dir"]) if kind == "adhip" else paths[kind]
        cmd = _cmd(kind, src, target, paths["dir"], v, getattr(model, "hip_flags", ()))
        deps = (_deps(paths["dir"], model.dynamics, kind) + (_ad_hip_deps() if kind == "adhip" else [])
                + _tile_deps(model, kind))
        h = _hash_inputs(deps, " ".join(cmd))
        stamp = target + ".hash"
        if not force and os.path.exists(target) and os.path.exists(stamp) and open(stamp).read() == h:
            _write_src_stamp(name, kind, variant)
            out[kind] = target
            continue
        t0 = time.time()
        tmp = f"{target}.{os.getpid()}.{threading.get_ident()}.tmp"
        cmd[-1] = tmp
        # stamps describe the sources as they were when the compiler read them: an edit
        # made during the compile leaves the library stale, not falsely fresh
        src_stamp = source_stamp(name, kind, variant)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"build of {name} [{kind}] failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr[-20000:]}")
        os.replace(tmp, target)
        with open(stamp, "w") as f:
            f.write(h)
        _write_src_stamp(name, kind, variant, src_stamp)
        if verbose:
            print(f"[tclb build] {name} [{kind}{'/' + v if v else ''}] {time.time() - t0:.1f}s", flush=True)
        out[kind] = target
    return out


def _write_src_stamp(name: str, kind: str, variant: str, s: Optional[str] = None):
    v = _variant_of(kind, variant)
    s = source_stamp(name, kind, variant) if s is None else s
    p = lib_path(name, kind, v) + ".src"
    if not os.path.exists(p) or open(p).read() != s:
        with open(p, "w") as f:
            f.write(s)


def _rt_headers() -> List[str]:
    """headers of the native runtime libraries (not of the model libraries: an edit here
    rebuilds libtclb_host.so / libtclb_device.so only)"""
    d = os.path.join(CSRC, "include", "tclb_rt")
    return [os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith(".hpp")] + \
        [os.path.join(CSRC, "include", "tclb", "core.hpp")]


def host_runtime_stale() -> Optional[str]:
    """why libtclb_host.so cannot be used as is (None: fresh)"""
    target = os.path.join(LIB, "libtclb_host.so")
    if not os.path.exists(target):
        return "missing"
    rdir = os.path.join(CSRC, "runtime")
    srcs = sorted(os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".cpp"))
    stamp = target + ".hash"
    if not os.path.exists(stamp) or open(stamp).read() != _rel_hash(srcs + _rt_headers(),
                                                                      " ".join(_host_cmd(srcs, target))):
        return "sources changed"
    return None


def _host_cmd(srcs: List[str], target: str) -> List[str]:
    return [CXX, "-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-I", os.path.join(CSRC, "include"),
            *srcs, "-lz", "-o", target]


def build_host(force: bool = False, verbose: bool = False) -> str:
    """native host runtime library (geometry voxeliser, scans, HDF5 and PNG writers): libtclb_host.so
    from every csrc/runtime/*.cpp"""
    rdir = os.path.join(CSRC, "runtime")
    srcs = sorted(os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".cpp"))
    target = os.path.join(LIB, "libtclb_host.so")
    os.makedirs(LIB, exist_ok=True)
    cmd = _host_cmd(srcs, target)
    h = _rel_hash(srcs + _rt_headers(), " ".join(cmd))
    stamp = target + ".hash"
    if not force and os.path.exists(target) and os.path.exists(stamp) and open(stamp).read() == h:
        return target
    # a per-process temporary: ranks started together may build at once (atomic rename)
    tmp = f"{target}.{os.getpid()}.tmp"
    r = subprocess.run(cmd[:-1] + [tmp], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host library build failed:\n{r.stderr[-10000:]}")
    os.replace(tmp, target)
    with open(stamp, "w") as f:
        f.write(h)
    if verbose:
        print("[tclb build] host runtime", flush=True)
    return target


BIN = os.path.join(BUILD, "bin")


def tool_path(name: str) -> str:
    return os.path.join(BIN, f"tclb-{name}")


def build_tools(force: bool = False, verbose: bool = False) -> Dict[str, str]:
    """native auxiliary executables (reference src/compare.cpp etc.): csrc/tools/<name>.cpp
    -> _build/bin/tclb-<name>"""
    tdir = os.path.join(CSRC, "tools")
    os.makedirs(BIN, exist_ok=True)
    out = {}
    for fn in sorted(os.listdir(tdir)):
        if not fn.endswith(".cpp"):
            continue
        name = fn[:-4]
        src = os.path.join(tdir, fn)
        target = tool_path(name)
        cmd = [CXX, "-O2", "-std=c++17", "-fopenmp", src, "-o", target + ".tmp"]
        h = _hash_inputs([src], " ".join(cmd))
        stamp = target + ".hash"
        if force or not (os.path.exists(target) and os.path.exists(stamp) and open(stamp).read() == h):
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"tool {name} build failed:\n{r.stderr[-10000:]}")
            os.replace(target + ".tmp", target)
            with open(stamp, "w") as f:
                f.write(h)
            if verbose:
                print(f"[tclb build] tool tclb-{name}", flush=True)
        out[name] = target
    return out


def bench_lib_path(name: str) -> str:
    return os.path.join(LIB, f"libtclb_{name}.so")


def _device_cmd(srcs: List[str]) -> List[str]:
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-I", os.path.join(CSRC, "include"), *srcs, "-ldl", "-o"]


def build_device_runtime(force: bool = False, verbose: bool = False) -> Optional[str]:
    """model-independent HIP kernels of the runtime (csrc/device/*.hip: the per-step
    particle kernels) -> _build/lib/libtclb_device.so"""
    if not os.path.exists(HIPCC):
        return None
    ddir = os.path.join(CSRC, "device")
    srcs = sorted(os.path.join(ddir, f) for f in os.listdir(ddir) if f.endswith(".hip"))
    target = os.path.join(LIB, "libtclb_device.so")
    os.makedirs(LIB, exist_ok=True)
    cmd = _device_cmd(srcs)
    h = _rel_hash(srcs + _rt_headers(), " ".join(cmd))
    stamp = target + ".hash"
    if not force and os.path.exists(target) and os.path.exists(stamp) and open(stamp).read() == h:
        return target
    tmp = f"{target}.{os.getpid()}.tmp"
    r = subprocess.run(cmd + [tmp], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"device runtime build failed:\n{r.stderr[-10000:]}")
    os.replace(tmp, target)
    with open(stamp, "w") as f:
        f.write(h)
    if verbose:
        print("[tclb build] device runtime", flush=True)
    return target


def device_runtime_stale() -> Optional[str]:
    """why libtclb_device.so cannot be used as is (None: fresh)"""
    ddir = os.path.join(CSRC, "device")
    srcs = sorted(os.path.join(ddir, f) for f in os.listdir(ddir) if f.endswith(".hip"))
    target = os.path.join(LIB, "libtclb_device.so")
    cmd = _device_cmd(srcs)
    if not os.path.exists(target):
        return "missing"
    stamp = target + ".hash"
    if not os.path.exists(stamp) or open(stamp).read() != _rel_hash(srcs + _rt_headers(), " ".join(cmd)):
        return "sources changed"
    return None


def build_bench_libs(force: bool = False, verbose: bool = False) -> Dict[str, str]:
    """stand-alone HIP micro-benchmarks (csrc/bench/<name>.hip -> _build/lib/libtclb_<name>.so),
    e.g. the LDS A/B of the 27-point stencil (tools/lds_ab.py)"""
    bdir = os.path.join(CSRC, "bench")
    os.makedirs(LIB, exist_ok=True)
    out = {}
    if not os.path.exists(HIPCC):
        return out
    for fn in sorted(os.listdir(bdir)):
        if not fn.endswith(".hip"):
            continue
        name = fn[:-4]
        src = os.path.join(bdir, fn)
        target = bench_lib_path(name)
        tmp = f"{target}.{os.getpid()}.tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", src, "-o"]
        h = _hash_inputs([src], " ".join(cmd))
        stamp = target + ".hash"
        if force or not (os.path.exists(target) and os.path.exists(stamp) and open(stamp).read() == h):
            r = subprocess.run(cmd + [tmp], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"bench lib {name} build failed:\n{r.stderr[-10000:]}")
            os.replace(tmp, target)
            with open(stamp, "w") as f:
                f.write(h)
            if verbose:
                print(f"[tclb build] bench lib {name}", flush=True)
        out[name] = target
    return out


def build_all(models: Optional[List[str]] = None, kinds=("cpu", "hip"), jobs: int = 0, force=False,
              verbose=False) -> Dict[str, Dict[str, str]]:
    models = models or registry.names()
    build_host(force=force, verbose=verbose)
    build_device_runtime(force=force, verbose=verbose)
    build_tools(force=force, verbose=verbose)
    jobs = jobs or max(1, min(8, os.cpu_count() or 1))
    tasks = [(m, k) for m in models for k in kinds]
    res: Dict[str, Dict[str, str]] = {m: {} for m in models}
    # emit serially (sympy + file writes), compile in parallel
    emitted = {m: emit_model(registry.get(m)) for m in models}
    errors = []

    def one(t):
        m, k = t
        try:
            return m, k, build_model(m, kinds=(k,), force=force, verbose=verbose, paths=emitted[m]).get(k), None
        except Exception as e:  # noqa
            return m, k, None, e

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for m, k, p, e in ex.map(one, tasks):
            if e is not None:
                errors.append(e)
            elif p:
                res[m][k] = p
    if errors:
        raise RuntimeError("\n\n".join(str(e) for e in errors))
    return res


def build_adjoint_libs(models: Optional[List[str]] = None, jobs: int = 0, force=False,
                       verbose=False) -> Dict[str, Dict[str, str]]:
    """dual-number adjoint executors (CPU "ad" and GPU "adhip") of the reference's ADJOINT=1
    models plus d2q9_kuper (the two-stage stencil model of the GPU adjoint test), so GPU
    runs load prebuilt libraries instead of compiling them on first use"""
    from .models.dsl import ADJOINT_MODELS
    models = models or sorted(ADJOINT_MODELS | {"d2q9_kuper"})
    kinds = ("ad", "adhip") if os.path.exists(HIPCC) else ("ad",)
    jobs = jobs or max(1, min(8, os.cpu_count() or 1))
    emitted = {m: emit_model(registry.get(m)) for m in models}

    def one(t):
        m, k = t
        return m, k, build_model(m, kinds=(k,), force=force, verbose=verbose, paths=emitted[m]).get(k)

    res: Dict[str, Dict[str, str]] = {m: {} for m in models}
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for m, k, p in ex.map(one, [(m, k) for m in models for k in kinds]):
            res[m][k] = p
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description="build tclb_amd model kernels")
    ap.add_argument("models", nargs="*")
    ap.add_argument("--kinds", default="cpu,hip")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build_all(a.models or None, kinds=tuple(a.kinds.split(",")), jobs=a.jobs, force=a.force, verbose=True)


if __name__ == "__main__":
    main()
