#!/usr/bin/env python3
"""Static instruction profile of the stage kernels of one model library (gfx950 ISA).

For every kernel of ``libtclb_<model>_hip[_variant].so`` whose name matches ``--match``
(default: the plain k_stage instantiations), print VGPR / AGPR / SGPR counts, scratch
bytes, the occupancy the register count allows (waves per SIMD, 512 VGPRs per SIMD lane
split in 8-register granules) and the static instruction mix of its code: VALU (split
into fp64 FMA / mul / add, other fp64, fp32, integer / moves), VMEM loads / stores,
LDS, SALU, SMEM, branches.  The counts are of the instruction stream, not dynamic
counts, but a straight-line collide kernel executes nearly all of it once per wave, so
they are the budget a change to the node code is weighed by (round-4 counters: the
pf_velocity mixed-shift collide issued 1 433 VALU per wave).

    python tools/isa_stats.py d3q27_pf_velocity [--variant V] [--match 'k_stage<'] [--stage 0]
    python tools/isa_stats.py --scan [--min-regs 256]    # every model: kernels above 256 regs
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def code_object(so: str, tmp: str) -> str:
    fb, co = os.path.join(tmp, "fb.bin"), os.path.join(tmp, "co.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so, os.path.join(tmp, "x.o")],
                   check=True, capture_output=True)
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={fb}"],
                       capture_output=True, text=True)
    tgt = [t for t in r.stdout.split() if "gfx950" in t][0]
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    f"--targets={tgt}", f"--output={co}"], check=True, capture_output=True)
    return co


def classify(op: str) -> str:
    if op.startswith("v_"):
        if re.match(r"v_(fma|fmac)_f64", op):
            return "valu_f64_fma"
        if op.startswith("v_mul_f64"):
            return "valu_f64_mul"
        if op.startswith("v_add_f64"):
            return "valu_f64_add"
        if "f64" in op:
            return "valu_f64_other"
        if "f32" in op or "f16" in op:
            return "valu_f32"
        return "valu_int_mov"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


def kernels(co: str):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    meta = {}
    # one YAML map per kernel, keys in alphabetical order: .agpr_count opens each entry
    for blk in notes.split(".agpr_count:")[1:]:
        m = re.search(r"\.name:\s*(\S+)", blk)
        if not m:
            continue
        g = lambda k: int(m2.group(1)) if (m2 := re.search(rf"\.{k}:\s*(\d+)", blk)) else -1  # noqa: E731
        agpr = int(blk.split("\n")[0].strip())
        meta[m.group(1)] = {"vgpr": g("vgpr_count"), "agpr": agpr, "sgpr": g("sgpr_count"),
                            "scratch": g("private_segment_fixed_size"), "lds": g("group_segment_fixed_size")}
    return meta


def disasm(co: str):
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                         text=True).stdout
    out, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            out[cur] = Counter()
            continue
        if cur and line.startswith("\t"):
            op = line.strip().split()[0] if line.strip() else ""
            if op:
                out[cur][classify(op)] += 1
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


def scan(min_regs: int, match: str):
    """every built model library (default variants): the kernels whose unified register
    count (arch VGPRs + AGPRs) exceeds min_regs — the ones whose occupancy and register
    allocation (AGPR use, spills) make them the riskiest code the compiler emits here"""
    from tclb_amd import build as B
    from tclb_amd.models import registry
    print("model,kernel,vgpr,agpr,scratch,waves_per_simd")
    for name in registry.all_variants():
        so = B.lib_path(name, "hip", "")
        if not os.path.exists(so):
            continue
        with tempfile.TemporaryDirectory() as tmp:
            try:
                meta = kernels(code_object(so, tmp))
            except (subprocess.CalledProcessError, IndexError):
                continue
        big = [n for n in sorted(meta) if meta[n]["vgpr"] > min_regs]
        for n, d in zip(big, demangle(big)):
            if match not in d:
                continue
            mt = meta[n]
            waves = min(8, 512 // ((mt["vgpr"] + 7) // 8 * 8))
            short = re.sub(r"tclb::M_\w+::Model, ", "", d)
            short = short if len(short) < 120 else short[:117] + "..."
            print(f"{name},\"{short}\",{mt['vgpr']},{mt['agpr']},{mt['scratch']},{waves}", flush=True)


def main():
    if "--scan" in sys.argv:
        ap = argparse.ArgumentParser()
        ap.add_argument("--scan", action="store_true")
        ap.add_argument("--min-regs", type=int, default=256)
        ap.add_argument("--match", default="tclb::exec::k_")
        a = ap.parse_args()
        scan(a.min_regs, a.match)
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("--variant", default="")
    ap.add_argument("--kind", default="hip")
    ap.add_argument("--match", default="k_stage<")
    ap.add_argument("--stage", type=int, default=None, help="stage index (4th template argument)")
    a = ap.parse_args()
    from tclb_amd import build as B
    so = B.lib_path(a.model, a.kind, a.variant)
    with tempfile.TemporaryDirectory() as tmp:
        co = code_object(so, tmp)
        meta = kernels(co)
        dis = disasm(co)
    names = sorted(meta)
    dem = dict(zip(names, demangle(names)))
    cols = ["valu_f64_fma", "valu_f64_mul", "valu_f64_add", "valu_f64_other", "valu_f32", "valu_int_mov",
            "vmem_load", "vmem_store", "lds", "salu", "smem", "branch", "scratch"]
    print("kernel,vgpr,agpr,sgpr,scratch,waves_per_simd,valu_total," + ",".join(cols))
    for n in names:
        d = dem[n]
        if a.match not in d:
            continue
        if a.stage is not None:
            targs = re.search(r"<(.*)>\(", d)
            if not targs or f", {a.stage}, " not in targs.group(1):
                continue
        mt, c = meta[n], dis.get(n.replace(".kd", ""), Counter())
        # .vgpr_count is the unified file (arch VGPRs + AGPRs, e.g. 344 = 256 + 88)
        regs = max(1, mt["vgpr"])
        waves = min(8, 512 // ((regs + 7) // 8 * 8))
        valu = sum(v for k, v in c.items() if k.startswith("valu"))
        short = d if len(d) < 140 else d[:137] + "..."
        print(f"\"{short}\",{mt['vgpr']},{mt['agpr']},{mt['sgpr']},{mt['scratch']},{waves},{valu}," +
              ",".join(str(c.get(k, 0)) for k in cols))


if __name__ == "__main__":
    main()
