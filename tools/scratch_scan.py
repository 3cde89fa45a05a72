#!/usr/bin/env python3
"""Scratch (private segment) use of every stage kernel in the built HIP libraries.

Reads the gfx950 code object out of each ``_build/lib/libtclb_*_hip.so`` (``.hip_fatbin``
section, clang-offload-bundler) and prints the stage kernels whose metadata declares a
private segment (``.private_segment_fixed_size`` > 0: spills or runtime-indexed arrays),
with their VGPR count and the number of scratch load/store instructions in their code
(a frame the backend reserves, e.g. an emergency register-scavenging slot, shows as bytes
with 0 accesses and costs nothing).  Kernels not listed keep the whole node in registers.

    python tools/scratch_scan.py [--lib-dir DIR] [--all]
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_scratch(so: str, tmp: str, kernel_filter: str = "k_stage"):
    fb, co = os.path.join(tmp, "fb.bin"), os.path.join(tmp, "co.o")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so, os.path.join(tmp, "x.o")],
                   check=True, capture_output=True)
    r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={fb}"],
                       capture_output=True, text=True)
    tgt = [t for t in r.stdout.split() if "gfx950" in t]
    if not tgt:
        return []
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    f"--targets={tgt[0]}", f"--output={co}"], check=True, capture_output=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    out = []
    for blk in notes.split(".name:")[1:]:
        name = blk.split("\n")[0].strip()
        m = re.search(r"\.private_segment_fixed_size:\s*(\d+)", blk)
        v = re.search(r"\.vgpr_count:\s*(\d+)", blk)
        if m and kernel_filter in name:
            out.append((int(m.group(1)), int(v.group(1)) if v else -1, name))
    return out


SCRATCH_OP = re.compile(r"\b(scratch_(load|store)\w*|buffer_(load|store)\w*)\b")


def scratch_accesses(co: str, name: str) -> int:
    """scratch load/store instructions in the disassembly of one kernel"""
    r = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"--disassemble-symbols={name}", co],
                       capture_output=True, text=True)
    return len(SCRATCH_OP.findall(r.stdout))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib-dir", default=os.path.join(REPO, "tclb_amd", "_build", "lib"))
    ap.add_argument("--all", action="store_true", help="also list the kernels without scratch")
    a = ap.parse_args()
    libs = sorted(glob.glob(os.path.join(a.lib_dir, "libtclb_*_hip.so")))
    nk = nscr = nacc = 0
    with tempfile.TemporaryDirectory() as tmp:
        for so in libs:
            for scr, vgpr, name in kernel_scratch(so, tmp):
                nk += 1
                acc = scratch_accesses(os.path.join(tmp, "co.o"), name) if scr > 0 else 0
                if scr > 0 or a.all:
                    nscr += scr > 0
                    nacc += acc > 0
                    print(f"{os.path.basename(so)}\t{scr} B/lane\t{acc} scratch ops\t{vgpr} VGPR\t{name}")
    print(f"{len(libs)} libraries, {nk} stage kernels, {nscr} with a private segment, "
          f"{nacc} with scratch accesses", file=sys.stderr)


if __name__ == "__main__":
    main()
