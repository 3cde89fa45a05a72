"""UndefinedBehaviorSanitizer run of the CPU executor (build variant "ubsan",
build.CPU_VARIANTS): the node code of a few model families steps a small lattice with
-fsanitize=undefined -fno-sanitize-recover (any signed overflow, misaligned or
out-of-bounds array access, invalid shift... aborts).  Each model runs in a child
process so an abort is reported, not fatal to pytest.  Host-side sanitizers only: GPU
sanitizer runs are not available on the MI355X pool."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import numpy as np, sys
from tclb_amd.lattice import Lattice
name, shape = sys.argv[1], tuple(int(v) for v in sys.argv[2].split(","))
lat = Lattice(name, shape, variant="ubsan")
assert lat.lib.path.endswith("_cpu_ubsan.so"), lat.lib.path
m = lat.model
coll = next(t for t in m.node_types if t.group == "COLLISION")
fl = np.full((lat.NZ, lat.NY, shape[0]), coll.value, dtype=np.uint32)
wall = m.node_type("Wall")
if wall is not None:
    fl[:, 0, :] = wall.value
lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
lat.init()
lat.iterate(3)
for q in m.quantities:
    if not q.adjoint:
        lat.quantity(q.name)
print("ok", name)
"""


@pytest.mark.parametrize("name,shape", [("d2q9", "16,8,1"), ("d3q27", "8,6,4"), ("d2q9_kuper", "12,8,1"),
                                        ("d3q27_cumulant", "6,6,4"),
                                        ("d3q27_tePSM_per_NEBB", "8,6,4"), ("d3q27_pf_velocity", "8,6,4")])
def test_model_under_ubsan(name, shape):
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-c", SCRIPT, name, shape], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert f"ok {name}" in r.stdout


@pytest.mark.parametrize("name,args", [("d3q27_tePSM_per_NEBB", []), ("d3q27_tePSM_per_NEBB", ["--glob"]),
                                       ("d3q27_pf_velocity", []),
                                       ("d3q27_pf_velocity_thermo", ["--stage", "NonLocalTemp"]),
                                       ("d2q9_pf_velocity", ["--stage", "WallIter"])])
def test_split_class_forms_under_msan(name, args):
    """the GPU-only class instantiations of split stages (Node<..., CLS_ 1 and 2>, run per
    node class as the GPU dispatches them) on the host under MemorySanitizer: no branch on
    an uninitialised value and no uninitialised byte stored into the output snapshot
    (tools/msan_node.py; verdict r05: the class-2 tePSM kernel's wrong wall values)"""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "msan_node.py"), name, *args],
                       capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert '"rc": 0' in r.stdout.splitlines()[-1]
