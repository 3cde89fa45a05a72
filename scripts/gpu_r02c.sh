#!/bin/bash
# r02 third GPU session: tests (sampler, reduced storage, scmp/csf fixes), benches of
# the storage modes, karman compute-only, counters / kernel stats.
#   scripts/gpu_r02c.sh [tests] [bench] [karman] [prof] [counters] [configs]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
step() { local name=$1 t=$2 log=$3; shift 3; echo "== $name"; timeout -k 10 $t "$@" > $log 2>&1; local rc=$?; tail -4 $log; echo "   rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
for W in "$@"; do case $W in
newtests) step "new gpu tests" 400 $O/pytest_gpu_r02c_new.log python -u -m pytest tests/test_gpu_oracles.py tests/test_gpu_kernels.py -v -m gpu --timeout 120 --timeout-method thread ;;
tests) step "gpu tests" 900 $O/pytest_gpu_r02c.log python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ;;
bench)
  step "bench fp64" 300 $O/bench_r02c_fp64.json python bench.py
  step "bench mixed-shift" 300 $O/bench_r02c_mixed_shift.json python bench.py --precision mixed-shift
  step "bench mixed" 300 $O/bench_r02c_mixed.json python bench.py --precision mixed
  step "bench half-shift" 300 $O/bench_r02c_half_shift.json python bench.py --precision half-shift ;;
karman) step "karman compute-only" 300 $O/karman_novtk.log python tools/bench_karman.py --iters 20000 --vtk 0 ;;
prof) step "rocprof mixed-shift" 400 $O/prof_mixed_shift.log rocprofv3 --kernel-trace --stats -d $O/prof_mixed_shift -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --precision mixed-shift ;;
counters)
  step "counters d3q27 mixed-shift" 500 $O/counters_d3q27_ms.log python tools/counters.py --tag d3q27_512_mixed_shift --nodes 134217728 --outdir $O/counters -- python3 $R/bench.py --steps 5 --warmup 1 --precision mixed-shift
  step "counters pf384" 500 $O/counters_pf384.log python tools/counters.py --tag pf384_fp64 --nodes 56623104 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs pf384 --steps 5 --warmup 1 ;;
adjoint)
  step "gpu adjoint tests" 600 $O/pytest_gpu_adjoint.log python -u -m pytest tests/test_gpu_adjoint.py -v -m gpu --timeout 300 --timeout-method thread
  step "adjoint bench 64" 300 $O/bench_adjoint_64.json python tools/bench_adjoint.py --size 64 --steps 10
  step "adjoint bench 128" 400 $O/bench_adjoint_128.json python tools/bench_adjoint.py --size 128 --steps 10 ;;
configs) step "configs" 400 $O/configs_r02c.log python tools/bench_configs.py ;;
esac; done
