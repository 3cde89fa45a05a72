#!/bin/bash
# r02 second GPU session: tests (new variants), host overhead, karman, bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
step() { local name=$1 t=$2 log=$3; shift 3; echo "== $name"; timeout -k 10 $t "$@" > $log 2>&1; local rc=$?; tail -4 $log; echo "   rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi; return 0; }
step "gpu tests" 900 $O/pytest_gpu_r02b.log python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread
step "host overhead" 120 $O/host_overhead.log python tools/host_overhead.py --steps 2000
step "karman" 300 $O/karman.log python tools/bench_karman.py --iters 10000
step "bench" 300 $O/bench_r02b.json python bench.py
