#!/bin/bash
# Developer GPU session (run through gpurun): tests, benches, counters, kernel stats.
#   scripts/gpu_round.sh [tests|bench|counters|prof|models|all] ...
# Every GPU step has its own timeout; a crash/timeout (rc >= 124) ends the call, and
# only an ordinary test failure (rc 1) lets the following steps run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
step() {  # step <name> <timeout> <logfile> cmd...
  local name=$1 t=$2 log=$3; shift 3
  echo "== $name"
  timeout -k 10 $t "$@" > $log 2>&1
  local rc=$?
  tail -3 $log
  echo "   rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for WHAT in "${@:-all}"; do
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  step "gpu tests" 900 $O/pytest_gpu.log python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  step "bench fp64" 300 $O/bench_fp64.json python bench.py --steps 100 --warmup 10
  step "bench fp32" 300 $O/bench_fp32.json python bench.py --steps 100 --warmup 10 --precision float
fi
if [ "$WHAT" = all ] || [ "$WHAT" = counters ]; then
  export TMPDIR=/tmp
  step "calib copy counters" 400 $O/counters_calib.log python tools/counters.py --tag calib_copy --outdir $O/counters -- python3 $R/tools/calib_copy.py
  step "d3q27 counters" 400 $O/counters_d3q27.log python tools/counters.py --tag d3q27_512_fp64 --nodes 134217728 --outdir $O/counters -- python3 $R/bench.py --steps 5 --warmup 1
fi
if [ "$WHAT" = all ] || [ "$WHAT" = models ]; then
  step "model table" 600 $O/perf_models_fp64.log python tools/perf_models.py
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  export TMPDIR=/tmp
  step "rocprof" 400 $O/prof.log rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2
fi
done
