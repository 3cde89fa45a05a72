#!/bin/bash
# Round-5 GPU session steps (run through gpurun):  scripts/gpu_r05.sh <step>...
# Every GPU step has its own timeout; a crash/timeout (rc >= 124, or any rc > 1) ends the
# call; an ordinary test failure (rc 1) lets the following steps run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-r05}
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
for WHAT in "$@"; do
case $WHAT in
tests) step "gpu tests" 900 $O/pytest_gpu.log python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider ;;
newtests) step "gpu native-loop tests" 600 $O/pytest_native.log python -u -m pytest tests/test_native_loop.py tests/test_particles.py -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider ;;
smoke) step "smoke" 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
bench) step "bench fp64 20" 300 $O/bench20.json python bench.py --steps 20 --warmup 5 ;;
split) step "tile split probe fp64" 600 $O/split_fp64.jsonl python tools/direction_probe.py --detail --repeat 3 --variants default ;;
splitms) step "tile split probe mixed-shift" 600 $O/split_ms.jsonl python tools/direction_probe.py --detail --repeat 2 --variants default --precision mixed-shift ;;
*) echo "unknown step $WHAT"; exit 2 ;;
esac
done
