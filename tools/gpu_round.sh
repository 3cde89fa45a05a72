#!/bin/bash
# One GPU session: tests, benches, rocprof stats.  Every GPU step has its own timeout;
# steps are chained with && so the first failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
echo "== gpu tests" && timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 ; tail -3 $O/pytest_gpu.log
echo "== bench fp64" && timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_fp64.json 2> $O/bench_fp64.err && cat $O/bench_fp64.json &&
echo "== bench fp32" && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --precision float > $O/bench_fp32.json 2> $O/bench_fp32.err && cat $O/bench_fp32.json &&
echo "== rocprof" && cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1 ; echo "rocprof rc=$?"; ls -R $O/prof | head -20
