set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python tools/bench_configs.py > $O/bench_configs_fp64.log 2>&1 || exit $?
cat $O/bench_configs_fp64.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_pf -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs pf384 --steps 10 > $GRAFT_REPO_ROOT/$O/prof_pf.log 2>&1 || exit $?
find $GRAFT_REPO_ROOT/$O/prof_pf -name "*stats*"
