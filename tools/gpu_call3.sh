set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python tools/perf_models.py > $O/perf_models_fp64.log 2>&1 || exit $?
tail -5 $O/perf_models_fp64.log
