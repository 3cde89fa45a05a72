set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python tools/debug_hip_cpu.py d2q9_pf 3 > $O/debug_pf.log 2>&1; rc=$?; cat $O/debug_pf.log | tail -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -m pytest tests -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
