#!/bin/bash
# Headline A/B on one box: round-2 HEAD (894c645, extracted to _ab_r02/ with its own
# d3q27 library) against this tree, interleaved A B A B ... so box drift hits both.
#   scripts/headline_ab.sh [rounds] [precision...]
# writes gpurun_out/ab/headline_ab.log (one JSON line per run, tagged)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab; mkdir -p $O; cd $R
ROUNDS=${1:-3}; shift || true
PRECS=${@:-double mixed-shift}
LOG=$O/headline_ab.log
: > $LOG
export TCLB_NO_BUILD=1
for r in $(seq 1 $ROUNDS); do
  for p in $PRECS; do
    for side in r02 head; do
      if [ $side = r02 ]; then dir=$R/_ab_r02; else dir=$R; fi
      out=$(cd $dir && timeout -k 10 240 python bench.py --steps 100 --warmup 10 --precision $p 2>$O/err_${side}.log)
      rc=$?
      if [ $rc -ne 0 ]; then echo "run $side $p failed rc=$rc" | tee -a $LOG; tail -5 $O/err_${side}.log; exit $rc; fi
      line=$(echo "$out" | grep '^{')
      echo "{\"side\": \"$side\", \"round\": $r, \"precision\": \"$p\", \"bench\": $line}" | tee -a $LOG
    done
  done
done
