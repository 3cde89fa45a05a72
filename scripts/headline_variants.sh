#!/bin/bash
# Headline build-variant A/B on one box: the default d3q27 library against the round-3
# A/B variants (flataddr = flat 64-bit addresses, gregs = register globals accumulators,
# plain = no non-temporal stores) and the round-2 tree, interleaved.
#   [VARIANTS="r02 default ..."] scripts/headline_variants.sh [rounds] [precision...]
#     -> gpurun_out/ab/variants.log
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab; mkdir -p $O; cd $R
ROUNDS=${1:-2}; shift || true
PRECS=${@:-mixed-shift double}
LOG=$O/variants.log
: > $LOG
export TCLB_NO_BUILD=1
for r in $(seq 1 $ROUNDS); do
  for p in $PRECS; do
    for v in ${VARIANTS:-r02 default flataddr gregs plain}; do
      if [ $v = r02 ]; then dir=$R/_ab_r02; var=""; else dir=$R; var=$v; [ $v = default ] && var=""; fi
      out=$(cd $dir && TCLB_VARIANT=$var timeout -k 10 240 python bench.py --steps 100 --warmup 10 --precision $p 2>$O/err_$v.log)
      rc=$?
      if [ $rc -ne 0 ]; then echo "run $v $p failed rc=$rc" | tee -a $LOG; tail -5 $O/err_$v.log; exit $rc; fi
      line=$(echo "$out" | grep '^{')
      echo "{\"variant\": \"$v\", \"round\": $r, \"precision\": \"$p\", \"bench\": $line}" | tee -a $LOG
    done
  done
done
