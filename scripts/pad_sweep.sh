# field-plane padding sweep for the headline d3q27 fp64 bench (one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
: > $O/pad_sweep.log
for pad in 0 64 512 4160 0 64 512 4160; do
  echo "pad=$pad" >> $O/pad_sweep.log
  TCLB_FIELD_PAD=$pad timeout -k 10 240 python bench.py --steps 30 --warmup 5 >> $O/pad_sweep.log 2>&1 || exit $?
done
grep -E "pad=|metric" $O/pad_sweep.log | sed 's/.*"value": \([0-9.]*\).*/\1/'
