#!/bin/bash
# RCCL self-send on a slab against the channel count: physics checks of bench.py decide
# (rc 3 = a check failed; rc >= 124 or a signal: stop)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-rcclch}; mkdir -p $O; cd $R
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  echo "== $name"
  timeout -k 10 300 env "${envs[@]}" python bench.py "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  tail -c 300 $O/$name.json; grep -h "physics check" $O/$name.err | cut -c1-300
  echo "   rc=$rc"
  if [ $rc -ge 124 ] || { [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 3 ]; }; then echo "stopping (rc=$rc)"; exit $rc; fi
}
S="--steps 50 --warmup 5 --loopback-dist --transport rccl"
run ch1_chunked NCCL_MAX_NCHANNELS=1 NCCL_MIN_NCHANNELS=1 -- --shape 512,512,64 $S
run ch1_whole NCCL_MAX_NCHANNELS=1 NCCL_MIN_NCHANNELS=1 TCLB_RCCL_CHUNK_MB=0 -- --shape 512,512,64 $S
run ch1_chunked_ms NCCL_MAX_NCHANNELS=1 NCCL_MIN_NCHANNELS=1 -- --shape 512,512,64 $S --precision mixed-shift
run ch2_chunked NCCL_MAX_NCHANNELS=2 NCCL_MIN_NCHANNELS=1 -- --shape 512,512,64 $S
for rep in 1 2; do
run default_chunked_$rep TCLB_X=0 -- --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport rccl
run default_whole_$rep TCLB_RCCL_CHUNK_MB=0 -- --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport rccl
run chunk16_$rep TCLB_RCCL_CHUNK_MB=16 -- --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport rccl
run plain_$rep TCLB_X=0 -- --shape 512,512,64 --steps 200 --warmup 20
done
