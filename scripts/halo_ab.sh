#!/bin/bash
# halo-exchange A/B on one MI355X (round 6): the per-rank slab shapes of the 8-GPU
# headline (512x512x64 fp64) and the 4-GPU part256 case (256x256x64) stepped as one rank
# through the multi-rank loop with each transport (copy / RCCL to itself / IPC pull from
# itself), against the plain one-rank lattice; kernel traces of the RCCL and IPC steps.
#   TAG=r06a scripts/halo_ab.sh [alltests] [tests] [ab] [prof] [models2d] [cavity] [catalog] [headline] [cavitycounters] [part]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${TAG:-halo}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
step() { local name=$1 t=$2 log=$3; shift 3; echo "== $name"; timeout -k 10 $t "$@" > $log 2>&1; local rc=$?; tail -3 $log; echo "   rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
for W in "$@"; do case $W in
alltests)
  step "gpu tests" 900 $O/pytest_gpu.log python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread ;;
tests)
  step "ipc + production tests" 600 $O/pytest_ipc.log python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_production.py -v -m gpu --timeout 300 --timeout-method thread ;;
ab)
  for rep in $(seq 1 ${REPS:-2}); do
    step "slab plain" 300 $O/slab_plain_$rep.json python bench.py --shape 512,512,64 --steps 200 --warmup 20
    for t in copy rccl ipc; do
      step "slab $t" 300 $O/slab_${t}_$rep.json python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport $t
      step "slab $t serial borders" 300 $O/slab_${t}_serial_$rep.json env TCLB_CONCURRENT_BORDERS=0 python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport $t
    done
    step "part slab plain" 300 $O/part_plain_$rep.jsonl python tools/bench_configs.py --configs part256 --shape 256,256,64 --steps 200 --warmup 20
    for t in copy rccl ipc; do
      step "part slab $t" 300 $O/part_${t}_$rep.jsonl python tools/bench_configs.py --configs part256 --shape 256,256,64 --steps 200 --warmup 20 --loopback-dist --transport $t
      step "part slab $t serial borders" 300 $O/part_${t}_serial_$rep.jsonl env TCLB_CONCURRENT_BORDERS=0 python tools/bench_configs.py --configs part256 --shape 256,256,64 --steps 200 --warmup 20 --loopback-dist --transport $t
    done
  done ;;
prof)
  for t in rccl ipc; do
    step "rocprof slab $t" 400 $O/prof_slab_$t.log rocprofv3 --kernel-trace --stats -d $O/prof_slab_$t -o run --output-format csv -- python3 $R/bench.py --shape 512,512,64 --steps 20 --warmup 2 --loopback-dist --transport $t
    step "rocprof part slab $t" 400 $O/prof_part_$t.log rocprofv3 --kernel-trace --stats -d $O/prof_part_$t -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs part256 --shape 256,256,64 --steps 20 --warmup 2 --loopback-dist --transport $t
  done ;;
models2d)
  step "2-D multi-stage models fp64" 600 $O/models2d.jsonl python tools/perf_models.py --models d2q9_pf_velocity,d2q9_csf,d2q9_lee --n2 2048 --steps 100 --allow-invalid
  step "rocprof 2-D models" 400 $O/prof_models2d.log rocprofv3 --kernel-trace --stats -d $O/prof_models2d -o run --output-format csv -- python3 $R/tools/perf_models.py --models d2q9_pf_velocity,d2q9_csf --n2 2048 --steps 20 --allow-invalid ;;
cavity)
  step "cavity fp64" 300 $O/cavity_fp64.jsonl python tools/bench_configs.py --configs cavity --steps 100 --warmup 10
  step "cavity ms" 300 $O/cavity_ms.jsonl python tools/bench_configs.py --configs cavity --steps 100 --warmup 10 --precision mixed-shift ;;
catalog)
  step "catalog fp64" 1100 $O/catalog_perf.jsonl python tools/perf_models.py --n3 256 --n2 2048 --steps 100 --allow-invalid ;;
headline)
  step "bench fp64" 300 $O/bench_fp64.json python bench.py ;;
peng)
  step "SIR_ModifiedPeng guard" 300 $O/peng.jsonl python tools/perf_models.py --models d2q9_reaction_diffusion_system_SIR_ModifiedPeng,d2q9_reaction_diffusion_system_SIR_ModifiedPeng_Euler,d2q9_reaction_diffusion_system_SIR_ModifiedPeng_Heun,d2q9_reaction_diffusion_system_SIR_ModifiedPeng_Midpoint,d2q9_reaction_diffusion_system_SIR_ModifiedPeng_Trapezoidal --n2 2048 --steps 100 ;;
cavitycounters)
  step "counters cavity fp64" 500 $O/counters_cavity.log python tools/counters.py --tag cavity_fp64 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs cavity --steps 5 --warmup 1 ;;
calcf)
  for r in 16 2 0.5; do
    step "calcf radius $r" 300 $O/calcf_$r.log rocprofv3 --kernel-trace --stats -d $O/calcf_$r -o run --output-format csv -- python3 $R/tools/calcf_probe.py --radius $r --steps 20
  done ;;
partcounters)
  step "counters part256 fp64" 500 $O/counters_part256.log python tools/counters.py --tag part256_fp64 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs part256 --steps 5 --warmup 1 ;;
part)
  step "part256 fp64" 300 $O/part256_fp64.jsonl python tools/bench_configs.py --configs part256 --steps 100 --warmup 10
  step "rocprof part256" 400 $O/prof_part256.log rocprofv3 --kernel-trace --stats -d $O/prof_part256 -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs part256 --steps 20 --warmup 2 ;;
esac; done
