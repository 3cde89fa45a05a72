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
counterlist) step "rocprofv3 -L" 120 $O/counters_avail.txt rocprofv3 -L ;;
place) step "placement probe torch" 300 $O/place_torch.jsonl python tools/placement_probe.py --k 6
       step "placement probe torch (2)" 300 $O/place_torch2.jsonl python tools/placement_probe.py --k 6 ;;
splitmodels) step "tile split heavy models" 900 $O/split_models.jsonl python tools/perf_models.py --models d3q27_cumulant,d3q19,d3q27_tePSM_per_NEBB,d3q27q27_cm_cht,d3q27_pf_velocity_thermo --n3 256 --steps 20 --rounds 2 --splits 0,2,3 --allow-invalid
       step "tile split pf384" 900 $O/split_pf384.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --splits 0,2,3 --allow-invalid --precision mixed-shift ;;
bench3) for i in 1 2 3; do step "bench fp64 20 #$i" 300 $O/bench20_$i.json python bench.py --steps 20 --warmup 5; done
        step "bench mixed-shift 20" 300 $O/bench20_ms.json python bench.py --steps 20 --warmup 5 --precision mixed-shift ;;
configs) step "bench_configs fp64" 900 $O/configs_fp64.jsonl python tools/bench_configs.py --steps 100 --warmup 5
         step "bench_configs mixed-shift" 900 $O/configs_ms.jsonl python tools/bench_configs.py --steps 100 --warmup 5 --precision mixed-shift ;;
partslab) step "part256 4-GPU slab shape, native loop, RCCL self-send" 300 $O/part_slab_rccl.jsonl python tools/bench_configs.py --configs part256 --shape 256,256,64 --loopback-dist --transport rccl --steps 200 --warmup 10
          step "part256 4-GPU slab shape, Python step path" 300 $O/part_slab_py.jsonl env TCLB_DIST_NATIVE=0 python tools/bench_configs.py --configs part256 --shape 256,256,64 --loopback-dist --transport rccl --steps 200 --warmup 10
          export TMPDIR=/tmp
          step "part256 slab trace" 300 $O/part_slab_prof.log rocprofv3 --kernel-trace --stats -d $O/prof_part_slab -o run --output-format csv -- python3 tools/bench_configs.py --configs part256 --shape 256,256,64 --loopback-dist --transport rccl --steps 50 --warmup 5 ;;
prodtests) step "production + native-loop GPU tests" 900 $O/pytest_prod.log python -u -m pytest tests/test_gpu_production.py tests/test_native_loop.py tests/test_bench_particle_case.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider ;;
adjoint) step "adjoint GPU tests" 600 $O/pytest_adjoint.log python -u -m pytest tests/test_adjoint_native.py tests/test_adjoint_reverse.py tests/test_adjoint.py -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
         for m in d3q19_adj d3q19_heat_adj; do
           step "bench adjoint $m native" 300 $O/adj_${m}_native.json python tools/bench_adjoint.py --model $m --size 128 --steps 80
           step "bench adjoint $m python" 300 $O/adj_${m}_python.json env TCLB_AD_NATIVE=0 python tools/bench_adjoint.py --model $m --size 128 --steps 80
         done
         step "bench adjoint d2q9_adj native" 300 $O/adj_d2q9_adj_native.json python tools/bench_adjoint.py --model d2q9_adj --size 2048 --steps 80
         step "bench adjoint d2q9_adj python" 300 $O/adj_d2q9_adj_python.json env TCLB_AD_NATIVE=0 python tools/bench_adjoint.py --model d2q9_adj --size 2048 --steps 80 ;;
addiag) for v in default row_w2 row_w2_wpe2 row row_wpe2 flat_wpe2; do
          vv=$v; [ $v = default ] && vv=""
          step "adjoint diag $v" 300 $O/addiag_$v.jsonl env TCLB_AD_VARIANT=$vv python tools/adjoint_diag.py --repeats 2
        done ;;
adbisect) step "row-form k_ad bisection" 900 $O/ad_bisect.jsonl python tools/ad_bisect.py check --limits ${LIMITS:-500,1000,2000,3000,4000,5000,6000,7000,8000,9000,10000,11000,12000,12696} ;;
splittests) step "split-stage model GPU tests" 600 $O/pytest_split.log python -u -m pytest tests -v -m gpu -k "pf_velocity or tePSM or split or kept" --timeout 120 --timeout-method thread -p no:cacheprovider ;;
splitperf) step "pf384 split A/B fp64" 600 $O/pf384_split_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ,cw3
           step "pf384 split A/B mixed-shift" 600 $O/pf384_split_ms.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ,cw3 --precision mixed-shift
           step "tePSM split A/B fp64" 600 $O/tepsm_split.jsonl python tools/perf_models.py --models d3q27_tePSM_per_NEBB --n3 256 --steps 20 --rounds 2 --variants ,cw2
           step "bench_configs pf384 fp64" 600 $O/configs_pf384_fp64.jsonl python tools/bench_configs.py --configs pf384 --steps 100 --warmup 5
           step "bench_configs pf384 mixed-shift" 600 $O/configs_pf384_ms.jsonl python tools/bench_configs.py --configs pf384 --steps 100 --warmup 5 --precision mixed-shift ;;
splitab) step "pf384 split vs one kernel, mixed-shift" 600 $O/pf384_nosplit_ms.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 3 --variants ,nosplit --precision mixed-shift
         step "pf384 split vs one kernel, fp64" 600 $O/pf384_nosplit_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ,nosplit
         step "tePSM split vs one kernel" 600 $O/tepsm_nosplit.jsonl python tools/perf_models.py --models d3q27_tePSM_per_NEBB --n3 256 --steps 20 --rounds 3 --variants ,nosplit
         step "pf thermo split vs one kernel" 600 $O/thermo_nosplit.jsonl python tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 20 --rounds 2 --variants ,nosplit ;;
pfconfigs) step "bench_configs pf384 fp64" 600 $O/configs_pf384_fp64.jsonl python tools/bench_configs.py --configs pf384 --steps 100 --warmup 5
           step "bench_configs pf384 mixed-shift" 600 $O/configs_pf384_ms.jsonl python tools/bench_configs.py --configs pf384 --steps 100 --warmup 5 --precision mixed-shift ;;
splitprof) export TMPDIR=/tmp
           step "pf384 ms kernel trace" 300 $O/prof_pf384.log rocprofv3 --kernel-trace --stats -d $O/prof_pf384 -o run --output-format csv -- python3 tools/bench_configs.py --configs pf384 --steps 20 --warmup 3 --precision mixed-shift
           step "tePSM kernel trace" 300 $O/prof_tepsm.log rocprofv3 --kernel-trace --stats -d $O/prof_tepsm -o run --output-format csv -- python3 tools/perf_models.py --models d3q27_tePSM_per_NEBB --n3 256 --steps 20 ;;
heavy) step "heavy models 256^3 fp64" 900 $O/heavy_256.jsonl python tools/perf_models.py --models d3q27_tePSM_per_NEBB,d3q27q27_cm_cht,d3q27_pf_velocity_thermo,d3q19,d3q27_cumulant --n3 256 --steps 20 --rounds 2 ;;
heavycounters) export TMPDIR=/tmp
           step "tePSM counters" 600 $O/ctr_tepsm.log python tools/counters.py --tag tepsm_256 --outdir $O/counters --nodes 16777216 --passes 0,1,2,3 -- python3 tools/perf_models.py --models d3q27_tePSM_per_NEBB --n3 256 --steps 5
           step "thermo counters" 600 $O/ctr_thermo.log python tools/counters.py --tag thermo_256 --outdir $O/counters --nodes 16777216 --passes 0,1,2,3 -- python3 tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 5
           step "pf384 fp64 counters" 600 $O/ctr_pf384.log python tools/counters.py --tag pf384_fp64 --outdir $O/counters --nodes 56623104 --passes 0,1,2,3 -- python3 tools/bench_configs.py --configs pf384 --steps 5 --warmup 1 ;;
tilewaves) step "thermo tile waves A/B" 600 $O/thermo_tw.jsonl python tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 20 --rounds 2 --variants ,tw6,tw8 ;;
cavitycounters) export TMPDIR=/tmp
           step "cavity counters" 600 $O/ctr_cavity.log python tools/counters.py --tag cavity_256 --outdir $O/counters --nodes 16777216 --passes 0,1,2,3 -- python3 tools/bench_configs.py --configs cavity --steps 10 --warmup 2
           step "d3q19 uniform counters" 600 $O/ctr_d3q19.log python tools/counters.py --tag d3q19_256 --outdir $O/counters --nodes 16777216 --passes 0,1,2 -- python3 tools/perf_models.py --models auto_d3q19_BGK --n3 256 --steps 10 ;;
cwab) step "pf384 fp64 class-1 floor A/B" 600 $O/pf384_cw_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ,cw3
      step "pf384 mixed-shift class-1 floor A/B" 600 $O/pf384_cw_ms.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ,cw3,cw4 --precision mixed-shift ;;
catalog) step "catalog perf (all models, guard on)" 1150 $O/catalog_perf.jsonl python tools/perf_models.py --n3 192 --n2 2048 --steps 10 --allow-invalid ;;
psm) step "PSM GPU tests" 600 $O/pytest_psm.log python -u -m pytest tests -v -m gpu -k "PSM or psm or particle" --timeout 120 --timeout-method thread -p no:cacheprovider
     step "PSM perf" 600 $O/psm_perf.jsonl python tools/perf_models.py --models d3q27_PSM_NEBB,d3q27_PSM_SUP,d3q27_PSM_MS_NEBB,d3q27_PSM_KL_NEBB,d3q27_PSM_TRT_NEBB,d3q27_PSM_NEBB_singlekernel --n3 192 --steps 10 --rounds 2 ;;
cumpart) step "cumulant/particle GPU tests" 600 $O/pytest_cumpart.log python -u -m pytest tests -v -m gpu -k "cumulant or particle or part" --timeout 120 --timeout-method thread -p no:cacheprovider
         step "cumulant_part perf" 600 $O/cumpart_perf.jsonl python tools/perf_models.py --models d3q27_cumulant_part,d3q27_cumulant_part_AVG_IB_SMAG,d3q27_cumulant --n3 192 --steps 10 --rounds 2 ;;
*) echo "unknown step $WHAT"; exit 2 ;;
esac
done
