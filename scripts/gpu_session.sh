#!/bin/bash
# developer GPU session: every step writes gpurun_out/$TAG/<step>.log
#   TAG=r02h scripts/gpu_session.sh [tests] [bench] [karman] [prof] [counters] [configs] ...
# each GPU step has its own timeout; a crash / timeout (rc >= 124) ends the call
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=${TAG:-run}; O=$R/gpurun_out/$TAG; mkdir -p $O; cd $R
step() { local name=$1 t=$2 log=$3; shift 3; echo "== $name"; timeout -k 10 $t "$@" > $log 2>&1; local rc=$?; tail -4 $log; echo "   rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
for W in "$@"; do case $W in
newtests) step "new gpu tests" 400 $O/pytest_gpu_new.log python -u -m pytest tests/test_gpu_oracles.py tests/test_gpu_kernels.py -v -m gpu --timeout 120 --timeout-method thread ;;
slabscan)
  # per-node cost against the z extent (one rank, one launch per step): where the 8-GPU
  # slab loses to the full lattice
  for nz in 64 128 256 512; do
    step "plain 512x512x$nz fp64" 300 $O/slabscan_$nz.json python bench.py --shape 512,512,$nz --steps 100 --warmup 10
  done
  for k in 0 1 3 4; do
    step "plain 512x512x64 fp64 tile split $k" 300 $O/slabscan_64_ts$k.json env TCLB_TILE_SPLIT=$k python bench.py --shape 512,512,64 --steps 100 --warmup 10
  done
  step "plain 512x512x64 fp64 no placement probe" 300 $O/slabscan_64_noplace.json env TCLB_PLACE=0 python bench.py --shape 512,512,64 --steps 100 --warmup 10
  step "rocprof slab 64" 400 $O/prof_slab64.log rocprofv3 --kernel-trace --stats -d $O/prof_slab64 -o run --output-format csv -- python3 $R/bench.py --shape 512,512,64 --steps 100 --warmup 10 ;;
tepsm6)
  step "defer + split + tePSM GPU tests" 600 $O/pytest_defer.log python -u -m pytest tests/test_defer_stage.py tests/test_split_stage.py tests/test_tepsm.py -v -m gpu --timeout 120 --timeout-method thread
  step "tePSM 256 fp64 uniform" 600 $O/tepsm_256.jsonl python tools/perf_models.py --models d3q27_tePSM_per_NEBB,d3q27_tePSM_per_SUP --n3 256 --steps 100 --rounds 2
  step "tePSM 256 8 particles" 600 $O/tepsm256_cfg.jsonl python tools/bench_configs.py --configs tepsm256 --steps 100 --warmup 5
  step "rocprof tePSM 8 particles" 400 $O/prof_tepsm256.log rocprofv3 --kernel-trace --stats -d $O/prof_tepsm256 -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs tepsm256 --steps 20 --warmup 2 ;;
calcf)
  # the part256 force stage against the particle's size and count (kernel trace per case)
  for c in "2 1" "8 1" "16 1" "16 4"; do set -- $c
    step "calcf r=$1 n=$2" 300 $O/calcf_r$1_n$2.log rocprofv3 --kernel-trace --stats -d $O/calcf_r$1_n$2 -o run --output-format csv -- python3 $R/tools/calcf_probe.py --radius $1 --nparticles $2 --steps 40
  done ;;
part6)
  step "particle / defer / ipc GPU tests" 600 $O/pytest_part.log python -u -m pytest tests/test_particles.py tests/test_bench_particle_case.py tests/test_gpu_ipc.py tests/test_defer_stage.py tests/test_catalog.py -k "part or defer or ipc or Particle or tePSM" -v -m gpu --timeout 120 --timeout-method thread
  step "part256 fp64" 300 $O/part256_fp64.jsonl python tools/bench_configs.py --configs part256 --steps 100 --warmup 5
  for t in plain rccl copy ipc; do
    if [ $t = plain ]; then
      step "part256 slab plain" 300 $O/part_slab_plain.jsonl python tools/bench_configs.py --configs part256 --shape 256,256,64 --steps 200 --warmup 10
    else
      step "part256 slab $t" 300 $O/part_slab_$t.jsonl python tools/bench_configs.py --configs part256 --shape 256,256,64 --loopback-dist --transport $t --steps 200 --warmup 10
    fi
  done ;;
slabts)
  for r in 1 2; do for nz in 64 128 256; do for k in 0 2; do
    step "plain 512x512x$nz ts$k #$r" 300 $O/slabts_${nz}_ts${k}_$r.json env TCLB_TILE_SPLIT=$k python bench.py --shape 512,512,$nz --steps 100 --warmup 10
  done; done; done ;;
rcclenv)
  # RCCL self-send on the 8-GPU headline slab against its channel count (the RCCL kernel's
  # work-groups compete with the interior launch for CUs)
  step "slab plain" 300 $O/rcclenv_plain.json python bench.py --shape 512,512,64 --steps 200 --warmup 20
  step "slab rccl default" 300 $O/rcclenv_default.json python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport rccl
  for c in 1 2 4 8; do
    step "slab rccl NCCL_MAX_NCHANNELS=$c" 300 $O/rcclenv_max$c.json env NCCL_MAX_NCHANNELS=$c NCCL_MIN_NCHANNELS=1 python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport rccl
  done
  step "slab rccl NCCL_NCHANNELS_PER_PEER=1" 300 $O/rcclenv_pp1.json env NCCL_NCHANNELS_PER_PEER=1 python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport rccl
  step "slab ipc" 300 $O/rcclenv_ipc.json python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport ipc
  step "slab copy" 300 $O/rcclenv_copy.json python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --transport copy ;;
c2probe)
  # the r05m class-2 fault against one backend stage at a time (build.py c2w0_* variants)
  for v in ${C2VARIANTS:-c2w0 c2w0_noagpr c2w0_nomisched c2w0_nopostra c2w0_nohrp c2w0_o1 c2w0_verify}; do
    step "split probe $v" 300 $O/c2probe_$v.log env MODE=noglob STEPS=1 VARIANT=$v python tools/split_probe.py d3q27_tePSM_per_NEBB
  done ;;
c2old)
  # the same probe on a checkout of the source in which the fault was found (git worktree
  # _wt_c2 of 2088283, before the deferring stages changed the class-2 kernel)
  for v in ${C2VARIANTS:-c2w0 c2w0_noagpr c2w0_nomisched c2w0_nopostra c2w0_nohrp c2w0_o1}; do
    step "old-source split probe $v" 300 $O/c2old_$v.log bash -c "cd $R/_wt_c2 && MODE=noglob STEPS=1 VARIANT=$v python tools/split_probe.py d3q27_tePSM_per_NEBB"
  done ;;
adsched)
  # the row-form k_ad fault (r05i-j) under the two scheduler switches that clear the class-2 one
  for v in row_w2 row_w2_nohrp row_w2_nomisched ""; do
    step "adjoint diag variant '$v'" 300 $O/adsched_${v:-default}.log env TCLB_AD_VARIANT=$v TCLB_NO_BUILD=1 python tools/adjoint_diag.py --repeats 1 --modes dual
  done ;;
final6)
  # round-6 closing evidence: every BASELINE config on the final tree, hardware counters
  # of the headline fp64 kernel, part256 and the tePSM collide
  step "configs" 500 $O/configs.log python tools/bench_configs.py
  step "counters d3q27 fp64" 500 $O/counters_d3q27_fp64.log python tools/counters.py --tag d3q27_512_fp64 --nodes 134217728 --outdir $O/counters -- python3 $R/bench.py --steps 5 --warmup 1
  step "counters part256" 500 $O/counters_part256.log python tools/counters.py --tag part256_fp64 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs part256 --steps 5 --warmup 1
  step "counters tePSM 256" 500 $O/counters_tepsm.log python tools/counters.py --tag tepsm_256_fp64 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/perf_models.py --models d3q27_tePSM_per_NEBB --n3 256 --steps 5 ;;
r06r)
  step "placement probe + IPC GPU tests" 400 $O/pytest_place_ipc.log python -u -m pytest tests/test_gpu_placement.py tests/test_gpu_ipc.py -v -m gpu --timeout 120 --timeout-method thread
  step "bench half-shift" 300 $O/bench_half_shift.json python bench.py --precision half-shift
  step "bench half" 300 $O/bench_half.json python bench.py --precision half ;;
tests) step "gpu tests" 900 $O/pytest_gpu.log python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread ;;
bench)
  step "bench fp64" 300 $O/bench_fp64.json python bench.py
  step "bench mixed-shift" 300 $O/bench_mixed_shift.json python bench.py --precision mixed-shift
  step "bench mixed" 300 $O/bench_mixed.json python bench.py --precision mixed
  step "bench half-shift" 300 $O/bench_half_shift.json python bench.py --precision half-shift ;;
karman) step "karman compute-only" 300 $O/karman_novtk.log python tools/bench_karman.py --iters 20000 --vtk 0 ;;
prof) step "rocprof mixed-shift" 400 $O/prof_mixed_shift.log rocprofv3 --kernel-trace --stats -d $O/prof_mixed_shift -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --precision mixed-shift ;;
counters)
  step "counters d3q27 mixed-shift" 500 $O/counters_d3q27_ms.log python tools/counters.py --tag d3q27_512_mixed_shift --nodes 134217728 --outdir $O/counters -- python3 $R/bench.py --steps 5 --warmup 1 --precision mixed-shift
  step "counters pf384" 500 $O/counters_pf384.log python tools/counters.py --tag pf384_fp64 --nodes 56623104 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs pf384 --steps 5 --warmup 1 ;;
pfcounters) step "counters pf384 mixed-shift" 500 $O/counters_pf384_ms.log python tools/counters.py --tag pf384_mixed_shift --nodes 56623104 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs pf384 --steps 5 --warmup 1 --precision mixed-shift ;;
modelcounters)
  step "counters stencil models" 600 $O/counters_models.log python tools/counters.py --tag models_16M --nodes 16777216 --outdir $O/counters -- python3 $R/tools/perf_models.py --models d3q27_PSM_NEBB,d2q9_ShanChen,d2q9_kuper --steps 5
  step "counters part256" 500 $O/counters_part256.log python tools/counters.py --tag part256_fp64 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs part256 --steps 5 --warmup 1 ;;
slabhost)
  # host cost of a native multi-rank step (launches, events, RCCL group calls) against its
  # GPU time, on the 8-GPU per-rank slab
  for P in mixed-shift double; do
    step "slab $P native rccl self" 300 $O/slab_${P}_rccl.json python bench.py --shape 512,512,64 --precision $P --steps 200 --warmup 20 --loopback-dist --transport rccl
  done ;;
headab2)
  VARIANTS="default xcd nt mclause" bash scripts/headline_variants.sh 2 double mixed-shift
  mkdir -p $O && cp $R/gpurun_out/ab/variants.log $O/headline_variants.log ;;
xcdab)
  VARIANTS="default xcd" bash scripts/headline_variants.sh 3 double mixed-shift
  mkdir -p $O && cp $R/gpurun_out/ab/variants.log $O/headline_variants.log
  step "models fp64 default vs xcd" 900 $O/xcd_models_fp64.jsonl python tools/perf_models.py --models d3q27_cumulant,d3q19,d3q27_tePSM_per_NEBB,d3q27q27_cm_cht,d3q27_pf_velocity_thermo --n3 256 --steps 20 --rounds 2 --variants ",xcd" --allow-invalid
  step "pf384 fp64 / ms default vs xcd" 900 $O/xcd_pf384.jsonl bash -c 'python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ",xcd" --allow-invalid && python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --precision mixed-shift --variants ",xcd" --allow-invalid' ;;
xcdsize)
  for r in 1 2; do for n in 384 448 512; do for v in "" xcd; do
    step "d3q27 fp64 $n ${v:-default}" 300 $O/xcd_size_${n}_${v:-default}_$r.json env TCLB_VARIANT=$v TCLB_NO_BUILD=1 python bench.py --size $n --steps 50 --warmup 5
  done; done; done
  step "d3q19 fp64 512 default vs xcd" 600 $O/xcd_d3q19_512.jsonl python tools/perf_models.py --models d3q19,d3q27_cumulant --n3 512 --steps 20 --rounds 2 --variants ",xcd" --allow-invalid ;;
padab)
  # row pitch / field padding of the 512^3 headline (runtime layout knobs, no rebuild)
  for r in 1 2; do for P in double mixed-shift; do
    for cfg in "0 0" "64 0" "128 0" "0 4096" "64 4096"; do set -- $cfg
      step "pad x=$1 f=$2 $P" 300 $O/pad_${P}_x$1_f$2_$r.json env TCLB_X_PAD=$1 TCLB_FIELD_PAD=$2 python bench.py --steps 50 --warmup 5 --precision $P
    done
  done; done ;;
padab2)
  for r in 1 2 3; do
    for x in 0 128 192 256; do
      step "pad x=$x fp64" 300 $O/pad2_double_x${x}_$r.json env TCLB_X_PAD=$x python bench.py --steps 50 --warmup 5
    done
    for x in 0 128; do
      step "pad x=$x ms" 300 $O/pad2_ms_x${x}_$r.json env TCLB_X_PAD=$x python bench.py --steps 50 --warmup 5 --precision mixed-shift
    done
  done ;;
pfdroplet)
  step "rocprof pf384 droplet ms" 400 $O/prof_pf384_droplet_ms.log rocprofv3 --kernel-trace --stats -d $O/prof_pf384_droplet_ms -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs pf384 --steps 10 --warmup 2 --precision mixed-shift
  step "rocprof pf384 uniform ms" 400 $O/prof_pf384_uniform_ms.log rocprofv3 --kernel-trace --stats -d $O/prof_pf384_uniform_ms -o run --output-format csv -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 10 --precision mixed-shift ;;
pfcount2)
  step "counters pf384 droplet ms" 500 $O/counters_droplet.log python tools/counters.py --tag pf384_droplet_ms --nodes 56623104 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs pf384 --steps 5 --warmup 1 --precision mixed-shift
  step "counters pf384 uniform ms" 500 $O/counters_uniform.log python tools/counters.py --tag pf384_uniform_ms --nodes 56623104 --outdir $O/counters -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 5 --precision mixed-shift ;;
pfmrt)
  # pf_velocity(_thermo) with the MRT collision their default build runs (perf_models fix)
  step "pf384 MRT ms/fp64 default vs rowplain" 900 $O/pf384_mrt.jsonl bash -c 'python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --precision mixed-shift --variants ",rowplain" --allow-invalid && python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ",rowplain" --allow-invalid'
  step "thermo 256 MRT default vs rowplain" 600 $O/thermo_mrt.jsonl python tools/perf_models.py --models d3q27_pf_velocity_thermo,d2q9_kuper --n3 256 --n2 4096 --steps 20 --rounds 2 --variants ",rowplain" --allow-invalid
  step "rocprof thermo 256 MRT" 400 $O/prof_thermo_mrt.log rocprofv3 --kernel-trace --stats -d $O/prof_thermo_mrt -o run --output-format csv -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 10 ;;
thermofinal)
  step "thermo 256 MRT" 600 $O/thermo_mrt_final.jsonl python tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 20 --rounds 2 --allow-invalid ;;
final)
  step "bench fp64" 300 $O/bench_fp64.json python bench.py
  step "bench fp64 100 steps" 300 $O/bench_fp64_100.json python bench.py --steps 100 --warmup 10
  step "bench mixed-shift 100 steps" 300 $O/bench_ms_100.json python bench.py --steps 100 --warmup 10 --precision mixed-shift
  step "rocprof fp64 headline" 400 $O/prof_fp64.log rocprofv3 --kernel-trace --stats -d $O/prof_fp64 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 2 ;;
thermo)
  step "pf thermo 256 fp64" 600 $O/thermo_256_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity_thermo,d2q9_ShanChen --n3 256 --n2 4096 --steps 20 --rounds 2 --allow-invalid
  step "rocprof pf thermo 256" 400 $O/prof_thermo.log rocprofv3 --kernel-trace --stats -d $O/prof_thermo -o run --output-format csv -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 10 ;;
thermocounters)
  step "counters pf_velocity_thermo 256" 700 $O/counters_thermo.log python tools/counters.py --tag thermo256_fp64 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 5
  step "rocprof pf thermo 256" 400 $O/prof_thermo.log rocprofv3 --kernel-trace --stats -d $O/prof_thermo -o run --output-format csv -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 10 ;;
ldsab)
  step "lds a/b 384" 300 $O/lds_ab_384.log python tools/lds_ab.py --n 384 --reps 20
  step "lds a/b 512" 300 $O/lds_ab_512.log python tools/lds_ab.py --n 512 --reps 10
  step "counters lds a/b" 400 $O/counters_lds.log python tools/counters.py --tag lds_ab_384 --nodes 56623104 --outdir $O/counters -- python3 $R/tools/lds_ab.py --n 384 --reps 3 --rounds 1 ;;
nwab) step "narrow-storage occupancy A/B" 900 $O/nw_ab.log python tools/perf_models.py --models d3q27_pf_velocity,d3q27 --n3 384 --steps 10 --precision mixed-shift --variants ",nw3,nw4" --rounds 2 ;;
adjoint)
  step "gpu adjoint tests" 600 $O/pytest_gpu_adjoint.log python -u -m pytest tests/test_gpu_adjoint.py -v -m gpu --timeout 300 --timeout-method thread
  step "adjoint bench 64" 300 $O/bench_adjoint_64.json python tools/bench_adjoint.py --size 64 --steps 40
  step "adjoint bench 128" 400 $O/bench_adjoint_128.json python tools/bench_adjoint.py --size 128 --steps 80 ;;
adbench)
  for M in d3q19_adj d3q19_heat_adj d3q19_heat_adj_art; do
    step "adjoint bench $M 128" 300 $O/adbench_${M}_128.json python tools/bench_adjoint.py --model $M --size 128 --steps 20
  done
  step "adjoint bench d3q19_heat_adj 128 dual" 300 $O/adbench_d3q19_heat_adj_128_dual.json python tools/bench_adjoint.py --model d3q19_heat_adj --size 128 --steps 20 --dual
  for M in d2q9_adj d2q9_heat_adj; do
    step "adjoint bench $M 2048^2" 300 $O/adbench_${M}_2048.json python tools/bench_adjoint.py --model $M --size 2048 --steps 20
  done
  step "adjoint bench d2q9_adj 2048^2 dual" 300 $O/adbench_d2q9_adj_2048_dual.json python tools/bench_adjoint.py --model d2q9_adj --size 2048 --steps 20 --dual ;;
adbench80)
  for M in d3q19_adj d3q19_heat_adj d3q19_heat_adj_art d3q19_heat_adj_prop; do
    step "adjoint bench $M 128 x80" 400 $O/adbench80_${M}_128.json python tools/bench_adjoint.py --model $M --size 128 --steps 80
  done
  for M in d2q9_adj d2q9_heat_adj; do
    step "adjoint bench $M 2048^2 x80" 400 $O/adbench80_${M}_2048.json python tools/bench_adjoint.py --model $M --size 2048 --steps 80
  done
  step "rocprof adjoint d3q19_heat_adj" 400 $O/prof_adj_heat.log rocprofv3 --kernel-trace --stats -d $O/prof_adj_heat -o run --output-format csv -- python3 $R/tools/bench_adjoint.py --model d3q19_heat_adj --size 128 --steps 40 ;;
adbench2d)
  for M in d2q9_kuper_adj d2q9_optimalMixing d2q9_plate; do
    step "adjoint bench $M 2048^2 x40" 400 $O/adbench_${M}_2048.json python tools/bench_adjoint.py --model $M --size 2048 --steps 40
  done ;;
tepsm)
  step "tePSM 256 fp64 default vs sw2" 600 $O/tepsm_256_ab.jsonl python tools/perf_models.py --models d3q27_tePSM_per_NEBB --n3 256 --steps 20 --rounds 2 --variants ,sw2 --allow-invalid
  step "rocprof tePSM 256" 400 $O/prof_tepsm.log rocprofv3 --kernel-trace --stats -d $O/prof_tepsm -o run --output-format csv -- python3 $R/tools/perf_models.py --models d3q27_tePSM_per_NEBB --n3 256 --steps 10 ;;
pfsw3)
  step "pf 384 mixed-shift default vs sw3" 600 $O/pf384_ms_sw3.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --precision mixed-shift --variants ",sw3" --rounds 2 --allow-invalid
  step "pf 384 fp64 default vs sw3" 600 $O/pf384_fp64_sw3.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --variants ",sw3" --rounds 2 --allow-invalid ;;
rowab)
  # plain kernels: flat offsets (default) vs the round-3 row form (rowplain) on the heavy models
  step "pf384 ms flat vs rowplain" 600 $O/rowab_pf384_ms.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --precision mixed-shift --rounds 2 --variants ",rowplain" --allow-invalid
  step "pf384 fp64 flat vs rowplain" 600 $O/rowab_pf384_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --variants ",rowplain" --allow-invalid
  step "heavy 256 flat vs rowplain" 900 $O/rowab_heavy_256.jsonl python tools/perf_models.py --models d3q27_tePSM_per_NEBB,d3q27_pf_velocity_thermo,d3q27q27_cm_cht,d3q19,d3q27_cumulant --n3 256 --steps 20 --rounds 2 --variants ",rowplain" --allow-invalid ;;
kuperlds)
  step "kuper / ShanChen LDS tiles vs nolds" 600 $O/kuper_lds_ab.jsonl python tools/perf_models.py --models d3q19_kuper,d2q9_kuper,d2q9_ShanChen --n3 256 --n2 4096 --steps 20 --rounds 2 --variants ",nolds" --allow-invalid ;;
headab)
  VARIANTS="r02 default rowplain r02like" bash scripts/headline_variants.sh 2 double mixed-shift
  mkdir -p $O && cp $R/gpurun_out/ab/variants.log $O/headline_variants.log ;;
tiles2)
  step "pf 384 fp64" 600 $O/tiles2_pf384_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --rounds 2 --allow-invalid
  step "pf 384 mixed-shift" 600 $O/tiles2_pf384_ms.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --precision mixed-shift --rounds 2 --allow-invalid
  step "rocprof pf384 ms" 400 $O/prof_pf384_ms.log rocprofv3 --kernel-trace --stats -d $O/prof_pf384_ms -o run --output-format csv -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 10 --precision mixed-shift ;;
configs4)
  step "configs fp64 100 steps" 600 $O/configs_fp64_100.jsonl python tools/bench_configs.py --steps 100 --warmup 10
  step "configs mixed-shift 100 steps" 600 $O/configs_ms_100.jsonl python tools/bench_configs.py --steps 100 --warmup 10 --precision mixed-shift
  step "part256 1000 steps" 600 $O/part256_1000.jsonl python tools/bench_configs.py --configs part256 --steps 1000 --warmup 10
  step "rocprof part256" 400 $O/prof_part256.log rocprofv3 --kernel-trace --stats -d $O/prof_part256 -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs part256 --steps 50 --warmup 5 ;;
addiag)
  for V in "" row row_o1 row_w1; do
    step "adjoint diag ${V:-flat}" 300 $O/adjoint_diag_${V:-flat}.jsonl env TCLB_AD_VARIANT=$V TCLB_NO_BUILD=1 python tools/adjoint_diag.py --repeats 2
  done ;;
addiag2)
  for V in "" row row_w2 row_w3; do
    step "adjoint diag ${V:-flat}" 300 $O/adjoint_diag_${V:-flat}.jsonl env TCLB_AD_VARIANT=$V TCLB_NO_BUILD=1 python tools/adjoint_diag.py --repeats 2
  done ;;
adhost)
  # host cost of an adjoint step: a lattice too small for the GPU time to matter
  for M in d3q19_adj d3q19_heat_adj; do
    step "adjoint host cost $M 16^3" 300 $O/adhost_${M}_16.json python tools/bench_adjoint.py --model $M --size 16 --steps 40
  done ;;
tiles)
  step "pf thermo 256 fp64 tiles vs nolds" 600 $O/tiles_thermo_256_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 20 --variants ",nolds" --rounds 2 --allow-invalid
  step "pf 384 fp64 tiles vs nolds" 600 $O/tiles_pf384_fp64.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --variants ",nolds" --rounds 2 --allow-invalid
  step "pf 384 mixed-shift tiles vs nolds" 600 $O/tiles_pf384_ms.jsonl python tools/perf_models.py --models d3q27_pf_velocity --n3 384 --steps 20 --precision mixed-shift --variants ",nolds" --rounds 2 --allow-invalid
  step "rocprof pf thermo 256" 400 $O/prof_thermo.log rocprofv3 --kernel-trace --stats -d $O/prof_thermo -o run --output-format csv -- python3 $R/tools/perf_models.py --models d3q27_pf_velocity_thermo --n3 256 --steps 10 ;;
gputests) step "gpu tests" 1100 $O/pytest_gpu.log python -u -m pytest tests -q -m gpu --maxfail=30 --timeout 120 --timeout-method thread -p no:cacheprovider ;;
distnative)
  step "gpu dist-path tests" 900 $O/pytest_gpu_dist.log python -u -m pytest tests/test_catalog.py -k dist_path_on_gpu -m gpu -x -q --timeout 120 --timeout-method thread
  for P in mixed-shift double; do
  step "slab $P plain" 300 $O/slab_${P}_plain.json python bench.py --shape 512,512,64 --precision $P --steps 200 --warmup 20
  step "slab $P native rccl self" 300 $O/slab_${P}_rccl.json python bench.py --shape 512,512,64 --precision $P --steps 200 --warmup 20 --loopback-dist --transport rccl
  step "slab $P native copy" 300 $O/slab_${P}_copy.json python bench.py --shape 512,512,64 --precision $P --steps 200 --warmup 20 --loopback-dist --transport copy
  step "slab $P python loop" 300 $O/slab_${P}_python.json python bench.py --shape 512,512,64 --precision $P --steps 200 --warmup 20 --loopback-dist --python-loop
  done
  step "rocprof slab rccl self" 400 $O/prof_slab_rccl.log rocprofv3 --kernel-trace --stats -d $O/prof_slab_rccl -o run --output-format csv -- python3 $R/bench.py --shape 512,512,64 --precision mixed-shift --steps 50 --warmup 5 --loopback-dist --transport rccl ;;
dist)
  step "slab 512x512x64 plain" 300 $O/dist_plain.json python bench.py --shape 512,512,64 --steps 200 --warmup 20
  step "slab loopback overlap" 300 $O/dist_loop_overlap.json python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist
  step "slab loopback no-overlap" 300 $O/dist_loop_nooverlap.json python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist --no-overlap
  step "slab loopback overlap, pack kernels" 300 $O/dist_loop_overlap_pack.json env TCLB_HALO_MIRROR=0 python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist
  step "rocprof loopback overlap" 400 $O/prof_loop.log rocprofv3 --kernel-trace --stats -d $O/prof_loop -o run --output-format csv -- python3 $R/bench.py --shape 512,512,64 --steps 20 --warmup 5 --loopback-dist ;;
pfms) step "pf384 storage modes" 600 $O/configs_pf_modes.log bash -c 'for p in double mixed-shift; do python tools/bench_configs.py --configs pf384,cavity --precision $p; done' ;;
configs) step "configs" 400 $O/configs.log python tools/bench_configs.py ;;
probe)
  step "stream probe" 300 $O/stream_probe.log python tools/stream_probe.py
  step "bench fp64 a" 300 $O/bench_fp64_a.json python bench.py
  step "bench fp64 pad 2112" 300 $O/bench_fp64_pad2112.json env TCLB_FIELD_PAD=2112 python bench.py
  step "bench fp64 b" 300 $O/bench_fp64_b.json python bench.py ;;
adwin)
  for v in "" w1 w2 w4; do
    step "adjoint bench 128 window ${v:-w3}" 300 $O/bench_adjoint_128_${v:-w3}.json env TCLB_AD_VARIANT=$v python tools/bench_adjoint.py --size 128 --steps 80
  done ;;
refcases)
  step "ThermocapillaryFlow x20, 200 its" 900 $O/examples_thermocapillary_gpu.jsonl python tools/run_examples.py --device cuda --iters 200 --out /tmp/tclb_ex $R/_refcases/ThermocapillaryFlow/*.xml ;&
annular)
  step "annular Taylor bubble 3000 its, output as written" 600 $O/annular_output.jsonl python tools/run_examples.py --device cuda --iters 3000 --out /tmp/tclb_ex $R/_refcases/d3q27_pf_velocity/annularTaylorBubble_DasC.xml
  step "annular Taylor bubble 3000 its, no output" 600 $O/annular_nooutput.jsonl python tools/run_examples.py --device cuda --iters 3000 --no-output --out /tmp/tclb_ex2 $R/_refcases/d3q27_pf_velocity/annularTaylorBubble_DasC.xml ;;
globab)
  step "bench fp64" 300 $O/bench_fp64.json python bench.py --steps 50
  step "bench fp64 globals every step" 300 $O/bench_fp64_globevery.json python bench.py --steps 50 --glob-every-step
  step "bench mixed-shift" 300 $O/bench_ms.json python bench.py --steps 50 --precision mixed-shift
  step "bench mixed-shift globals every step" 300 $O/bench_ms_globevery.json python bench.py --steps 50 --precision mixed-shift --glob-every-step
  step "rocprof globals every step" 400 $O/prof_globevery.log rocprofv3 --kernel-trace --stats -d $O/prof_globevery -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --glob-every-step ;;
heavy)
  step "perf heavy models 256^3 fp64" 600 $O/perf_heavy.log python tools/perf_models.py --models d3q27_tePSM_per_NEBB,d3q27q27_cm_cht,d3q27_pf_velocity_thermo,d3q27_pf_velocity_OutFlow,d3q27_pf_velocity --n3 256 --steps 10
  step "counters heavy models" 600 $O/counters_heavy.log python tools/counters.py --tag r03_heavy_256 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/perf_models.py --models d3q27_tePSM_per_NEBB,d3q27q27_cm_cht,d3q27_pf_velocity_thermo --n3 256 --steps 3
  step "counters cavity 256" 400 $O/counters_cavity.log python tools/counters.py --tag r03_cavity_256 --nodes 16777216 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs cavity --steps 5 --warmup 1 ;;
r03m)
  step "configs fp64 (cavity, pf384, part256)" 600 $O/configs_fp64.log python tools/bench_configs.py
  step "configs mixed-shift pf384" 400 $O/configs_pf384_ms.log python tools/bench_configs.py --configs pf384 --precision mixed-shift
  step "YZ grid loopback 512x256x128" 300 $O/yz_loop.json env TCLB_GRID=1,1 python bench.py --shape 512,256,128 --steps 50 --warmup 5 --loopback-dist
  step "plain 512x256x128" 300 $O/yz_plain.json python bench.py --shape 512,256,128 --steps 50 --warmup 5
  step "host overhead: 128^3 plain" 300 $O/ov_plain.json python bench.py --shape 128,128,128 --steps 300 --warmup 20
  step "host overhead: 128^3 dist path" 300 $O/ov_dist.json python bench.py --shape 128,128,128 --steps 300 --warmup 20 --loopback-dist
  step "slab 512x512x64 plain" 300 $O/slab_plain.json python bench.py --shape 512,512,64 --steps 200 --warmup 20
  step "slab 512x512x64 dist path" 300 $O/slab_dist.json python bench.py --shape 512,512,64 --steps 200 --warmup 20 --loopback-dist
  step "rocprof YZ grid loopback" 400 $O/prof_yz.log env TCLB_GRID=1,1 rocprofv3 --kernel-trace --stats -d $O/prof_yz -o run --output-format csv -- python3 $R/bench.py --shape 512,256,128 --steps 10 --warmup 2 --loopback-dist ;;
adjrev)
  step "gpu adjoint tests" 600 $O/pytest_gpu_adjoint.log python -u -m pytest tests/test_gpu_adjoint.py tests/test_adjoint_reverse.py tests/test_adjoint_dist.py -v -m gpu --timeout 300 --timeout-method thread
  step "adjoint bench 128" 400 $O/bench_adjoint_128.json python tools/bench_adjoint.py --size 128 --steps 80
  step "rocprof adjoint 128" 400 $O/prof_adjoint.log rocprofv3 --kernel-trace --stats -d $O/prof_adjoint -o run --output-format csv -- python3 $R/tools/bench_adjoint.py --size 128 --steps 20 ;;
examples_a) step "reference examples (part a) on the GPU, 100 its" 1100 $O/examples_gpu_a.jsonl python tools/run_examples.py --infer --device cuda --iters 100 --timeout 120 --cwd $R/_refcases --out /tmp/tclb_exa $(cat $R/_refcases/cases_a.txt) ;;
examples_b) step "reference examples (part b) on the GPU, 100 its" 1100 $O/examples_gpu_b.jsonl python tools/run_examples.py --infer --device cuda --iters 100 --timeout 120 --cwd $R/_refcases --out /tmp/tclb_exb $(cat $R/_refcases/cases_b.txt) ;;
globms) step "rocprof mixed-shift globals every step" 400 $O/prof_ms_globevery.log rocprofv3 --kernel-trace --stats -d $O/prof_ms_globevery -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --glob-every-step --precision mixed-shift ;;
smoke) step "smoke" 300 $O/smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
bench1) step "bench fp64" 300 $O/bench_fp64.json python bench.py ;;
r03k)
  for r in a b; do
    step "pf384 mixed-shift globals every step ($r)" 300 $O/pf384_ms_glob_$r.log python tools/bench_configs.py --configs pf384 --precision mixed-shift --glob-every-step
    step "pf384 mixed-shift globals every step, gw2 ($r)" 300 $O/pf384_ms_glob_gw2_$r.log env TCLB_VARIANT=gw2 python tools/bench_configs.py --configs pf384 --precision mixed-shift --glob-every-step
  done
  step "pf384 fp64 globals every step, gw2" 300 $O/pf384_fp64_glob_gw2.log env TCLB_VARIANT=gw2 python tools/bench_configs.py --configs pf384 --glob-every-step
  step "pf384 fp64 / mixed-shift plain" 300 $O/pf384_plain.log bash -c 'python tools/bench_configs.py --configs pf384 && python tools/bench_configs.py --configs pf384 --precision mixed-shift'
  step "d3q27 mixed-shift globals every step, gw2" 300 $O/bench_ms_glob_gw2.json env TCLB_VARIANT=gw2 python bench.py --steps 50 --precision mixed-shift --glob-every-step
  step "rocprof part256 grid" 300 $O/prof_part256.log rocprofv3 --kernel-trace --stats -d $O/prof_part256 -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs part256 --steps 20 --warmup 3
  step "rocprof part256 tree" 300 $O/prof_part256_tree.log env TCLB_SOLID_CONTAINER=tree rocprofv3 --kernel-trace --stats -d $O/prof_part256_tree -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs part256 --steps 20 --warmup 3
  step "adjoint tests" 600 $O/pytest_gpu_adjoint.log python -u -m pytest tests/test_gpu_adjoint.py tests/test_adjoint_reverse.py tests/test_adjoint_dist.py -v -m gpu --timeout 300 --timeout-method thread
  step "adjoint bench 128" 400 $O/bench_adjoint_128.json python tools/bench_adjoint.py --size 128 --steps 80 ;;
r03l)
  step "configs fp64 (cavity, pf384, part256)" 600 $O/configs_fp64.log python tools/bench_configs.py
  step "part256 tree container" 300 $O/part256_tree.log env TCLB_SOLID_CONTAINER=tree python tools/bench_configs.py --configs part256
  step "pf384 globals every step (fp64, mixed-shift)" 400 $O/pf384_glob.log bash -c 'python tools/bench_configs.py --configs pf384 --glob-every-step && python tools/bench_configs.py --configs pf384 --precision mixed-shift --glob-every-step && python tools/bench_configs.py --configs pf384 --precision mixed-shift'
  step "heavy models globals every step, default vs gw2 cap" 600 $O/heavy_glob_ab.log python tools/perf_models.py --models d3q27_pf_velocity_thermo,d3q27_pf_velocity_OutFlow,d3q27_tePSM_per_NEBB --n3 192 --steps 6 --glob-every-step --variants ",gw2"
  step "heavy models plain steps" 400 $O/heavy_plain.log python tools/perf_models.py --models d3q27_pf_velocity_thermo,d3q27_pf_velocity_OutFlow,d3q27_tePSM_per_NEBB --n3 192 --steps 6
  step "adjoint bench 128" 400 $O/bench_adjoint_128.json python tools/bench_adjoint.py --size 128 --steps 80
  step "bench fp64" 300 $O/bench_fp64.json python bench.py ;;
r03n)
  step "configs fp64 (cavity, pf384, part256)" 600 $O/configs_fp64.log python tools/bench_configs.py
  step "configs mixed-shift (pf384)" 300 $O/configs_ms.log python tools/bench_configs.py --configs pf384 --precision mixed-shift
  step "part256 host time per step (32^3)" 300 $O/part32_host.log python tools/bench_configs.py --configs part256 --size 32 --steps 300 --warmup 20
  step "rocprof part256 trace" 300 $O/prof_part256.log rocprofv3 --kernel-trace --stats -d $O/prof_part256 -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs part256 --steps 20 --warmup 3
  step "counters pf384 mixed-shift (waves, instruction mix)" 500 $O/counters_pf384_ms.log python tools/counters.py --tag pf384_ms_mix --passes 2,3 --nodes 56623104 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs pf384 --steps 3 --warmup 1 --precision mixed-shift
  step "counters pf384 fp64 (waves, instruction mix)" 500 $O/counters_pf384.log python tools/counters.py --tag pf384_fp64_mix --passes 2,3 --nodes 56623104 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs pf384 --steps 3 --warmup 1 ;;
r03o)
  for v in "" gregs flataddr; do
    step "d3q27 fp64/ms +- globals every step, variant '$v'" 400 $O/bench_glob_${v:-default}.log bash -c "TCLB_VARIANT=$v python bench.py --steps 50 && TCLB_VARIANT=$v python bench.py --steps 50 --glob-every-step && TCLB_VARIANT=$v python bench.py --steps 50 --precision mixed-shift && TCLB_VARIANT=$v python bench.py --steps 50 --precision mixed-shift --glob-every-step"
    step "pf384 fp64/ms +- globals every step, variant '$v'" 500 $O/pf384_${v:-default}.log bash -c "export TCLB_VARIANT=$v; python tools/bench_configs.py --configs pf384,cavity,part256 && python tools/bench_configs.py --configs pf384 --glob-every-step && python tools/bench_configs.py --configs pf384,cavity --precision mixed-shift && python tools/bench_configs.py --configs pf384 --precision mixed-shift --glob-every-step"
  done ;;
pfvar)
  for r in a b; do for v in "" nt ntld xcd; do
    step "pf384 mixed-shift variant '$v' ($r)" 300 $O/pf384_ms_${v:-default}_$r.log env TCLB_VARIANT=$v python tools/bench_configs.py --configs pf384 --precision mixed-shift
  done; done ;;
r03s)
  step "pf384 fp64 / mixed-shift, plain and globals every step" 500 $O/pf384_glob.log bash -c 'python tools/bench_configs.py --configs pf384 && python tools/bench_configs.py --configs pf384 --glob-every-step && python tools/bench_configs.py --configs pf384 --precision mixed-shift && python tools/bench_configs.py --configs pf384 --precision mixed-shift --glob-every-step'
  step "uncapped globals kernels: cm_cht / pf_velocity_BGK, plain and globals every step" 500 $O/heavy_glob.log bash -c 'python tools/perf_models.py --models d3q27q27_cm_cht,d3q27q7_cm_cht,d3q27_pf_velocity_BGK --n3 192 --steps 6 && python tools/perf_models.py --models d3q27q27_cm_cht,d3q27q7_cm_cht,d3q27_pf_velocity_BGK --n3 192 --steps 6 --glob-every-step' ;;
pfprof)
  step "rocprof pf384 mixed-shift" 400 $O/prof_pf384_ms.log rocprofv3 --kernel-trace --stats -d $O/prof_pf384_ms -o run --output-format csv -- python3 $R/tools/bench_configs.py --configs pf384 --precision mixed-shift --steps 5 --warmup 1
  step "counters pf384 mixed-shift" 500 $O/counters_pf384_ms.log python tools/counters.py --tag pf384_mixed_shift --nodes 56623104 --outdir $O/counters -- python3 $R/tools/bench_configs.py --configs pf384 --steps 5 --warmup 1 --precision mixed-shift ;;
r03i)
  step "part256 grid container" 300 $O/part256_grid.log python tools/bench_configs.py --configs part256
  step "part256 tree container" 300 $O/part256_tree.log env TCLB_SOLID_CONTAINER=tree python tools/bench_configs.py --configs part256
  step "pf384 mixed-shift, scalar zonal reads" 300 $O/pf384_ms_zscal_a.log env TCLB_VARIANT=zscal python tools/bench_configs.py --configs pf384 --precision mixed-shift
  step "pf384 mixed-shift, vector zonal reads" 300 $O/pf384_ms_a.log python tools/bench_configs.py --configs pf384 --precision mixed-shift
  step "pf384 fp64 + globals every step" 300 $O/pf384_fp64_glob.log bash -c 'python tools/bench_configs.py --configs pf384 && python tools/bench_configs.py --configs pf384 --glob-every-step'
  step "pf384 mixed-shift globals every step" 300 $O/pf384_ms_glob.log python tools/bench_configs.py --configs pf384 --precision mixed-shift --glob-every-step
  step "d3q27 bench fp64 / globals every step" 400 $O/bench_glob.log bash -c 'python bench.py --steps 50 && python bench.py --steps 50 --glob-every-step && python bench.py --steps 50 --precision mixed-shift && python bench.py --steps 50 --precision mixed-shift --glob-every-step' ;;
esac; done
