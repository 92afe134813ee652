#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprof.  Each GPU step has its own
# time limit; a fault/timeout (exit >= 124 or signal) stops the script before the next GPU step.
# Usage: tools/gpu_round.sh <tag> [steps...]   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift || true
STEPS=${*:-"smoke tests bench"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "GPU step $name ended with $rc: stopping"; exit $rc; fi
  return 0
}
python3 tools/standins.py scene5 scene6 > /dev/null
for s in $STEPS; do
  case $s in
    smoke) run smoke 240 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run tests 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    ptests) run ptests 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    testsall) run testsall 1500 python3 -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 900 python3 bench.py --verbose ;;
    benchq) run benchq 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --verbose ;;
    walks) for w in ${WALKS:-w8 bvh2}; do run walk_$w 600 python3 bench.py --walk $w --steps 2 --warmup 1 --no-cpu-baseline --no-post --verbose; done ;;
    twalks) for w in ${TWALKS:-w8 bvh2}; do run twalk_$w 600 python3 bench.py --trace-walk $w --steps 2 --warmup 1 --no-cpu-baseline --no-post --no-count --verbose; done ;;
    s6frames) for f in ${FRAMES:-world auto}; do run s6_frame_$f 900 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --frame $f --steps 1 --warmup 1 --no-cpu-baseline --no-post --verbose; done ;;
    s6var) for v in ${VARS:-$(ls c-raytracer_amd/lib/var)}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/$v/librtx.so run s6var_$v 900 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --steps 1 --warmup 1 --no-cpu-baseline --no-post --verbose; done ;;
    s6slot) for sl in ${SLOTS:-64 16}; do run s6slot_$sl 900 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --shadow-slot $sl --steps 1 --warmup 1 --no-cpu-baseline --no-post --no-count --verbose; done ;;
    cfgs) # every BASELINE config on one GPU, each line with the reference CPU baseline and closest-only rate
      run cfg0_scene1_512 600 python3 bench.py --scene scene1 --width 512 --height 512 --steps 5 --warmup 1 --verbose &&
      run cfg1_scene3_1080p_n16 600 python3 bench.py --scene scene3 --spp 16 --steps 3 --warmup 1 --verbose &&
      run cfg2_scene5_1080p_n64 600 python3 bench.py --steps 3 --warmup 1 --verbose &&
      run cfg3_scene5_1080p_n256 900 python3 bench.py --spp 256 --steps 1 --warmup 1 --verbose &&
      run cfg4_scene6_2160p_n128 900 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --steps 2 --warmup 1 --verbose &&
      run cfgl8_scene5_l8 900 python3 bench.py --scene scene5_l8 --steps 2 --warmup 1 --verbose ;;
    s3walks) for w in ${S3WALKS:-linear bvh2}; do run s3_walk_$w 600 python3 bench.py --scene scene3 --spp 16 --walk $w --steps 3 --warmup 1 --no-cpu-baseline --no-post --verbose; done ;;
    nowalk) RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/nowalk/librtx.so run nowalk 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count --no-post --verbose ;;
    uploadprof) for sc in ${UPSCENES:-scene5 scene6}; do run uploadprof_$sc 300 rocprofv3 --kernel-trace --stats -d "$OUT/uploadprof_$sc" -o run --output-format csv -- python3 tools/dev/upload_phases.py $sc; done ;;
    grouptests) run grouptests 900 python3 -u -m pytest tests/test_gpu_group.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    treediff) run treediff 600 python3 -u -m pytest tests/test_gpu_build.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "collapse_equals or builds_the_host" ;;
    grabs) for g in ${GRABS:-2048 8192}; do run grab_$g 600 python3 bench.py --shadow-grab $g --steps 2 --warmup 1 --no-cpu-baseline --no-count --no-post; done ;;
    loopback) for n in ${LOOPN:-2 8}; do run loopback_$n 600 python3 bench.py --gpus $n --loopback --steps 3 --warmup 1 --no-cpu-baseline ${LOOPARGS:-}; done ;;
    slottests) run slottests 600 python3 -u -m pytest tests/test_gpu_slots.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    trtests) run trtests 600 python3 -u -m pytest tests/test_gpu_torchrun.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    trbench) RTX_BENCH_REHEARSE=gloo run trbench 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=${TRN:-2} --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${TRN:-2} --steps 2 --warmup 1 --cpu-target-s 4 ;;
    frametests) run frametests 900 python3 -u -m pytest tests/test_gpu_frame.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    buildtests) run buildtests 900 python3 -u -m pytest tests/test_gpu_build.py tests/test_gpu_frame.py tests/test_gpu_group.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    uploadhip) for sc in ${UPSCENES:-scene6}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/meas/librtx.so run uploadhip_$sc 300 rocprofv3 --hip-trace --kernel-trace --stats -d "$OUT/uploadhip_$sc" -o run --output-format csv -- python3 tools/dev/upload_phases.py $sc; done ;;
    upload) for sc in ${UPSCENES:-scene5 scene6}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/meas/librtx.so run upload_$sc 300 python3 tools/dev/upload_phases.py $sc; done ;;
    s3) run s3 600 python3 bench.py --scene scene3 --width 1920 --height 1080 --spp 16 --steps 3 --warmup 1 --no-cpu-baseline --no-post --verbose ;;
    l8) run l8 900 python3 bench.py --scene scene5_l8 --steps 1 --warmup 1 --no-cpu-baseline --no-post --verbose ;;
    s6) for w in ${TWALKS:-w8}; do run s6_$w 900 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --trace-walk $w --steps 1 --warmup 1 --no-cpu-baseline --no-post --verbose; done ;;
    occsweep) for o in ${OCCS:-1 6 7 8}; do RTX_SHADOW_OCC=$o run occ$o 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count --no-post; done ;;
    benchr1) RTX_SH_R=1 run benchr1 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --verbose ;;
    variantsc) for v in ${VARS:-$(ls c-raytracer_amd/lib/var)}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/$v/librtx.so run varc_$v 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --verbose; done ;;
    variants) for v in ${VARS:-$(ls c-raytracer_amd/lib/var)}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/$v/librtx.so run var_$v 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count --no-post; done ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count --no-post ${PMCARGS:-} ;;
    pmcf) run pmcf 900 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-} ;;
    pmcw) run pmcw 900 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-} ;;
    pmcv) run pmcv 900 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/pmc_valu" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-} ;;
    pmcvars) for v in ${VARS:-$(ls c-raytracer_amd/lib/var)}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/$v/librtx.so run pmcv_$v 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/pmcv_$v" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-}; done ;;
    envsweep) for kv in ${SWEEP}; do env $kv timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-count --no-post > "$OUT/env_$kv.log" 2>&1; rc=$?; echo "$kv rc=$rc $(grep -o '"shadow_ms": [0-9.]*' "$OUT/env_$kv.log")" | tee -a "$OUT/steps.log"; if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then exit $rc; fi; done ;;
    pmcivars) for v in ${VARS:-$(ls c-raytracer_amd/lib/var)}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/$v/librtx.so run pmci_$v 600 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS -d "$OUT/pmci_$v" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post; done ;;
    pmcvalu) run pmcvalu 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_valu2" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-} ;;
    pmcrates) run pmcrates 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_rates" -o run --output-format csv -- ./tools/dev/valu_rates ;;
    pmcmem) B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-}"
      run pmcm1 600 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d "$OUT/pmc_m1" -o run --output-format csv -- $B &&
      run pmcm2 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE -d "$OUT/pmc_m2" -o run --output-format csv -- $B &&
      run pmcm3 600 rocprofv3 --pmc TD_LOAD_WAVEFRONT_sum TD_SPI_STALL_sum TA_FLAT_READ_WAVEFRONTS_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_RW_READ_REQ_sum GRBM_GUI_ACTIVE -d "$OUT/pmc_m3" -o run --output-format csv -- $B ;;
    pmcta) run pmcta 600 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT -d "$OUT/pmc_ta" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-} ;;
    varcount) for v in ${VARS:-$(ls c-raytracer_amd/lib/var)}; do RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/$v/librtx.so run varcount_$v 600 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-post --verbose; done ;;
    s6sweep) for kv in ${SWEEP}; do env $kv timeout -k 10 300 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --steps 1 --warmup 1 --no-cpu-baseline --no-count --no-post > "$OUT/s6_$kv.log" 2>&1; rc=$?; echo "$kv rc=$rc $(grep -o '"shadow_ms": [0-9.]*' "$OUT/s6_$kv.log")" | tee -a "$OUT/steps.log"; if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then exit $rc; fi; done ;;
    pmcsum) python3 tools/pmc_summary.py ${PMCKEY:-scene5_1920x1080_n64_g1} "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_valu" $( [ -d "$OUT/pmc_ta" ] && echo "$OUT/pmc_ta" ) > "$OUT/pmcsum.log" 2>&1; cp profiles/pmc_k_shadow.json "$OUT/" ;;
  esac
done
echo done
