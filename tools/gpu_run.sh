#!/usr/bin/env bash
# Run GPU steps on the gpurun box, each under its own time limit; stop at the first step that
# crashes, aborts or times out (exit codes other than 0 / 1), continue past plain test failures.
# usage: tools/gpu_run.sh <step>...   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${GPU_RUN_OUT:-gpurun_out}
mkdir -p "$OUT"
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name exited $rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -x --timeout 170 --timeout-method thread -p no:cacheprovider ;;
    tests_all) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider ;;
    tests_r02) run pytest_gpu_r02 600 python -u -m pytest tests/test_gpu_r02.py -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider ;;
    bench) run bench 600 python bench.py --steps 10 --warmup 3 ;;
    bench_c*) run "$s" 600 python bench.py --workload "${s#bench_}" --steps 10 --warmup 3 --no-cpu-baseline ;;
    prof) run rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline ;;
    ablate) run ablate 600 python tools/ablate.py ${ABLATE_ARGS:-} ;;
    ablate_libs)  # every variant build (tools/build_variants.sh), same ablation variants
      for lib in fpga-fmcw-radar-processor_amd/lib/var_*.so; do
        v=$(basename "$lib" .so)
        FMCW_LIB="$PWD/$lib" run "ablib_${v#var_}" 300 python tools/ablate.py ${ABLATE_ARGS:-}
      done ;;
    cfar2d) run cfar2d 300 python tools/cfar2d_bench.py ${CFAR2D_ARGS:-} ;;
    cfar2d_steps)  # k_cfar2d alone per strip length (FMCW_CFAR2D_STEPS; 0 = cost model)
      for st in ${STEPS:-0 16 64 128}; do
        FMCW_CFAR2D_STEPS=$st run "cfar2d_steps$st" 300 python tools/cfar2d_bench.py ${CFAR2D_ARGS:-}
      done ;;
    cfar2d_libs)  # the standalone 2-D CFAR timing for every variant build
      for lib in fpga-fmcw-radar-processor_amd/lib/var_*.so; do
        v=$(basename "$lib" .so)
        FMCW_LIB="$PWD/$lib" run "cfar2d_${v#var_}" 300 python tools/cfar2d_bench.py ${CFAR2D_ARGS:-}
      done ;;
    gpu_cfar_tests) run pytest_cfar 600 python -u -m pytest tests -m gpu -v -x -k "cfar or 2d or os2d or config5 or c5 or tb" --timeout 170 --timeout-method thread -p no:cacheprovider ;;
    pmcf_c*) w=${s#pmcf_}; run "pmcf_$w" 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmcf_$w" -o run --output-format csv -- python3 bench.py --workload "$w" --steps 2 --warmup 1 --no-cpu-baseline --no-h2d ;;
    pmcw_c*) w=${s#pmcw_}; run "pmcw_$w" 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmcw_$w" -o run --output-format csv -- python3 bench.py --workload "$w" --steps 2 --warmup 1 --no-cpu-baseline --no-h2d ;;
    bench_libs)  # config-2 bench for every variant library, then the default one again
      for lib in fpga-fmcw-radar-processor_amd/lib/var_*.so; do
        v=$(basename "$lib" .so)
        FMCW_LIB="$PWD/$lib" run "bench_lib_${v#var_}" 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d ${BENCH_ARGS:-}
      done
      run bench_lib_default 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d ${BENCH_ARGS:-} ;;
    bench_f16) run bench_f16 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --spectrum f16 ;;
    bench_generic) FMCW_K2_GENERIC=1 run bench_generic 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d ;;
    bench_quick) run bench_quick 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d ;;
    chunk_sweep)  # config-2 bench per K1/K2 chunk size (frames per launch)
      for c in ${CHUNKS:-96 128 256 512 1024}; do
        run "bench_chunk$c" 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --chunk "$c"
      done ;;
    counters) run counters 120 rocprofv3 -L ;;
    # round 3: one default bench command (config 2 + the config-3 / config-5 sub-records), its
    # kernel-trace stats and its three PMC passes (tools/pmc_summary.py normalises per frame)
    prof3) run rocprof3_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof3" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d ;;
    pmc3_fetch) run pmc3_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc3_fetch" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-h2d ;;
    pmc3_write) run pmc3_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc3_write" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-h2d ;;
    pmc3_sq) run pmc3_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d "$OUT/pmc3_sq" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-h2d ;;
    pmc3_sq2) run pmc3_sq2 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU -d "$OUT/pmc3_sq2" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-h2d ;;
    gloo2)  # N = 2 ranks on this one GPU over gloo: a rehearsal of bench.py's launch, barrier and max-over-ranks timing
      run bench_2rank_gloo 600 env FMCW_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-h2d --no-sub --frames 256 ;;
    k3lab) run k3lab_c5 300 tools/k3_lab 16 5 ;;
    k3labs)  # every tools/k3_lab_<variant> binary (built on the CPU host with other -D switches)
      for b in tools/k3_lab_*; do run "k3lab_c5_${b#tools/k3_lab_}" 300 "$b" 16 5; done ;;
    lib_c5)  # config 5 with a variant library (LIB=var_x) at chunk sizes CHUNKS
      for c in ${CHUNKS:-0 12}; do
        FMCW_LIB="$PWD/fpga-fmcw-radar-processor_amd/lib/${LIB}.so" run "bench_c5_${LIB}_chunk$c" 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --chunk "$c"
      done ;;
    k1lab)  # K1 variants stand-alone (tools/k1_lab, built on the CPU host): configs 5, 3, 2048
      run k1lab_c5_3f 120 tools/k1_lab 8192 1024 1 3 1 &&
      run k1lab_c5_12f 120 tools/k1_lab 8192 1024 1 12 1 &&
      run k1lab_c3_3f 120 tools/k1_lab 4096 512 4 3 0 &&
      run k1lab_c3_12f 120 tools/k1_lab 4096 512 4 12 0 ;;
    chunkc_c*)  # configs 3 / 5: K1 / K2 per-launch times per chunk size (24 frames per step)
      w=${s#chunkc_}
      for c in ${CHUNKS:-3 6 12 24}; do
        run "bench_${w}_chunk$c" 300 python bench.py --workload "$w" --frames 24 --steps 6 --warmup 2 --no-cpu-baseline --no-h2d --chunk "$c"
      done ;;
    chunk16_c*)  # configs 3 / 5 at the bench's 16 frames per step, small chunk sizes
      w=${s#chunk16_}
      for c in ${CHUNKS:-1 2 3 4}; do
        run "bench16_${w}_chunk$c" 300 python bench.py --workload "$w" --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --chunk "$c"
      done ;;
    pmcsq2_c*) w=${s#pmcsq2_}; run "pmcsq2_$w" 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d "$OUT/pmcsq2_$w" -o run --output-format csv -- python3 bench.py --workload "$w" --steps 2 --warmup 1 --no-cpu-baseline --no-h2d ;;
    prof_c*) w=${s#prof_}; run "rocprof_stats_$w" 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv -- python3 bench.py --workload "$w" --steps 5 --warmup 2 --no-cpu-baseline --no-h2d ;;
    pmcsq_c*) w=${s#pmcsq_}; run "pmcsq_$w" 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/pmcsq_$w" -o run --output-format csv -- python3 bench.py --workload "$w" --steps 2 --warmup 1 --no-cpu-baseline --no-h2d ;;
    pmc_sq) run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT -d "$OUT/pmc_sq" -o run --output-format csv -- python3 tools/ablate.py --frames 256 --steps 2 --variants base ;;
    pmc_var_*) v=${s#pmc_var_}; run "pmc_$v" 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/pmc_$v" -o run --output-format csv -- python3 tools/ablate.py --frames 256 --steps 2 --variants "$v" ;;
    pmc2_var_*) v=${s#pmc2_var_}; run "pmc2_$v" 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES -d "$OUT/pmc2_$v" -o run --output-format csv -- python3 tools/ablate.py --frames 256 --steps 2 --variants "$v" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== all done"
