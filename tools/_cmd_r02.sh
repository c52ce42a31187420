set -u
L=$PWD/fpga-fmcw-radar-processor_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "range_ct or config5 or 8192 or fp16" --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sel.log 2>&1 || { tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -2 gpurun_out/pytest_sel.log
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d > gpurun_out/bench_c5_t1.log 2>&1 || exit 1
FMCW_LIB=$L/var_t2.so timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d > gpurun_out/bench_c5_t2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --spectrum f16 > gpurun_out/bench_c5_t1_f16.log 2>&1 || exit 1
