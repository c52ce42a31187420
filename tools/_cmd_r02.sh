set -u
L=$PWD/fpga-fmcw-radar-processor_amd/lib
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "range_ct or config5 or process_parity or fused or tb" --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sel.log 2>&1 || { tail -30 gpurun_out/pytest_sel.log; exit 1; }
tail -2 gpurun_out/pytest_sel.log
for w in c2 c3 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-h2d > gpurun_out/bench_${w}_hw2.log 2>&1 || exit 1
  FMCW_LIB=$L/var_holdw1.so timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-h2d > gpurun_out/bench_${w}_hw1.log 2>&1 || exit 1
done
