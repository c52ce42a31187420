set -u
L=$PWD/fpga-fmcw-radar-processor_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_all.log; grep -E "FAILED" gpurun_out/pytest_all.log | head; [ $rc -le 1 ] || exit $rc
for w in c3 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-h2d > gpurun_out/bench_${w}_pf.log 2>&1 || exit 1
  FMCW_LIB=$L/var_pf256.so timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-h2d > gpurun_out/bench_${w}_nopf.log 2>&1 || exit 1
done
