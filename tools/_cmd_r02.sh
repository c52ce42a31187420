set -u
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_all.log; grep -E "FAILED|Error" gpurun_out/pytest_all.log | head -20
[ $rc -le 1 ] || exit $rc
for sp in f32 f16; do
  timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --spectrum $sp > gpurun_out/bench_c5_$sp.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --spectrum f16 > gpurun_out/bench_c2_f16.log 2>&1 || exit 1
