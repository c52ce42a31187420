set -u
bash tools/gpu_run.sh gpu_cfar_tests || exit 1
timeout -k 10 200 python tools/cfar2d_bench.py --frames 16 > gpurun_out/cfar2d_16.log 2>&1 || exit 1
for w in c3 c5; do timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-h2d > gpurun_out/bench_${w}_x.log 2>&1 || exit 1; done
