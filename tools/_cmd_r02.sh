set -u
# round-2 final measurement set (tools/gpu_run.sh steps)
bash tools/gpu_run.sh tests_all smoke bench prof pmc_fetch pmc_write bench_c3 bench_c5 prof_c3 prof_c5
