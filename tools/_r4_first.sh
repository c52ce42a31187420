set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r4a
timeout -k 10 120 tools/k2_read_probe 3 20 > gpurun_out/r4a/k2_read_probe_3f.log 2>&1 &&
timeout -k 10 120 tools/k2_read_probe 12 10 > gpurun_out/r4a/k2_read_probe_12f.log 2>&1 &&
bash tools/gpu_run.sh tests_all smoke bench
