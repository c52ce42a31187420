#!/bin/bash
# A/B of variant libraries (tools/build_variants.sh) on the headline workload alone (config 2,
# --no-sub), interleaved ROUNDS times: $AB_OUT/<variant>_<round>.log, one summary line each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=${AB_OUT:-gpurun_out/ab_c2}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:?}; do
    FMCW_LIB=$PWD/fpga-fmcw-radar-processor_amd/lib/var_$v.so timeout -k 10 200 \
      python bench.py --no-sub --no-cpu-baseline --no-h2d ${BENCH_ARGS:-} > $O/${v}_$r.log 2>&1 || exit $?
    python3 - "$O/${v}_$r.log" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        k = d["kernels"]
        print(sys.argv[1].split("/")[-1], round(d["value"]), {n: k[n]["avg_launch_ms"] for n in k})
PY
  done
done
