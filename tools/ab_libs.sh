#!/bin/bash
# A/B of variant libraries (tools/build_variants.sh) on the full default bench (configs 2, 3, 5),
# interleaved ROUNDS times: gpurun_out/ab/<variant>_<round>.log
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=${AB_OUT:-gpurun_out/ab}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:?}; do
    FMCW_LIB=$PWD/fpga-fmcw-radar-processor_amd/lib/var_$v.so timeout -k 10 300 \
      python bench.py --no-cpu-baseline --no-h2d > $O/${v}_$r.log 2>&1 || exit $?
  done
done
for f in $O/*.log; do
  python3 - "$f" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        rs = (d, d["config3"], d["config5"])
        print(sys.argv[1].split("/")[-1], [round(x["value"]) for x in rs],
              [x["kernels"]["k_compact"]["avg_launch_ms"] for x in rs])
PY
done
