#!/bin/bash
# A/B of the corner-turned spectrum format at config 2 (bench.py --spectrum f32 | s48), with the
# default library and optional variant libraries (VARIANTS, tools/build_variants.sh), interleaved
# ROUNDS times: gpurun_out/<AB_OUT>/<lib>_<spec>_<round>.log, then a one-line summary per log.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=${AB_OUT:-gpurun_out/spec_ab}
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in default ${VARIANTS:-}; do
    lib=$PWD/fpga-fmcw-radar-processor_amd/lib/libfmcw.so
    [ "$v" != default ] && lib=$PWD/fpga-fmcw-radar-processor_amd/lib/var_$v.so
    for sp in ${SPECS:-f32 s48}; do
      FMCW_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-h2d --no-sub --spectrum $sp \
        ${BENCH_ARGS:-} > $O/${v}_${sp}_$r.log 2>&1 || exit $?
    done
  done
done
for f in $O/*.log; do
  python3 - "$f" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        k = d["kernels"]
        print(sys.argv[1].split("/")[-1], round(d["value"]), "chunk", d["chunk_frames"],
              {n: (k[n]["avg_launch_ms"], k[n].get("frac")) for n in ("k_range", "k_doppler", "k_compact") if n in k})
PY
done
