#!/bin/bash
# K3 strip direction A/B (round 5): variant libraries VARIANTS (default: before / altdir),
# interleaved bench runs of workload WL (c3) and one FETCH_SIZE pass each (K3's map traffic)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=${AB_OUT:-gpurun_out/k3dir}
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/fpga-fmcw-radar-processor_amd/lib
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-before altdir}; do
    FMCW_LIB=$L/var_$v.so timeout -k 10 300 python bench.py --workload ${WL:-c3} --no-cpu-baseline --no-h2d --no-sub \
      > $O/${v}_$r.log 2>&1 || exit $?
  done
done
for v in ${VARIANTS:-before altdir}; do
  FMCW_LIB=$L/var_$v.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$v -o run --output-format csv -- \
    python3 bench.py --workload ${WL:-c3} --steps 2 --warmup 1 --prewarm-s 0 --no-cpu-baseline --no-h2d --no-sub > $O/fetch_$v.log 2>&1 || exit $?
done
for f in $O/*_[0-9].log; do
  python3 - "$f" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1].split("/")[-1], round(d["value"]), {n: d["kernels"][n]["avg_launch_ms"] for n in ("k_range", "k_doppler", "k_cfar")})
PY
done
for v in ${VARIANTS:-before altdir}; do
  python3 - $O/fetch_$v/run_counter_collection.csv $v <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if k.startswith("void fmcw::k_cfar2d") and ("<512" in k or "<1024" in k):
        name = k.split("(")[0].replace("void fmcw::", "")
        acc[name] += float(r["Counter_Value"]); n[name] += 1
for k in acc:
    # FETCH_SIZE in KiB, x2 for the gfx950 wide-read undercount; 80 frames per run as tools/pmc_summary.py
    print(sys.argv[2], k, "launches", n[k], "fetch MB per frame %.2f" % (acc[k] * 2 * 1024 / 1e6 / 80), "(algorithmic: config 3 8.39, config 5 33.55)")
PY
done
