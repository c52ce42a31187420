#!/bin/bash
# Config-5 K1 launches by grid size (lab library, FMCW_GRID_RANGE caps k_range_px's persistent grid):
# rocprofv3 kernel traces of bench.py --workload c5, then per-launch means of the 3-frame launches
# and of the 1-frame tail launch over the last 10 steps.   usage: GRIDS="512 384 256" tools/k1_tail_lab.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=${LAB_OUT:-gpurun_out/k1_tail}
mkdir -p $O
export TMPDIR=/tmp
for g in ${GRIDS:-512 256}; do
  FMCW_LIB=$PWD/fpga-fmcw-radar-processor_amd/lib/var_lab.so FMCW_GRID_RANGE=$g timeout -k 10 300 \
    rocprofv3 --kernel-trace -d $O/g$g -o run --output-format csv -- \
    python3 bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --no-h2d --no-sub > $O/g$g.log 2>&1 || exit $?
  python3 - $O/g$g/run_kernel_trace.csv $g <<'PY'
import csv, sys, statistics as st
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
for pat in ("k_range_px<", "k_doppler<1024"):
    d = [(e - s) / 1e3 for s, e, n in rows if pat in n]
    tail = [d[i] for i in range(5, len(d), 6)][-10:]
    full = [d[i] for i in range(len(d)) if i % 6 != 5][-50:]
    print("grid", sys.argv[2], pat, "3-frame %.2f us" % st.mean(full), "1-frame %.2f us" % st.mean(tail),
          "mean %.2f us" % ((5 * st.mean(full) + st.mean(tail)) / 6))
PY
done
