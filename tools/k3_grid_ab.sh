#!/bin/bash
# K3b / K3c grid sweep (round 5): the lab library (tools/build_variants.sh lab=) with FMCW_GRID_K3B /
# FMCW_GRID_K3C, config-5 K3 alone (tools/cfar2d_bench.py), two interleaved passes
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=${AB_OUT:-gpurun_out/k3grid}
mkdir -p $O
L=$PWD/fpga-fmcw-radar-processor_amd/lib/${LIB:-var_lab}.so
for r in 1 2; do
  for g in ${GRIDS:-2048,1024 1024,1024 4096,1024 2048,256 2048,512}; do
    b=${g%,*}; c=${g#*,}
    FMCW_LIB=$L FMCW_GRID_K3B=$b FMCW_GRID_K3C=$c timeout -k 10 120 python tools/cfar2d_bench.py --workloads ${WL:-c5} --ovr 0 \
      > $O/g${b}_${c}_$r.log 2>&1 || exit $?
    echo "$b $c $r $(grep -h '^{' $O/g${b}_${c}_$r.log | python3 -c 'import json,sys; print(*[json.loads(l)["k_cfar2d_us_per_launch"] for l in sys.stdin])')"
  done
done
