#!/usr/bin/env bash
# Round 6: K3 A/B on the GPU box -- the 2-D CFAR GPU tests with the in-tree library, then
# tools/cfar2d_bench.py (configs 3 / 5, bench maps) interleaved: libfmcw.so ("new") against
# lib/var_base.so ("base", the library before the change, built on the CPU host with
# `git stash; tools/build_variants.sh base=-DFMCW_VAR_BASE=1; git stash pop`).
# usage (gpurun): bash tools/k3_cd_ab.sh    logs: gpurun_out/r06d/
set -u
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "cfar or 2d or os2d or c5 or c3 or tb or clutter or override or lattice" --timeout 170 --timeout-method thread -p no:cacheprovider > $O/pytest_k3.log 2>&1; rc=$?; tail -3 $O/pytest_k3.log; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  for v in new base; do
    if [ $v = base ]; then L=$PWD/fpga-fmcw-radar-processor_amd/lib/var_base.so; else L=$PWD/fpga-fmcw-radar-processor_amd/lib/libfmcw.so; fi
    FMCW_LIB=$L timeout -k 10 300 python tools/cfar2d_bench.py --workloads c3,c5 --iters 20 > $O/cfar2d_${v}_$i.log 2>&1 || exit $?
    echo "== $v $i"; grep '^{' $O/cfar2d_${v}_$i.log | cut -c1-220
  done
done
