#!/usr/bin/env bash
# Build variant libraries lib/var_<name>.so of libfmcw.so with build-time switches, for A/B
# timing on the GPU box:  FMCW_LIB=$PWD/fpga-fmcw-radar-processor_amd/lib/var_<name>.so python bench.py ...
# usage: tools/build_variants.sh name=-DFLAG=1,-DFLAG2=1 ...   (variants build one after another,
# each with make -j8 over the translation units)
set -eu
cd "$(dirname "$0")/../fpga-fmcw-radar-processor_amd"
# FMCW_LAB=1: the A/B knobs read from the environment at fmcw_create (FMCW_K1, FMCW_CFAR2D_STEPS,
# FMCW_GRID_*, FMCW_K2_GENERIC); the release library (make) reads none
BASE="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -Wall -Wno-unused-result -Wno-unused-value -DFMCW_LAB=1"
for spec in "$@"; do
  name=${spec%%=*}
  defs=${spec#*=}
  make -s -j8 LIBDIR="build/var_$name" OBJDIR="build/var_$name" HIPFLAGS="$BASE ${defs//,/ }"
  cp "build/var_$name/libfmcw.so" "lib/var_$name.so"
done
ls -la lib/var_*.so
