#!/usr/bin/env bash
# Build variant libraries lib/var_<name>.so of libfmcw.so with build-time switches, for
# A/B timing on the GPU box:  FMCW_LIB=.../lib/var_<name>.so python tools/ablate.py ...
# usage: tools/build_variants.sh name=-DFLAG=1,-DFLAG2=1 ...
set -eu
cd "$(dirname "$0")/../fpga-fmcw-radar-processor_amd"
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -fvisibility=hidden -Wall -Wno-unused-result -Wno-unused-value"
pids=()
for spec in "$@"; do
  name=${spec%%=*}
  defs=${spec#*=}
  /opt/rocm/bin/hipcc $FLAGS ${defs//,/ } -shared -o "lib/var_${name}.so" csrc/fmcw_api.hip csrc/fmcw_gather.hip csrc/tws_tracker.cpp -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la lib/var_*.so
