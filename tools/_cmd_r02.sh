set -u
L=$PWD/fpga-fmcw-radar-processor_amd/lib
timeout -k 10 300 python tools/ablate.py --variants base,nocfar,bare > gpurun_out/abl_def.log 2>&1 || exit 1
for v in c1a1 c1a2; do FMCW_LIB=$L/var_$v.so timeout -k 10 300 python tools/ablate.py --variants base > gpurun_out/abl_$v.log 2>&1 || exit 1; done
