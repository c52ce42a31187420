#!/usr/bin/env bash
# Config-2 bench under the chunking variants of fmcw_enqueue (serial chunks, two-stream
# pipeline with chunk / buffer count, fused kernel); one line per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # label env...
  local label=$1; shift
  local line
  line=$(env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d 2>/dev/null | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); k=d['kernels']; print(sys.argv[1], d['value'], {n:(round(v['avg_ms']*1e3,1), v['launches_per_step']) for n,v in k.items()})" "$label" "$line" || { echo "$label FAILED"; exit 1; }
}
run serial_128 FMCW_PIPE=0
for c in ${CHUNKS:-16 32 64}; do
  for b in ${BUFS:-2 3}; do
    run pipe_c${c}_b${b} FMCW_PIPE=1 FMCW_PIPE_CHUNK=$c FMCW_PIPE_BUFS=$b
  done
done
