#!/usr/bin/env bash
# Config-2 bench of the fused kernel under role splits (FMCW_FUSED_NB) plus its phase trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # label env...
  local label=$1; shift
  local line
  line=$(env "$@" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-h2d 2>/dev/null | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); k=d['kernels']; print(sys.argv[1], d['value'], d['fused_path'], {n:(round(v['avg_ms']*1e3,1), v['launches_per_step']) for n,v in k.items()})" "$label" "$line" || { echo "$label FAILED"; exit 1; }
}
for nb in ${NBS:-64 96}; do
  run fused_nb$nb FMCW_FUSED=1 FMCW_FUSED_NB=$nb FMCW_FUSED_VERBOSE=1
done
FMCW_FUSED=1 FMCW_FUSED_NB=${TRACE_NB:-96} timeout -k 10 120 python tools/fused_trace.py
