#!/bin/bash
# Warm-up study (round 4): timed frames/s vs untimed warm-up length.  --prewarm-s 0 turns off
# bench.py's time-based pre-warm so only --warmup steps run before the timed region.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/warmup
mkdir -p $O
run() { timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-h2d > $O/$(echo "$@" | tr ' -' '_').log 2>&1; }
run --steps 10 --warmup 3 --prewarm-s 0 &&
run --steps 10 --warmup 100 --prewarm-s 0 &&
run --steps 100 --warmup 3 --prewarm-s 0 &&
run --steps 10 --warmup 3
echo rc=$?
for f in $O/*.log; do
  python3 - "$f" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1].split("/")[-1], d.get("warmup_steps_run"),
              [round(x["value"]) for x in (d, d["config3"], d["config5"])])
PY
done
