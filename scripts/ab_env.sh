#!/bin/bash
# A/B of an environment knob on a bench workload, alternating in one call.
#   usage: TAG VAR "v1 v2 ..." ROUNDS [bench.py args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; VAR=$2; VALS=$3; ROUNDS=$4; shift 4
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/${VAR}_${v}_$r.log" 2>&1 || exit $?
    echo "$VAR=$v r$r $(tail -1 "$OUT/${VAR}_${v}_$r.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
