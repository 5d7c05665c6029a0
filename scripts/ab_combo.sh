#!/bin/bash
# A/B of environment settings on a bench workload, alternating in one call.
#   usage: TAG "A=1,B=0 A=3,B=0 ..." ROUNDS [bench.py args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/$1; SETS=$2; ROUNDS=$3; shift 3
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for set in $SETS; do
    tag=$(echo "$set" | tr ',=' '__')
    env $(echo "$set" | tr ',' ' ') timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/${tag}_$r.log" 2>&1 || exit $?
    echo "$set r$r $(tail -1 "$OUT/${tag}_$r.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
