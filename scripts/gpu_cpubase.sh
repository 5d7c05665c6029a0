#!/bin/bash
# BASELINE.md §3 CPU rows on the GPU box's host (no GPU use): one bounded slice per
# lease, runs accumulated in gpurun_out/cpu_baseline_full.json (--append), which is
# copied to profiles/ when complete.   usage: ROWS THREADS RUNS SECONDS
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p gpurun_out
J=gpurun_out/cpu_baseline_full.json
[ -f "$J" ] || cp profiles/cpu_baseline_full.json "$J" 2>/dev/null || true
timeout -k 10 "$4" python -u scripts/cpu_baseline_full.py --rows "$1" --threads "$2" --runs "$3" --out "$J" --append
