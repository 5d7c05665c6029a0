#!/bin/bash
# headline A/B: the round-4 tree at 46a4e48 (ab_old/, a git worktree built in-tree) vs the current tree, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/${1:-ab_old}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  (cd ab_old && timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline) > "$OUT/old_$i.out" 2>&1 || exit 1
  echo "old $i: $(grep '^{' $OUT/old_$i.out | tail -1 | cut -c100-200)"
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/new_$i.out" 2>&1 || exit 1
  echo "new $i: $(grep '^{' $OUT/new_$i.out | tail -1 | cut -c100-200)"
done
