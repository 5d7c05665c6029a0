#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SKIP_TESTS= bash scripts/gpu_full.sh "$1" || exit $?
bash scripts/gpu_seq.sh "$1_seq" || exit $?
