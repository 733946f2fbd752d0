#!/bin/bash
# rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box from the repo root).
#   pass 1: --kernel-trace --stats (per-kernel durations)
#   pass 2: --pmc FETCH_SIZE   pass 3: --pmc WRITE_SIZE (separate passes: TCC slots)
# Usage: scripts/profile_gram.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-latest}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS=(--cpu-seconds 0 --warmup 0 --steps 1 --no-c3 --no-c5 "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/kt.log" 2>&1 || { echo "kt pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "profile passes done"
find "$OUT" -name "*.csv" | head -50
