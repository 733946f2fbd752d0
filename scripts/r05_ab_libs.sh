#!/bin/bash
# Same-process A/B of library builds (scripts/ab_libs.py): AB_LIBS, TAG
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05_ab
mkdir -p "$OUT"
TAG=${TAG:-libs}
timeout -k 10 500 python3 "$ROOT/scripts/ab_libs.py" ${AB_N:-1000000} ${AB_D:-768} ${AB_ROUNDS:-2} > "$OUT/$TAG.log" 2>&1 || { echo "ab run failed rc=$?"; tail -20 "$OUT/$TAG.log"; exit 1; }
tail -1 "$OUT/$TAG.log"
