#!/bin/bash
# Same-process A/B of sweep variants (tuning knobs): AB_ENVS / AB_PROBES as ab_sweep.py
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r06_ab
mkdir -p "$OUT"
TAG=${TAG:-ab}
timeout -k 10 ${AB_TIMEOUT:-500} python3 "$ROOT/scripts/ab_sweep.py" ${AB_N:-1000000} ${AB_D:-768} ${AB_ROUNDS:-2} > "$OUT/$TAG.log" 2>&1 || { echo "ab run failed rc=$?"; tail -20 "$OUT/$TAG.log"; exit 1; }
tail -3 "$OUT/$TAG.log"
