#!/bin/bash
# rocprofv3 kernel trace of the C3 item Laplacian (UNION + MAX) at C3 size
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05_prof_lap
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
AB_LIBS="$ROOT/matternet-rs_amd/libmatternet_hip.so" AB_ROUNDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/scripts/ab_lap.py" > "$OUT/log.txt" 2>&1 || { echo "prof failed rc=$?"; tail "$OUT/log.txt"; exit 1; }
echo done
