#!/bin/bash
# Round-6 measurement: the driver's bench command, then the rocprofv3 legs
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r06}
mkdir -p "$ROOT/gpurun_out"
timeout -k 10 400 python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$ROOT/gpurun_out/${TAG}_bench.log" 2>&1 || { echo "bench failed rc=$?"; tail -5 "$ROOT/gpurun_out/${TAG}_bench.log"; exit 1; }
echo "bench ok"
[ "${LEGS:-1}" = "1" ] || exit 0
bash "$ROOT/scripts/profile_legs.sh" "$TAG"
