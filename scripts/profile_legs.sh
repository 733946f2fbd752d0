#!/bin/bash
# rocprofv3 evidence for EVERY kernel of one bench.py step (C2 graph, the C3
# legs, the C5 leg): kernel trace, separate FETCH_SIZE / WRITE_SIZE passes and
# four SQ counter groups (no trace domain is combined with --pmc).  Run on the
# GPU box from the repo root; summarise with scripts/legs_summary.py.
#   usage: scripts/profile_legs.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-legs}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/legs_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
ARGS=(--cpu-seconds 0 --warmup 0 --steps 1 --no-c4-sim "$@")
run() {  # name, rocprofv3 options...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/$name.log" 2>&1 || { echo "$name pass failed rc=$?"; exit 1; }
    echo "pass $name ok"
}
run kt --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run p1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run p2 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS
run p3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU
run p4 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS
echo "legs passes done"
