#!/bin/bash
# SQ-level counters for one kernel-bearing python command, one --pmc pass per group
# (no trace domains combined with --pmc).  Run on the GPU box from the repo root.
# Usage: scripts/pmc_sq.sh <tag> <python script> [args...]
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sq_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
SCRIPT=$ROOT/$1; shift
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
           "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
        python3 "$SCRIPT" "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
python3 "$ROOT/scripts/sq_summary.py" "$OUT"
