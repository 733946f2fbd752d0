#!/bin/bash
# rocprofv3 SQ counters for the K3 kernels (scripts/energy_ab.py, default
# variant): kernel trace + three SQ passes (no trace domain combined with --pmc)
set -o pipefail
TAG=${1:-energy}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp EAB_VARIANTS=default
cd /tmp || exit 1
run() {
    local name=$1; shift
    timeout -k 10 200 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 "$ROOT/scripts/energy_ab.py" > "$OUT/$name.log" 2>&1 || { echo "$name pass failed rc=$?"; exit 1; }
    echo "pass $name ok"
}
run kt --kernel-trace --stats
run p1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES
run p3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU
run p4 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM
echo "energy passes done"
