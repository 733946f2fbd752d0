#!/bin/bash
# Round 5 K1 diagnosis: sweep vs K-loop / L2-resident probes (same process),
# then the sweep's L2 hit counters (own --pmc pass).  GPU box, repo root.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r05_k1
mkdir -p "$OUT"
AB_PROBES=${AB_PROBES:-noepi,l2res,l2res_noepi} AB_ENVS="MN_X1_SYM=1" timeout -k 10 300 \
    python3 "$ROOT/scripts/ab_sweep.py" 1000000 768 2 > "$OUT/probes.log" 2>&1 || { echo "probe run failed rc=$?"; exit 1; }
export TMPDIR=/tmp
cd /tmp || exit 1
[ -n "$NO_PMC" ] && { echo done; exit 0; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/l2" -o run -- \
    python3 "$ROOT/scripts/bench_k1.py" --n 1000000 --reps 1 > "$OUT/l2.log" 2>&1 || { echo "pmc pass failed rc=$?"; exit 1; }
echo done
