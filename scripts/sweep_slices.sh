#!/bin/bash
# Corpus-slice sweep for the bf16 Gram kernels (L2-sharing of the query panel):
# C2 (1M x 768 L2, bf16-split) and a 262k x 3072 C5-shaped cosine run.
#   usage (repo root, under gpurun): bash scripts/sweep_slices.sh "2 4 8" [c5]
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/sweep
mkdir -p "$OUT"
export TMPDIR=/tmp MN_GRAM_MAX_SL=480
for s in $1; do
    MN_L2_MIN_SLICES=$s timeout -k 10 200 python -u bench.py --no-c3 --no-c5 --cpu-seconds 0 \
        > "$OUT/c2_s$s.log" 2>&1 || { echo "c2 s=$s failed"; exit 1; }
    echo "c2 s=$s: $(grep -o '"ms_gram": [0-9.]*' "$OUT/c2_s$s.log" | tail -1)"
    if [ "$2" = "c5" ]; then
        MN_BF16_MIN_SLICES=$s timeout -k 10 200 python -u scripts/bench_bf16.py --n 524288 \
            > "$OUT/c5_s$s.log" 2>&1 || { echo "c5 s=$s failed"; exit 1; }
        echo "c5 s=$s: $(grep -o '"gram_tflops": [0-9.]*' "$OUT/c5_s$s.log" | tail -1)"
    fi
done
