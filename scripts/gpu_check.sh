#!/bin/bash
# One GPU-box pass (run from the repo root under gpurun): parity tests, the
# bench line, rocprofv3 evidence for the dominant kernel (kernel trace + HBM
# PMC passes), and a kernel trace of the C3 legs.  Every GPU step has its own
# time limit; the chain stops at the first failure.
#   usage: bash scripts/gpu_check.sh <tag> [tests|bench|prof|c3]...  (default: all)
set -o pipefail
TAG=${1:-latest}; shift
STEPS=${*:-tests bench prof c3}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
    case $s in
    tests)
        timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 \
            --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests failed rc=$?"; exit 1; } ;;
    bench)
        timeout -k 10 300 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed rc=$?"; exit 1; } ;;
    prof)
        bash scripts/profile_gram.sh "$TAG" > "$OUT/prof.log" 2>&1 || { echo "prof failed"; exit 1; } ;;
    c3)
        (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$OUT/prof_c3" -o run -- python3 "$R/bench.py" --cpu-seconds 0 --no-c5 \
            --warmup 0 --steps 1 > "$OUT/prof_c3.log" 2>&1) || { echo "c3 trace failed"; exit 1; } ;;
    esac
    echo "step $s ok"
done
