set -o pipefail
OUT=gpurun_out/r06_search
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_search_gpu.py > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python3 scripts/r06_search_ab.py > $OUT/ab.log 2>&1
