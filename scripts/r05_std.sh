set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sorted_index_gpu.py > gpurun_out/sidx_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/std_probe.py > gpurun_out/std_rl_ab.log 2>&1
