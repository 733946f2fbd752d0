#!/bin/bash
# r03 GPU pass: K1 tests (+ full-size with their printed stats), bench, and a
# kernel trace of the item-Laplacian probe.
cd /root/repo
bash scripts/gpu_steps.sh \
  "knn_tests|500|python -u -m pytest tests/test_knn_gpu.py tests/test_fullsize_gpu.py tests/test_shard_gpu.py -x -v -s --timeout 300 --timeout-method thread" \
  "bench|300|python -u bench.py" \
  "lap_trace|180|rocprofv3 --kernel-trace --stats -d gpurun_out/lap_prof -o lap -- python3 scripts/lap_probe.py"
