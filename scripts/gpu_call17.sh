#!/bin/bash
cd /root/repo
bash scripts/gpu_steps.sh \
  "bf16_tests|400|python -u -m pytest tests/test_knn_bf16_gpu.py tests/test_graph_gpu.py tests/test_knn_gpu.py -x -q -s --timeout 250 --timeout-method thread" \
  "c5_ab|400|C5P_VARIANTS='default;MN_BF16_SYM=0' python -u scripts/c5_probe.py" \
  "full|400|python -u -m pytest tests/test_fullsize_gpu.py -x -q -s --timeout 300 --timeout-method thread"
