#!/bin/bash
# cosine exact dot with 4 gathers in flight: bf16/cos parity tests + C5 timing
cd /root/repo
bash scripts/gpu_steps.sh \
  "ctests|400|python -u -m pytest tests/test_knn_bf16_gpu.py tests/test_knn_cos_gpu.py -x -q --timeout 200 --timeout-method thread" \
  "c5rr|300|C5P_VARIANTS='default' C5P_REPS=2 python -u scripts/c5_probe.py"
