#!/bin/bash
# re-rank fold with 4 float4 gathers in flight: kNN parity tests + C2 timing
cd /root/repo
bash scripts/gpu_steps.sh \
  "ktests|400|python -u -m pytest tests/test_knn_gpu.py tests/test_knn_bf16_gpu.py -x -q --timeout 200 --timeout-method thread" \
  "ab_rr|200|AB_ENVS='MN_X1_SYM=1' AB_PROBES= python -u scripts/ab_sweep.py 1000000 768 3"
