#!/bin/bash
# r03: SW_SYM block order / tiles-per-block A/B (+ K-loop probes), then the
# full-size C2-clustered and C4 one-rank tests with their printed stats
cd /root/repo
bash scripts/gpu_steps.sh \
  "ab_order|400|AB_ENVS='MN_SYM_ORDER=0;MN_SYM_ORDER=1;MN_SYM_ORDER=1,MN_SYM_TPB=64;MN_SYM_ORDER=1,MN_SYM_TPB=128;MN_SYM_ORDER=1,MN_SYM_TPB=512' AB_PROBES=noepi python -u scripts/ab_sweep.py 1000000 768 2" \
  "full|500|python -u -m pytest tests/test_fullsize_gpu.py tests/test_shard_gpu.py -x -v -s --timeout 300 --timeout-method thread"
