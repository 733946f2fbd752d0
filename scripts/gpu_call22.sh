#!/bin/bash
# C5 phase-1 sample grid under the symmetric cosine sweep (same process)
cd /root/repo
bash scripts/gpu_steps.sh \
  "c5grid|400|C5P_VARIANTS='default;MN_BF16_SAMPLE_DIV=24,MN_BF16_L1=12;MN_BF16_SAMPLE_DIV=32,MN_BF16_L1=8;MN_BF16_SAMPLE_DIV=32,MN_BF16_L1=12;MN_BF16_SAMPLE_DIV=24,MN_BF16_L1=16' python -u scripts/c5_probe.py"
