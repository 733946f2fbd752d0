#!/bin/bash
# K3 energy timing probes (row loads / gathers / tau select) + C5 sample grid 2
cd /root/repo
bash scripts/gpu_steps.sh \
  "eab|200|EAB_VARIANTS='default;MN_ENERGY_PROBE=16;MN_ENERGY_PROBE=32;MN_ENERGY_PROBE=48;MN_TAU_SEL=1;MN_ENERGY_ROWS=4' python -u scripts/energy_ab.py" \
  "c5grid2|400|C5P_VARIANTS='default;MN_BF16_SAMPLE_DIV=32,MN_BF16_L1=16;MN_BF16_SAMPLE_DIV=48,MN_BF16_L1=16;MN_BF16_SAMPLE_DIV=64,MN_BF16_L1=16;MN_BF16_SAMPLE_DIV=48,MN_BF16_L1=24' python -u scripts/c5_probe.py"
