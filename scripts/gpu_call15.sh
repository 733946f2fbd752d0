#!/bin/bash
cd /root/repo
bash scripts/gpu_steps.sh \
  "grid|500|AB_ENVS='MN_X1_SAMPLE_DIV=32,MN_X1_L1=8;MN_X1_SAMPLE_DIV=32,MN_X1_L1=6;MN_X1_SAMPLE_DIV=32,MN_X1_L1=10;MN_X1_SAMPLE_DIV=48,MN_X1_L1=6;MN_X1_SAMPLE_DIV=24,MN_X1_L1=8' AB_PROBES= python -u scripts/ab_sweep.py 1000000 768 2" \
  "tests|600|python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread" \
  "lap|120|python -u scripts/lap_probe.py" \
  "bench|300|python -u bench.py"
