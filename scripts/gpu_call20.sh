#!/bin/bash
cd /root/repo
bash scripts/gpu_steps.sh \
  "tests|700|python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread" \
  "bench|300|python -u bench.py"
