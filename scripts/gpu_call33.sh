#!/bin/bash
# r03 final tree: full GPU suite + bench line
cd /root/repo
bash scripts/gpu_steps.sh \
  "tests|700|python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread" \
  "bench|400|python -u bench.py"
