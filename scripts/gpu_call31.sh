#!/bin/bash
# r03 closing evidence: full GPU suite, bench line, legs profile
cd /root/repo
bash scripts/gpu_steps.sh \
  "tests|700|python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread" \
  "bench|400|python -u bench.py" \
  "legs|900|bash scripts/profile_legs.sh r03d"
