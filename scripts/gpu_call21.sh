#!/bin/bash
# r03 final evidence: full GPU suite, then the per-kernel legs profile
cd /root/repo
bash scripts/gpu_steps.sh \
  "tests|700|python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread" \
  "legs|900|bash scripts/profile_legs.sh r03b"
