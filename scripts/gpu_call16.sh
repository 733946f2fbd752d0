#!/bin/bash
# r03 evidence pass: the full GPU suite, then the per-kernel rocprofv3 legs
# profile of one bench step (trace + FETCH/WRITE + SQ groups)
cd /root/repo
bash scripts/gpu_steps.sh \
  "tests|600|python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread" \
  "legs|900|bash scripts/profile_legs.sh r03"
