#!/bin/bash
# energy signals with batched row gathers: energy tests + item-graph signals timing
cd /root/repo
bash scripts/gpu_steps.sh \
  "etests|300|python -u -m pytest tests/test_energy_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "eab5|300|EAB_VARIANTS='default' EAB_SIGNALS=1 python -u scripts/energy_ab.py"
