#!/bin/bash
# K3 v2: energy parity tests, then v1/v2 timing at the C3 shape
cd /root/repo
bash scripts/gpu_steps.sh \
  "etests|300|python -u -m pytest tests/test_energy_gpu.py tests/test_search_gpu.py tests/test_graph_gpu.py -x -v --timeout 120 --timeout-method thread" \
  "eab2|200|EAB_VARIANTS='default;MN_ENERGY_V1=1' python -u scripts/energy_ab.py"
