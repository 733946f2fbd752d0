#!/bin/bash
# K3 v2 A/B: separate tau kernel (default) vs select inside the entry-loop kernel
cd /root/repo
bash scripts/gpu_steps.sh \
  "etests|300|python -u -m pytest tests/test_energy_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "etests_tk|300|MN_ENERGY_TAU=1 python -u -m pytest tests/test_energy_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "eab3|200|EAB_VARIANTS='default;MN_ENERGY_TAU=1;MN_ENERGY_V1=1' python -u scripts/energy_ab.py"
