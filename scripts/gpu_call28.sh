#!/bin/bash
# diffusion: degree-ordered lanes + batched row loads (bit-exact tests + timing)
cd /root/repo
bash scripts/gpu_steps.sh \
  "etests|300|python -u -m pytest tests/test_energy_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread" \
  "eab4|200|EAB_VARIANTS='default' python -u scripts/energy_ab.py"
