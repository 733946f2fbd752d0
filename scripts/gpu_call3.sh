#!/bin/bash
# r03: K2 bucketed assembly — parity tests, V1/V2 A/B probe, kernel trace
cd /root/repo
bash scripts/gpu_steps.sh \
  "k2_tests|400|python -u -m pytest tests/test_laplacian_gpu.py tests/test_graph_gpu.py tests/test_energy_gpu.py tests/test_sparsify_gpu.py tests/test_knn_gpu.py -k 'not golden' -x -v -s --timeout 200 --timeout-method thread" \
  "lap_ab|120|python -u scripts/lap_probe.py" \
  "lap_trace|180|rocprofv3 --kernel-trace --stats -d gpurun_out/lap_prof3 -o lap -- python3 scripts/lap_probe.py" \
  "c3_full|300|python -u -m pytest tests/test_fullsize_gpu.py -k c3 -x -v -s --timeout 280 --timeout-method thread"
