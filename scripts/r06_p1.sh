# Round 6: the phase-1 sample sweeps on gram_sweep3's query-major mode, and the
# two-row energy select: parity tests, then same-process A/Bs
set -o pipefail
OUT=gpurun_out/r06_p1
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_energy_gpu.py > $OUT/energy_tests.log 2>&1 &&
EAB_VARIANTS="default;MN_ENERGY_SEL=2;default;MN_ENERGY_SEL=2" timeout -k 10 300 python -u scripts/energy_ab.py > $OUT/energy_sel_ab.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_knn_gpu.py tests/test_knn_bf16_gpu.py tests/test_fullsize_gpu.py > $OUT/knn_tests.log 2>&1 &&
AB_ENVS="MN_P1_SWEEP3=1;MN_P1_SWEEP3=0" timeout -k 10 300 python3 scripts/ab_sweep.py 1000000 768 2 > $OUT/c2_p1_ab.log 2>&1 &&
C5P_VARIANTS="default;MN_P1_SWEEP3=0;default" timeout -k 10 300 python3 scripts/c5_probe.py > $OUT/c5_p1_ab.log 2>&1
