set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_energy_gpu.py > gpurun_out/energy_tests.log 2>&1 &&
EAB_VARIANTS="default;MN_ENERGY_SEL=0;default;MN_ENERGY_SEL=0" timeout -k 10 300 python -u scripts/energy_ab.py > gpurun_out/energy_sel_ab.log 2>&1
