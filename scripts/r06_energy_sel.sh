# K3 median tau: the two-row histogram select (MN_ENERGY_SEL=1, default) against
# round 5's single-row select (MN_ENERGY_SEL=2), after the energy parity tests
set -o pipefail
mkdir -p gpurun_out/r06_energy
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_energy_gpu.py > gpurun_out/r06_energy/tests.log 2>&1 &&
EAB_VARIANTS="default;MN_ENERGY_SEL=2;default;MN_ENERGY_SEL=2" timeout -k 10 300 python -u scripts/energy_ab.py > gpurun_out/r06_energy/sel_ab.log 2>&1
