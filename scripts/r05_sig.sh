set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_energy_gpu.py -k "signal" > gpurun_out/sig_tests.log 2>&1 &&
SIG_VARIANTS="MN_SIG_FS=0;MN_SIG_FS=64;MN_SIG_FS=32;MN_SIG_FS=64+MN_SIG_SNE=4;MN_SIG_FS=32+MN_SIG_SNE=4" timeout -k 10 300 python -u scripts/sig_ab.py 1000000 768 3 > gpurun_out/sig_ab.log 2>&1
