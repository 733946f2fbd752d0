# K1: query fragments register-direct (MN_SWEEP=7, QREG) vs the default sweep3
set -o pipefail
OUT=gpurun_out/r06_qreg
mkdir -p $OUT
AB_ENVS="MN_SWEEP=4;MN_SWEEP=7" AB_PROBES="noepi" timeout -k 10 300 python3 scripts/ab_sweep.py 1000000 768 2 > $OUT/c2_qreg_ab.log 2>&1
