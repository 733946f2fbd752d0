# K1: the MFMA window without s_setprio (MN_SWEEP=8) vs the default, same process
set -o pipefail
OUT=gpurun_out/r06_prio
mkdir -p $OUT
AB_ENVS="MN_SWEEP=4;MN_SWEEP=8;MN_SWEEP=4;MN_SWEEP=8" AB_PROBES="" timeout -k 10 300 python3 scripts/ab_sweep.py 1000000 768 1 > $OUT/c2_prio.log 2>&1
