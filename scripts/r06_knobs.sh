# C2 knob scan on the round-6 kernels (same process, outputs compared)
set -o pipefail
OUT=gpurun_out/r06_knobs
mkdir -p $OUT
AB_ENVS="MN_SYM_GSHAPE=2;MN_SYM_GSHAPE=1;MN_SYM_GSHAPE=4;MN_SYM_TPB=128;MN_SYM_TPB=512;MN_X1_SAMPLE_DIV=20;MN_X1_SAMPLE_DIV=28;MN_X1_L1=10;MN_X1_L1=14" timeout -k 10 500 python3 scripts/ab_sweep.py 1000000 768 2 > $OUT/c2_knobs.log 2>&1
