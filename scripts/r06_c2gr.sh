# C2 group shape scan on sweep3 (same process): 2 x 16 (default), 8 x 4, 16 x 2
set -o pipefail
OUT=gpurun_out/r06_c2gr
mkdir -p $OUT
AB_ENVS="MN_SYM_GSHAPE=2;MN_SYM_GSHAPE=8;MN_SYM_GSHAPE=16" AB_PROBES="" timeout -k 10 300 python3 scripts/ab_sweep.py 1000000 768 2 > $OUT/c2_gr.log 2>&1
