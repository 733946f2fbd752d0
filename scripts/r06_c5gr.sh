# C5 group shape scan on sweep3 (same process): 4 x 8 (default), 2 x 16, 8 x 4
set -o pipefail
OUT=gpurun_out/r06_c5gr
mkdir -p $OUT
C5P_VARIANTS="${C5V:-default;MN_SYM_GR=2;MN_SYM_GR=8;default}" timeout -k 10 300 python3 scripts/c5_probe.py > $OUT/c5_gr.log 2>&1
