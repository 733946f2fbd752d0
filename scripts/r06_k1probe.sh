# K1 SW_SYM K-loop probes on sweep3 (timing only): K loop alone, and also
# without the DMA issue / the barriers / the fragment reads
set -o pipefail
OUT=gpurun_out/r06_k1probe
mkdir -p $OUT
AB_ENVS="MN_SWEEP=4" AB_PROBES="noepi,nodma,nobar,noread" timeout -k 10 300 python3 scripts/ab_sweep.py 1000000 768 2 > $OUT/probes.log 2>&1
