# re-rank first-pass margin (k_rerank_x1 m1): 0 (round 5) vs 16 vs 32, uniform then clustered C2
set -o pipefail
OUT=gpurun_out/r06_rr
mkdir -p $OUT
AB_ENVS="${RRV:-MN_RR_M1=0;MN_RR_M1=16;MN_RR_M1=32}" AB_PROBES="" timeout -k 10 300 python3 scripts/ab_sweep.py 1000000 768 2 > $OUT/c2_rr.log 2>&1 &&
[ -n "$RRV" ] || AB_DATA=clustered AB_ENVS="MN_RR_M1=0;MN_RR_M1=16" AB_PROBES="" timeout -k 10 400 python3 scripts/ab_sweep.py 1000000 768 1 > $OUT/c2clu_rr.log 2>&1
