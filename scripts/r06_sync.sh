# Group soft-sync A/B (gram_sweep3.hpp SYNC): C5 then C2, same process each
set -o pipefail
OUT=gpurun_out/r06_sync
mkdir -p $OUT
C5P_VARIANTS="default;MN_SWEEP_SYNC=1;default;MN_SWEEP_SYNC=1" timeout -k 10 300 python3 scripts/c5_probe.py > $OUT/c5_sync_ab.log 2>&1 &&
AB_ENVS="MN_SWEEP_SYNC=0;MN_SWEEP_SYNC=1" timeout -k 10 300 python3 scripts/ab_sweep.py 1000000 768 2 > $OUT/c2_sync_ab.log 2>&1
