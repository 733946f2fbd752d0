#!/bin/bash
# Run one gpurun command, waiting for a free box: retried ONLY while gpurun
# answers 3 (no box / slot free, nothing ran, nothing charged).
#   scripts/gpurun_when_free.sh <timeout_s> '<command>'
T=$1; shift
for i in $(seq 1 20); do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
    rc=$?
    [ $rc -ne 3 ] && exit $rc
    sleep 120
done
exit 3
