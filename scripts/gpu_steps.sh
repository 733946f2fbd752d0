#!/bin/bash
# Run GPU steps in order on the gpurun box; each "name|seconds|command" step
# gets its own time limit and log (gpurun_out/<name>.log).  A plain failure
# (tests failing) moves on to the next step; a time limit, abort or crash
# (rc 124 / 134 / 137 / 139) ends the call there (nothing else touches the GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in "$@"; do
    name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
    echo "[step $name] start $(date +%T)"
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "[step $name] rc=$rc $(date +%T)"
    tail -3 "gpurun_out/$name.log"
    case $rc in
        124|134|137|139) echo "[step $name] fatal rc=$rc: stopping"; exit $rc ;;
    esac
done
