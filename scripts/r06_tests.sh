#!/bin/bash
# GPU parity suite + smoke on the current tree (TAG names the logs)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r06}
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log; exit $rc
