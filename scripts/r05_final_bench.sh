set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r05d_bench.log 2>&1
