set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_knn_cos_gpu.py tests/test_graph_gpu.py > gpurun_out/cos_tests12.log 2>&1 &&
C3_VARIANTS="default;MN_COS_GBLK=16384;MN_COS_GBLK=2048" timeout -k 10 200 python -u scripts/c3_probe.py 1000000 768 3 > gpurun_out/c3_gblk2_ab.log 2>&1
