# C5 re-rank first-pass margin (k_cos_rerank_x1 m1) A/B, then the C5 parity tests
set -o pipefail
OUT=gpurun_out/r06_crr
mkdir -p $OUT
C5P_VARIANTS="MN_CRR_M1=0;MN_CRR_M1=8;MN_CRR_M1=4;MN_CRR_M1=16;MN_CRR_M1=8" timeout -k 10 300 python3 scripts/c5_probe.py > $OUT/c5_crr.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_knn_bf16_gpu.py "tests/test_fullsize_gpu.py::test_c5_1m_3072_bf16_cosine_sampled_rows" > $OUT/c5_tests.log 2>&1
