set -o pipefail
mkdir -p gpurun_out
AB_LIBS="matternet-rs_amd/libmatternet_hip_tuning.so;matternet-rs_amd/libmatternet_hip_tuning.so|MN_SYM_GSHAPE=4;matternet-rs_amd/libmatternet_hip_tuning.so|MN_SYM_GSHAPE=1;matternet-rs_amd/libmatternet_hip_tuning.so|MN_X1_SAMPLE_DIV=20;matternet-rs_amd/libmatternet_hip_tuning.so|MN_X1_SAMPLE_DIV=28" timeout -k 10 500 python -u scripts/ab_libs.py 1000000 768 2 > gpurun_out/r05_gshape_ab.log 2>&1
