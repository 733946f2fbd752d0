set -o pipefail
mkdir -p gpurun_out
AB_WORK=c3 AB_LIBS="matternet-rs_amd/libmatternet_hip_tuning_A.so;matternet-rs_amd/libmatternet_hip.so;matternet-rs_amd/libmatternet_hip_tuning_A.so|MN_COS_PF=2" timeout -k 10 300 python -u scripts/ab_libs.py 1000000 768 3 > gpurun_out/c3_ab_vm.log 2>&1
