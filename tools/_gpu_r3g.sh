# config 2 (B=1): tile-plan sweeps of the slow shapes
set -o pipefail
mkdir -p gpurun_out
C3="conv3_l0_320 conv3_l3_1280 conv3_l1_640 conv3_l2_1280 conv3_up_l0_960 conv3_l3_2560 conv3_l1_in_320 conv3_l2_in_640"
G1="gemm_proj_1280_l2 gemm_proj_640 gemm_ff2_2560 gemm_proj_320 gemm_geglu_1280 gemm_ff2_5120 gemm_geglu_320 gemm_ff2_1280 gemm_geglu_640 gemm_qkv_1280 gemm_proj_1280_l3 gemm_short_l3_2560 gemm_qkv_320 gemm_qkv_640"
P="auto 128,160,1 128,160,2 128,160,4 128,160,8 64,160,1 64,160,2 64,160,4 64,160,8 64,160,16 64,64,1 64,64,2 64,64,4 64,64,8 32,64,1 32,64,4 32,64,8 32,64,16 128,128,1 128,128,4"
timeout -k 10 500 python -u tools/opbench.py --batch 1 --iters 20 --only $C3 $G1 --plans $P > gpurun_out/r3g_b1_plans.txt 2>&1 || exit 1
cat gpurun_out/r3g_b1_plans.txt | grep -v amdgpu.ids
