cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r5d_pytest|python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k 'pipeline_variants or gemm8 or wgrad or weight_grad'" \
 "300|r5d_gemm|GEMM_BENCH_ONLY=c4_ffn_dw,ffn_dw16k_s1_store,rate_1k_16k_s1,ffn_dw16k_s8,ca_dw16k python -u tools/gemm_bench.py --variants=-1,0x30000" \
 "600|r5d_ab1|CFGS='target c1' ENVS='|MMT_GEMM8=1|MMT_GEMM8=1 MMT_GEMM_BIG_KMIN=512' bash tools/gpu_ab_env.sh" \
 "600|r5d_ab2|CFGS='target c1' ENVS='|MMT_GEMM8=1|MMT_GEMM8=1 MMT_GEMM_BIG_KMIN=512' bash tools/gpu_ab_env.sh"
