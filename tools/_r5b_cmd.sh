cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r5c_pytest|python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k 'pipeline_variants or gemm8 or identity or embedding or wgrad'" \
 "300|r5c_gemm|GEMM_BENCH_ONLY=tgt_,c4_ffn0,sq4k,sq8k,c4_ffn_dw,ffn_dw16k_s1_store python -u tools/gemm_bench.py --variants=-1,0x10000,0x30000" \
 "400|r5c_full|python -u -m pytest tests/test_gpu_scale.py -x -v -s --timeout 300 --timeout-method thread -k full_size"
