cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ac
bash tools/gpu_steps.sh \
 "300|${T}_pytest_t2|python -u -m pytest tests/test_gpu_kernels.py -q -x -k 't2_tile or pipeline_variants' --timeout 120 --timeout-method thread -p no:cacheprovider" \
 "200|${T}_gb0|MMT_GEMM_T2=0 GEMM_BENCH_ONLY=tgt_,c3_ python -u tools/gemm_bench.py --variants -1" \
 "200|${T}_gb1|MMT_GEMM_T2=1 GEMM_BENCH_ONLY=tgt_,c3_ python -u tools/gemm_bench.py --variants -1" \
 && PROBES="ffn0,ffn2_dx,*_dw" CFGS="target c3" ENVS="|MMT_GEMM_T2=1" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="ffn0,ffn2_dx,*_dw" CFGS="target c3 c1" ENVS="MMT_GEMM_T2=1|" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
