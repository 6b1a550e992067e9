cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ai
bash tools/gpu_steps.sh \
 "300|${T}_pytest|python -u -m pytest tests/test_gpu_kernels.py -q -x -k 'wgrad or pipeline_variants' --timeout 120 --timeout-method thread -p no:cacheprovider" \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c1 target" ENVS="|MMT_GEMM_BIG_VARIANT=3" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c1 target" ENVS="MMT_GEMM_BIG_VARIANT=3| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
