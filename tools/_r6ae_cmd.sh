cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ae
bash tools/gpu_steps.sh \
 "600|${T}_pytest|python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_kernels.py -q -x -k 'f8 or fp8 or c4 or t4096 or scale' --timeout 300 --timeout-method thread -p no:cacheprovider" \
 && PROBES="ffn0,ffn2_dx,attn_fwd" CFGS="c4" ENVS="|MMT_MASK_T2=0|MMT_MASK_AHEAD=1" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="ffn0,ffn2_dx,attn_fwd" CFGS="c4" ENVS="MMT_MASK_AHEAD=1|MMT_MASK_T2=0| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
