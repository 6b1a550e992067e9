cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ad
bash tools/gpu_steps.sh \
 "700|${T}_pytest|python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_scale.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider" \
 && PROBES="ffn0,ffn2_dx,*_dw" CFGS="c3 target c1" ENVS="|MMT_MASK_T2=0" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="ffn0,ffn2_dx,*_dw" CFGS="c3 target c1" ENVS="MMT_MASK_T2=0| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1 \
 && PROBES="ffn0,ffn2_dx,*_dw" CFGS="c3" ENVS="|MMT_MASK_T2=0" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab3.txt 2>&1
