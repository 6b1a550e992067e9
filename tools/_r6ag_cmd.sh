cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ag
bash tools/gpu_steps.sh \
 "300|${T}_pytest|MMT_DW_ATTN_SMALL=1 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_determinism.py -q -x --timeout 300 --timeout-method thread -p no:cacheprovider" \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c1 target" ENVS="|MMT_DW_ATTN_SMALL=1" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c1 target" ENVS="MMT_DW_ATTN_SMALL=1| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1 \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c1" ENVS="|MMT_DW_ATTN_SMALL=1" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab3.txt 2>&1
