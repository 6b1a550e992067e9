cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6an
PROBES="attn_bwd,*_dw,*_dx" CFGS="c3 target" ENVS="|MMT_WGRAD_BLOCKS=64|MMT_WGRAD_BLOCKS=80" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c3 target" ENVS="MMT_WGRAD_BLOCKS=80|MMT_WGRAD_BLOCKS=64| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1 \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c4" ENVS="|MMT_WGRAD_BLOCKS=64" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab3.txt 2>&1
