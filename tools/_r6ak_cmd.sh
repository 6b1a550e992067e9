cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ak
PROBES="attn_bwd,*_dw,*_dx" CFGS="c1 target" ENVS="|MMT_WGRAD_BLOCKS=96|MMT_WGRAD_BLOCKS=160|MMT_WGRAD_BLOCKS=192" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c1 target" ENVS="MMT_WGRAD_BLOCKS=192|MMT_WGRAD_BLOCKS=160|MMT_WGRAD_BLOCKS=96| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
