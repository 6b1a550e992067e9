cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6al
PROBES="attn_bwd,*_dw,*_dx" CFGS="c3 c4 target c1" ENVS="|MMT_WGRAD_BLOCKS=96" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="attn_bwd,*_dw,*_dx" CFGS="c3 c4 target c1" ENVS="MMT_WGRAD_BLOCKS=96| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
