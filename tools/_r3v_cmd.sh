cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "700|r3v_ab|CFGS='c3 target' ENVS='|MMT_WGRAD_BLOCKS=256|MMT_WGRAD_BLOCKS=192||MMT_WGRAD_BLOCKS=256|MMT_WGRAD_BLOCKS=192' bash tools/gpu_ab_env.sh"
