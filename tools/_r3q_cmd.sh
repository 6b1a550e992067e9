cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_prof_r3.sh r3p 2 && bash tools/gpu_steps.sh \
 "600|r3q_ab|CFGS='c1 target' ENVS='|MMT_SIDE_CUS=64|MMT_SIDE_CUS=128||MMT_SIDE_CUS=64|MMT_SIDE_CUS=128' bash tools/gpu_ab_env.sh"
