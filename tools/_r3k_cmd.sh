cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "600|r3k_ab|CFGS='c1' ENVS='|MMT_LIB_PATH=build_variants/kt0/libmmt_hip.so||MMT_LIB_PATH=build_variants/kt0/libmmt_hip.so||MMT_LIB_PATH=build_variants/kt0/libmmt_hip.so' bash tools/gpu_ab_env.sh"
