cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3k_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'attention' -q --timeout 120 --timeout-method thread" \
 "300|r3k_model|python -u -m pytest tests/test_gpu_model.py tests/test_gpu_scale.py -q -x --timeout 120 --timeout-method thread" \
 "600|r3k_ab|CFGS='c1' ENVS='|MMT_LIB_PATH=build_variants/kt0/libmmt_hip.so||MMT_LIB_PATH=build_variants/kt0/libmmt_hip.so||MMT_LIB_PATH=build_variants/kt0/libmmt_hip.so' bash tools/gpu_ab_env.sh"
