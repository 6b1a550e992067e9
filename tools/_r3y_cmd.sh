cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3y_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'gemm' -q --timeout 120 --timeout-method thread" \
 "600|r3y_ab|CFGS='target c3' ENVS='|MMT_GEMM_TILEM=0||MMT_GEMM_TILEM=0' bash tools/gpu_ab_env.sh"
