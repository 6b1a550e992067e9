cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3r_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'ln_bwd' -q --timeout 120 --timeout-method thread && MMT_LNB_W_BK=64 python -u -m pytest tests/test_gpu_kernels.py -k 'ln_bwd' -q --timeout 120 --timeout-method thread" \
 "600|r3r_ab|CFGS='target c3' ENVS='|MMT_LNB_W_BK=64||MMT_LNB_W_BK=64' bash tools/gpu_ab_env.sh"
