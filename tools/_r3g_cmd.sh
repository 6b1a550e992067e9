cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3g_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'attention' -q --timeout 120 --timeout-method thread" \
 "600|r3g_pytest|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
 "200|r3g_attn|python -u tools/attn_bench.py --shapes target,c3,c4 --rings 1,3" \
 "600|r3g_ab|CFGS='target c3' ENVS='|MMT_ATTN_RING=1||MMT_ATTN_RING=1' bash tools/gpu_ab_env.sh"
