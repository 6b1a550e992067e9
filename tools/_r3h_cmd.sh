cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3h_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'attention' -q --timeout 120 --timeout-method thread" \
 "300|r3h_attn|python -u tools/attn_bench.py --shapes target,c3,c3_ca,c4 --rings 19,3,11" \
 "600|r3h_ab|CFGS='c3 target' ENVS='|MMT_ATTN_RING=19||MMT_ATTN_RING=19' bash tools/gpu_ab_env.sh"
