cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3u_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'attention' -q --timeout 120 --timeout-method thread" \
 "300|r3u_attn|python -u tools/attn_bench.py --shapes target,c3,c3_ca,c4 --rings 3,7,35" \
 "500|r3u_ab|CFGS='target c3' ENVS='|MMT_ATTN_RING=7|MMT_ATTN_RING=35' bash tools/gpu_ab_env.sh"
