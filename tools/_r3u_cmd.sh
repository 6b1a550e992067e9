cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "600|r3u_pytest|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
 "300|r3u_attn|python -u tools/attn_bench.py --shapes target,c3,c3_ca,c4 --rings 3,7,35" \
 "600|r3u_ab|CFGS='target c3' ENVS='|MMT_ATTN_RING=7|MMT_ATTN_RING=35|MMT_LN_FUSE_FWD=0' bash tools/gpu_ab_env.sh"
