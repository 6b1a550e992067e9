cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3f_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'ln_bwd or attention' -q --timeout 120 --timeout-method thread" \
 "200|r3f_attn|python -u tools/attn_bench.py --shapes target,c3,c4 --rings 1,3 && MMT_ATTN_DQ_X2=0 python -u tools/attn_bench.py --shapes target,c3 --rings 3" \
 "600|r3f_pytest|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread"
