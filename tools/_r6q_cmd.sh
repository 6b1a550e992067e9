cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6q
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_steps.sh \
 "400|${T}_hs32|$PT tests/test_gpu_kernels.py -k 'hs32 or attention_fwd_bwd'" \
 "400|${T}_attn|for v in base nb0 nbnoatom new; do echo == \$v; lib=''; [ \$v != new ] && lib=MMT_LIB_PATH=ab_variants/\$v/libmmt_hip.so; env \$lib python -u tools/attn_bench.py --shapes c1 --rings 79 2>&1 | grep -v amdgpu.ids; done"
