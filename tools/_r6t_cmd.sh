cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6t
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_steps.sh \
 "400|${T}_hs32|MMT_LIB_PATH=ab_variants/nb2/libmmt_hip.so $PT tests/test_gpu_kernels.py -k 'hs32 or attention_fwd_bwd'" \
 "400|${T}_model|MMT_LIB_PATH=ab_variants/nb2/libmmt_hip.so $PT tests/test_gpu_model.py tests/test_gpu_determinism.py" \
 "300|${T}_attn|for v in base nb2; do echo == \$v; MMT_LIB_PATH=ab_variants/\$v/libmmt_hip.so python -u tools/attn_bench.py --shapes c1 --rings 79 2>&1 | grep -v amdgpu.ids; done" \
 "600|${T}_ab|VARDIR=ab_variants LIBS='base nb2' CFGS='c1' REPS=3 PROBES=attn_bwd bash tools/gpu_ab_lib.sh"
