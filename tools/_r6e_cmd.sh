cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r6e_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'hs32_backward_variants or attention_fwd_bwd' -x -q --timeout 120 --timeout-method thread" \
 "300|r6e_model|python -u -m pytest tests/test_gpu_model.py -k 'dropout' -x -q --timeout 200 --timeout-method thread" \
 "300|r6e_attn|for i in 1 2; do echo == v2; MMT_LIB_PATH=ab_variants/f32v2/libmmt_hip.so python -u tools/attn_bench.py --shapes c1 --rings 79 --reps 20 --rounds 3; echo == v3; python -u tools/attn_bench.py --shapes c1 --rings 79 --reps 20 --rounds 3; done"
