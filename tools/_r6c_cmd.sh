cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "120|r6c_probe|python -u tools/probe_shapes.py 24,3 40,5 72,3 48,6 24,1 32,4" \
 "300|r6c_attn|for v in base f32br f32sel f32skip; do echo == \$v; MMT_LIB_PATH=ab_variants/\$v/libmmt_hip.so python -u tools/attn_bench.py --shapes c1 --rings 15,79 --reps 20 --rounds 2; done; echo == new; python -u tools/attn_bench.py --shapes c1 --rings 15,79 --reps 20 --rounds 2" \
 "300|r6c_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'hs32_backward_variants or attention_fwd_bwd or embedding' -x -q --timeout 120 --timeout-method thread" \
 "400|r6c_model|python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_model.py tests/test_gpu_scale.py -x -q -k 'not full_size' --timeout 200 --timeout-method thread"
