cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r6g_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'hs32_backward_variants or attention_fwd_bwd' -x -q --timeout 120 --timeout-method thread" \
 "300|r6g_model|python -u -m pytest tests/test_gpu_model.py tests/test_gpu_scale.py tests/test_gpu_determinism.py -x -q -k 'not full_size' --timeout 200 --timeout-method thread" \
 "300|r6g_attn|python -u tools/attn_bench.py --shapes c1,c1_ca --rings 15,79 --reps 20 --rounds 3" \
 "300|r6g_ab|VARDIR=ab_variants LIBS='base new' CFGS='c1' REPS=2 bash tools/gpu_ab_lib.sh"
