cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r6b_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'hs32_backward_variants or attention_fwd_bwd or embedding' -x -q --timeout 120 --timeout-method thread" \
 "400|r6b_model|python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_model.py tests/test_gpu_scale.py -x -q -k 'not full_size' --timeout 200 --timeout-method thread" \
 "200|r6b_attn|python -u tools/attn_bench.py --shapes c1 --rings 15,79 --reps 20" \
 "300|r6b_bench_c1|python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --exact-steps 0"
