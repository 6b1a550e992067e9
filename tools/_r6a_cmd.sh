cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r6a_det|python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_model.py -x -v -s --timeout 120 --timeout-method thread" \
 "300|r6a_bench_c1|python -u bench.py --steps 100 --warmup 10" \
 "200|r6a_attn|python -u tools/attn_bench.py --shapes c1 --rings 15 --reps 20"
