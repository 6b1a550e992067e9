cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "600|r3b_pytest|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "300|r3b_bench_c1|python -u bench.py" \
 "200|r3b_bench_target|python -u bench.py --config target --no-cpu-baseline --steps 20" \
 "200|r3b_attn|python -u tools/attn_bench.py --shapes target,c3,c4 --rings 0,1,3"
