cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "600|r3c_pytest|python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread" \
 "200|r3c_gemm_v0|MMT_GEMM_BIG_VARIANT=0 GEMM_BENCH_ONLY=sq4k,c4_,rate_ python -u tools/gemm_bench.py --variants -1 --reps 10" \
 "200|r3c_gemm_v3|MMT_GEMM_BIG_VARIANT=3 GEMM_BENCH_ONLY=sq4k,c4_,rate_ python -u tools/gemm_bench.py --variants -1 --reps 10" \
 "200|r3c_gemm_v4|MMT_GEMM_BIG_VARIANT=4 GEMM_BENCH_ONLY=sq4k,c4_,rate_ python -u tools/gemm_bench.py --variants -1 --reps 10" \
 "200|r3c_gemm_t0|MMT_GEMM_BIG_KMIN=512 MMT_GEMM_BIG_VARIANT=0 GEMM_BENCH_ONLY=tgt_ python -u tools/gemm_bench.py --variants -1 --reps 10" \
 "200|r3c_gemm_t3|MMT_GEMM_BIG_KMIN=512 MMT_GEMM_BIG_VARIANT=3 GEMM_BENCH_ONLY=tgt_ python -u tools/gemm_bench.py --variants -1 --reps 10" \
 "200|r3c_gemm_ts|GEMM_BENCH_ONLY=tgt_ python -u tools/gemm_bench.py --variants -1 --reps 10"
