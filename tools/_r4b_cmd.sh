cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "400|r4b_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|r4b_bench_c1|python -u bench.py --steps 50 --no-cpu-baseline --exact-steps 0" \
 "200|r4b_bench_target|python -u bench.py --config target --no-cpu-baseline --steps 10 --exact-steps 0" \
 "200|r4b_gemm|GEMM_BENCH_ONLY=tgt_,sq4k,c4_ffn0_store,ffn0_fwd,ffn2_dx python -u tools/gemm_bench.py --variants -1 --reps 20" \
 "200|r4b_gemm_big|MMT_GEMM_BIG_KMIN=256 GEMM_BENCH_ONLY=tgt_,ffn0_fwd,ffn2_dx python -u tools/gemm_bench.py --variants -1 --reps 20" \
 "300|r4b_prof_ts|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b_prof_ts -o run -- python3 bench.py --config target --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|r4b_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r4b_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
