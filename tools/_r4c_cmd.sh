cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "400|r4c_pytest|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
 "200|r4c_bench_c1|python -u bench.py --steps 50 --no-cpu-baseline --exact-steps 0" \
 "200|r4c_bench_target|python -u bench.py --config target --no-cpu-baseline --steps 10 --exact-steps 0" \
 "250|r4c_gemm|GEMM_BENCH_ONLY=tgt_ffn0,tgt_ffn2_dx,rate_1k,sq4k,c4_ffn0_store,ffn0_fwd,qkv1_fwd,ffn2_dx python -u tools/gemm_bench.py --variants -1,7,8,768,1024 --reps 20" \
 "300|r4c_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
