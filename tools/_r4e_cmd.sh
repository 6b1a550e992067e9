cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="tests/test_gpu_scale.py -k full_size -q -s --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
 "300|r4e_default|python -u -m pytest $T" \
 "300|r4e_v1|MMT_QKV2_BWD_V1=1 python -u -m pytest $T" \
 "300|r4e_ring0|MMT_ATTN_RING=0 python -u -m pytest $T" \
 "300|r4e_gemm|GEMM_BENCH_ONLY=tgt_ffn0,tgt_ffn2_dx,rate_1k,sq4k,c4_ffn0_store,ffn0_fwd,qkv1_fwd,ffn2_dx python -u tools/gemm_bench.py --variants=-1,7,8,768,1024 --reps 20" \
 "300|r4e_prof_c1|rocprofv3 --kernel-trace --stats -d gpurun_out/r4e_prof_c1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|r4e_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
