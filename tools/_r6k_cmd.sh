cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6k
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
PR="rocprofv3 --kernel-trace --stats -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
bash tools/gpu_steps.sh \
 "400|${T}_det|$PT tests/test_gpu_determinism.py" \
 "300|${T}_prof_q2|MMT_SIDE_STREAM=0 MMT_ATTN_QKV2=1 ${PR/-o run/-d gpurun_out/${T}_prof_q2 -o run}" \
 "300|${T}_prof_noq2|MMT_SIDE_STREAM=0 MMT_ATTN_QKV2=0 ${PR/-o run/-d gpurun_out/${T}_prof_noq2 -o run}" \
 "300|${T}_prof_noatom|MMT_SIDE_STREAM=0 MMT_LIB_PATH=ab_variants/q2noatom/libmmt_hip.so ${PR/-o run/-d gpurun_out/${T}_prof_noatom -o run}" \
 && bash tools/prof_post.sh $T
