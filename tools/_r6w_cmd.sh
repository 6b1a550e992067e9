cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6w
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
PR="rocprofv3 --kernel-trace --stats -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
bash tools/gpu_steps.sh \
 "600|${T}_model|$PT tests/test_gpu_model.py tests/test_gpu_determinism.py" \
 "300|${T}_prof_base|MMT_SIDE_STREAM=0 MMT_LIB_PATH=ab_variants/base/libmmt_hip.so ${PR/-o run/-d gpurun_out/${T}_prof_base -o run}" \
 "300|${T}_prof_new|MMT_SIDE_STREAM=0 ${PR/-o run/-d gpurun_out/${T}_prof_new -o run}" \
 "600|${T}_ab|VARDIR=ab_variants LIBS='base new' CFGS='c1' REPS=3 PROBES=attn_bwd bash tools/gpu_ab_lib.sh" \
 && bash tools/prof_post.sh $T && for v in base new; do grep -E "per step|fused32" gpurun_out/${T}_prof_${v}_summary.txt | head -2; done
