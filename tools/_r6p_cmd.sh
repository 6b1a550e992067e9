cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6p
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
PR="rocprofv3 --kernel-trace --stats -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
bash tools/gpu_steps.sh \
 "400|${T}_hs32|$PT tests/test_gpu_kernels.py -k 'hs32 or attention_fwd_bwd'" \
 "600|${T}_model|$PT tests/test_gpu_model.py tests/test_gpu_determinism.py" \
 "300|${T}_attn|for v in base new; do echo == \$v; lib=''; [ \$v != new ] && lib=MMT_LIB_PATH=ab_variants/\$v/libmmt_hip.so; env \$lib python -u tools/attn_bench.py --shapes c1 --rings 79 2>&1 | grep -v amdgpu.ids; done" \
 "300|${T}_prof|MMT_SIDE_STREAM=0 ${PR/-o run/-d gpurun_out/${T}_prof -o run}" \
 "600|${T}_ab|VARDIR=ab_variants LIBS='base new' CFGS='c1' REPS=3 PROBES=attn_bwd bash tools/gpu_ab_lib.sh" \
 && bash tools/prof_post.sh $T && grep -E "per step|fused32" gpurun_out/${T}_prof_summary.txt | head -3
