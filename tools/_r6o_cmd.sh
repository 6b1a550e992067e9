cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6o
PR="rocprofv3 --kernel-trace --stats -o run -- python3 bench.py --config target --steps 6 --warmup 2 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
bash tools/gpu_steps.sh \
 "300|${T}_prof_base|MMT_SIDE_STREAM=0 MMT_LIB_PATH=ab_variants/base/libmmt_hip.so ${PR/-o run/-d gpurun_out/${T}_prof_base -o run}" \
 "300|${T}_prof_occ3|MMT_SIDE_STREAM=0 MMT_LIB_PATH=ab_variants/q2occ3/libmmt_hip.so ${PR/-o run/-d gpurun_out/${T}_prof_occ3 -o run}" \
 "900|${T}_ab|VARDIR=ab_variants LIBS='base q2occ3' CFGS='target c1' REPS=2 PROBES=attn_bwd bash tools/gpu_ab_lib.sh" \
 && bash tools/prof_post.sh $T && for v in base occ3; do grep -E "per step|qkv2_bwd" gpurun_out/${T}_prof_${v}_summary.txt | head -3; done
