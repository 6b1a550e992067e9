cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3e_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'ln_bwd or layernorm or attention' -q --timeout 120 --timeout-method thread" \
 "600|r3e_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "500|r3e_ab|CFGS='c1 target' ENVS='|MMT_LN_FUSE=0||MMT_LN_FUSE=0' bash tools/gpu_ab_env.sh" \
 "200|r3e_ring|MMT_ATTN_RING_SLOTS=6 python -u tools/attn_bench.py --shapes target,c3,c4 --rings 1,3 && python -u tools/attn_bench.py --shapes target,c3,c4 --rings 1,3" \
 "300|r3e_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r3e_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0"
