cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3i_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'ln_bwd or attention' -q --timeout 120 --timeout-method thread" \
 "600|r3i_ab|CFGS='c1' ENVS='|MMT_LNB_TILE=0||MMT_LNB_TILE=0' bash tools/gpu_ab_env.sh" \
 "300|r3i_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/r3i_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0"
