cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "600|r3t_pytest|python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread" \
 "600|r3t_ab|CFGS='c1' ENVS='|MMT_LN_FUSE_FWD=0|MMT_DW_XCD_PLANE=0||MMT_LN_FUSE_FWD=0|MMT_DW_XCD_PLANE=0' bash tools/gpu_ab_env.sh" \
 "400|r3t_abt|CFGS='target c3' ENVS='|MMT_DW_XCD_PLANE=0' bash tools/gpu_ab_env.sh" \
 "180|r3t_pmc_t|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3t_pmc_t -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0"
