cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|r3s_kern|MMT_DW_XCD_PLANE=1 python -u -m pytest tests/test_gpu_kernels.py -k 'weight_grad or wgrad' -q --timeout 120 --timeout-method thread" \
 "180|r3s_pmc_f0|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3s_pmc_f0 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "180|r3s_pmc_f1|MMT_DW_XCD_PLANE=1 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3s_pmc_f1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "180|r3s_pmc_t0|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3s_pmc_t0 -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "180|r3s_pmc_t1|MMT_DW_XCD_PLANE=1 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3s_pmc_t1 -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "600|r3s_ab|CFGS='c1 target' ENVS='|MMT_DW_XCD_PLANE=1||MMT_DW_XCD_PLANE=1' bash tools/gpu_ab_env.sh"
