cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "200|pt_kern|MMT_GEMM_BIG_VARIANT=1 python -u -m pytest tests/test_gpu_kernels.py -x -q -k gemm --timeout 120 --timeout-method thread" \
 "200|b_off|MMT_GEMM_BIG=0 python -u bench.py --no-cpu-baseline" \
 "200|b_v0|MMT_GEMM_BIG_VARIANT=0 python -u bench.py --no-cpu-baseline" \
 "200|b_v1|MMT_GEMM_BIG_VARIANT=1 python -u bench.py --no-cpu-baseline" \
 "200|b_v2|MMT_GEMM_BIG_VARIANT=2 python -u bench.py --no-cpu-baseline" \
 "200|t_off|MMT_GEMM_BIG=0 python -u bench.py --config target --no-cpu-baseline --steps 10" \
 "200|t_v1|MMT_GEMM_BIG_VARIANT=1 python -u bench.py --config target --no-cpu-baseline --steps 10" \
 "200|t_v1k|MMT_GEMM_BIG_VARIANT=1 MMT_GEMM_BIG_KMIN=256 python -u bench.py --config target --no-cpu-baseline --steps 10" \
 "300|prof|MMT_GEMM_BIG_VARIANT=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof13 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
