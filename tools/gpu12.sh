cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|pt_kern|python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread" \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|bench|python -u bench.py --no-cpu-baseline" \
 "200|bench_t|python -u bench.py --config target --no-cpu-baseline --steps 10" \
 "300|prof|rocprofv3 --kernel-trace --stats -d gpurun_out/prof12 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
