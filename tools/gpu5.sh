cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|bench|python -u bench.py --no-cpu-baseline" \
 "200|bench256|MMT_DW_TARGET=256 python -u bench.py --no-cpu-baseline" \
 "200|bench1024|MMT_DW_TARGET=1024 python -u bench.py --no-cpu-baseline" \
 "300|prof|rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline"
