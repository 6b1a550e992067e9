cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|pytest_dp|python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread" \
 "200|lnb256|MMT_LNB_CAP=256 rocprofv3 --kernel-trace --stats -d gpurun_out/lnb256 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
 "200|lnb512|MMT_LNB_CAP=512 rocprofv3 --kernel-trace --stats -d gpurun_out/lnb512 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline" \
 "200|lnb4096|MMT_LNB_CAP=4096 rocprofv3 --kernel-trace --stats -d gpurun_out/lnb4096 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
