cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline" \
 "300|prof_ts|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ts -o run -- python3 bench.py --config target --steps 10 --warmup 3 --no-cpu-baseline"
