cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6j
bash tools/gpu_steps.sh \
 "300|${T}_prof_c1|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|${T}_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "200|${T}_bench_target|python -u bench.py --config target --no-cpu-baseline --steps 10 --exact-steps 0" && bash tools/prof_post.sh $T
