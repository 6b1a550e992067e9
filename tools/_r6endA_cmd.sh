cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6end
bash tools/gpu_steps.sh \
 "300|${T}_bench_c1|python -u bench.py" \
 "200|${T}_bench_target|python -u bench.py --config target --no-cpu-baseline --steps 10" \
 "200|${T}_bench_c3|python -u bench.py --config c3 --no-cpu-baseline --steps 10" \
 "300|${T}_bench_c4|python -u bench.py --config c4 --no-cpu-baseline --steps 6 --warmup 2" \
 "300|${T}_prof_c1|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|${T}_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|${T}_prof_ts|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ts -o run -- python3 bench.py --config target --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|${T}_prof_c3|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c3 -o run -- python3 bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|${T}_prof_c4|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 && python3 tools/live_vs_serial.py gpurun_out/${T}_prof_c1/run_results.db gpurun_out/${T}_prof_c1s/run_results.db 30 > gpurun_out/${T}_c1_live_vs_serial.txt \
 && bash tools/prof_post.sh $T
