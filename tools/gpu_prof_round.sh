cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|bench_c1|python -u bench.py" \
 "200|bench_target|python -u bench.py --config target --no-cpu-baseline --steps 10" \
 "300|prof_c1|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline" \
 "300|prof_c1_serial|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline" \
 "180|pmc_fetch|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline" \
 "180|pmc_write|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline" \
 "180|pmc_fetch_t|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_t -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline" \
 "180|pmc_write_t|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_t -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline"
