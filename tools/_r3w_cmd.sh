cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r3w
PMC() { echo "180|${T}_$1|timeout -s KILL 170 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/${T}_$1 -o run -- python3 bench.py $3 --no-cpu-baseline --exact-steps 0"; }
bash tools/gpu_steps.sh \
 "600|${T}_pytest|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
 "200|${T}_bench_target|python -u bench.py --config target --no-cpu-baseline --steps 20" \
 "200|${T}_bench_c3|python -u bench.py --config c3 --no-cpu-baseline --steps 10" \
 "300|${T}_bench_c4|python -u bench.py --config c4 --no-cpu-baseline --steps 6 --warmup 2" \
 "300|${T}_prof_ts|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_ts -o run -- python3 bench.py --config target --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0" \
 "300|${T}_prof_c3|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c3 -o run -- python3 bench.py --config c3 --steps 4 --warmup 2 --no-cpu-baseline --exact-steps 0" \
 "300|${T}_prof_c4|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "$(PMC pmc_fetch_t FETCH_SIZE '--config target --steps 2 --warmup 1')" \
 "$(PMC pmc_write_t WRITE_SIZE '--config target --steps 2 --warmup 1')" \
 "$(PMC pmc_fetch_c3 FETCH_SIZE '--config c3 --steps 1 --warmup 1')" \
 "$(PMC pmc_write_c3 WRITE_SIZE '--config c3 --steps 1 --warmup 1')" \
 "$(PMC pmc_fetch_c4 FETCH_SIZE '--config c4 --steps 1 --warmup 1')" \
 "$(PMC pmc_write_c4 WRITE_SIZE '--config c4 --steps 1 --warmup 1')"
