cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6af
bash tools/gpu_steps.sh \
 "900|${T}_pytest|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200|${T}_smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300|${T}_bench_c1|python -u bench.py" \
 "300|${T}_prof_c1|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|${T}_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 && for d in prof_c1 prof_c1s; do db=$(ls gpurun_out/${T}_$d/*.db | head -1); python3 tools/launches.py $db x --all --back 1 > gpurun_out/${T}_${d}_all.txt; done \
 && bash tools/prof_post.sh $T
