cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6g
bash tools/gpu_steps.sh \
 "900|${T}_pytest|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200|${T}_smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300|${T}_bench_c1|python -u bench.py" \
 "300|${T}_prof_c1|rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "300|${T}_prof_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "180|${T}_pmc_fetch|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "180|${T}_pmc_write|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "150|${T}_sq_c1_pmc1|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/${T}_sq_c1_pmc1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "150|${T}_sq_c1_pmc2|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_sq_c1_pmc2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --serial-steps 0" \
 "200|${T}_bench_target|python -u bench.py --config target --no-cpu-baseline --steps 10" \
 && bash tools/prof_post.sh $T
