cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6end
B="--no-cpu-baseline --exact-steps 0 --serial-steps 0"
bash tools/gpu_steps.sh \
 "180|${T}_pmc_fetch|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 $B" \
 "180|${T}_pmc_write|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 $B" \
 "180|${T}_pmc_fetch_t|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc_fetch_t -o run -- python3 bench.py --config target --steps 2 --warmup 1 $B" \
 "180|${T}_pmc_write_t|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc_write_t -o run -- python3 bench.py --config target --steps 2 --warmup 1 $B" \
 "180|${T}_pmc_fetch_c3|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc_fetch_c3 -o run -- python3 bench.py --config c3 --steps 1 --warmup 1 $B" \
 "180|${T}_pmc_write_c3|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc_write_c3 -o run -- python3 bench.py --config c3 --steps 1 --warmup 1 $B" \
 "180|${T}_pmc_fetch_c4|timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_pmc_fetch_c4 -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 $B" \
 "180|${T}_pmc_write_c4|timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_pmc_write_c4 -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 $B" \
 "150|${T}_sq_c1_pmc1|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/${T}_sq_c1_pmc1 -o run -- python3 bench.py --steps 2 --warmup 1 $B" \
 "150|${T}_sq_c1_pmc2|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_sq_c1_pmc2 -o run -- python3 bench.py --steps 2 --warmup 1 $B" \
 "150|${T}_sq_t_pmc1|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/${T}_sq_t_pmc1 -o run -- python3 bench.py --config target --steps 2 --warmup 1 $B" \
 "150|${T}_sq_t_pmc2|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_sq_t_pmc2 -o run -- python3 bench.py --config target --steps 2 --warmup 1 $B" \
 && bash tools/prof_post.sh $T
