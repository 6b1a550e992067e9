cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|prof_t0|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t0 -o run -- python3 bench.py --config target --steps 10 --warmup 3 --no-cpu-baseline --dropout 0" \
 "120|pmc_t1|timeout -s KILL 110 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_t1 -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline" \
 "120|pmc_t2|timeout -s KILL 110 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_t2 -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline"
