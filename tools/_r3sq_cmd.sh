cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export MMT_SIDE_STREAM=0
A1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
A2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
 "150|r3sq_c1a|timeout -s KILL 140 rocprofv3 --pmc $A1 --output-format csv -d gpurun_out/r3sq_c1a -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "150|r3sq_c1b|timeout -s KILL 140 rocprofv3 --pmc $A2 --output-format csv -d gpurun_out/r3sq_c1b -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "150|r3sq_ta|timeout -s KILL 140 rocprofv3 --pmc $A1 --output-format csv -d gpurun_out/r3sq_ta -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "150|r3sq_tb|timeout -s KILL 140 rocprofv3 --pmc $A2 --output-format csv -d gpurun_out/r3sq_tb -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0"
