# SQ counter passes (two runs, each within one pass's counter limits) of bench.py.
# usage: bash tools/gpu_pmc.sh <tag> [bench args...]     (outputs under gpurun_out/<tag>_pmc{1,2})
T=${1:-pmc}; shift
ARGS="${*:---steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0}"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "150|${T}_pmc1|timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/${T}_pmc1 -o run -- python3 bench.py $ARGS" \
 "150|${T}_pmc2|timeout -s KILL 140 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${T}_pmc2 -o run -- python3 bench.py $ARGS"
