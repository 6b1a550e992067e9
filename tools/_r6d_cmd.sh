cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
A2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
 "200|r6d_attn|python -u tools/attn_bench.py --shapes c1 --rings 15,79 --reps 20 --rounds 3" \
 "150|r6d_sq1|timeout -s KILL 140 rocprofv3 --pmc $A1 --output-format csv -d gpurun_out/r6d_sq1 -o run -- python3 tools/attn_bench.py --shapes c1 --rings 15,79 --reps 2 --rounds 1" \
 "150|r6d_sq2|timeout -s KILL 140 rocprofv3 --pmc $A2 --output-format csv -d gpurun_out/r6d_sq2 -o run -- python3 tools/attn_bench.py --shapes c1 --rings 15,79 --reps 2 --rounds 1" \
 "150|r6d_pmc|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r6d_pmc -o run -- python3 tools/attn_bench.py --shapes c1 --rings 15,79 --reps 2 --rounds 1" \
 "150|r6d_pmcw|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r6d_pmcw -o run -- python3 tools/attn_bench.py --shapes c1 --rings 15,79 --reps 2 --rounds 1"
python3 tools/pmcsq.py gpurun_out/r6d_sq1/*/run_counter_collection.csv gpurun_out/r6d_sq2/*/run_counter_collection.csv > gpurun_out/r6d_sq.txt 2>&1 || true
