cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
A2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
 "200|r3d_attn_prof|rocprofv3 --kernel-trace --stats -d gpurun_out/r3d_attn_prof -o run -- python3 tools/attn_bench.py --shapes target,c3,c1 --rings 1 --rounds 1 --reps 5" \
 "150|r3d_sqt1|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc $A1 --output-format csv -d gpurun_out/r3d_sqt1 -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "150|r3d_sqt2|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc $A2 --output-format csv -d gpurun_out/r3d_sqt2 -o run -- python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0" \
 "500|r3d_ab|CFGS='target c1' ENVS='|MMT_WGRAD_BLOCKS=256|MMT_WGRAD_BLOCKS=192||MMT_WGRAD_BLOCKS=256|MMT_WGRAD_BLOCKS=192' bash tools/gpu_ab_env.sh"
