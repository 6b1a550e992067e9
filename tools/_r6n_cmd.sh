cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6n
A1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
A2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="python3 bench.py --config target --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
S=()
for rb in 0 1; do
  S+=("150|${T}_rb${rb}_sq1|MMT_SIDE_STREAM=0 MMT_RELU_BITS=$rb timeout -s KILL 140 rocprofv3 --pmc $A1 --output-format csv -d gpurun_out/${T}_rb${rb}_sq1 -o run -- $B")
  S+=("150|${T}_rb${rb}_sq2|MMT_SIDE_STREAM=0 MMT_RELU_BITS=$rb timeout -s KILL 140 rocprofv3 --pmc $A2 --output-format csv -d gpurun_out/${T}_rb${rb}_sq2 -o run -- $B")
  S+=("150|${T}_rb${rb}_fetch|MMT_SIDE_STREAM=0 MMT_RELU_BITS=$rb timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_rb${rb}_fetch -o run -- $B")
  S+=("150|${T}_rb${rb}_write|MMT_SIDE_STREAM=0 MMT_RELU_BITS=$rb timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_rb${rb}_write -o run -- $B")
done
C="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
S+=("150|${T}_c1_sq1|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc $A1 --output-format csv -d gpurun_out/${T}_c1_sq1 -o run -- $C")
S+=("150|${T}_c1_sq2|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc $A2 --output-format csv -d gpurun_out/${T}_c1_sq2 -o run -- $C")
S+=("150|${T}_c1_fetch|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_c1_fetch -o run -- $C")
S+=("150|${T}_c1_write|MMT_SIDE_STREAM=0 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_c1_write -o run -- $C")
S+=("600|${T}_ab|for rep in 1 2; do for rb in 0 1; do MMT_RELU_BITS=\$rb timeout -k 10 200 python -u bench.py --config target --steps 20 --warmup 5 --no-cpu-baseline --exact-steps 0 --probe ffn0,ffn2_dx 2>/dev/null | tail -1 > gpurun_out/${T}_ab_\${rb}_\${rep}.json || exit 1; python3 -c \"import json; d=json.load(open('gpurun_out/${T}_ab_\${rb}_\${rep}.json')); print('relu_bits=\$rb', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']], flush=True)\"; done; done")
bash tools/gpu_steps.sh "${S[@]}" || exit 1
for x in rb0 rb1 c1; do
  f=$(ls gpurun_out/${T}_${x}_sq1/*counter_collection.csv); g=$(ls gpurun_out/${T}_${x}_sq2/*counter_collection.csv)
  python3 tools/pmcsq.py $f $g > gpurun_out/${T}_${x}_sq.txt
  f=$(ls gpurun_out/${T}_${x}_fetch/*counter_collection.csv); g=$(ls gpurun_out/${T}_${x}_write/*counter_collection.csv)
  python3 tools/pmcsum.py $f $g > gpurun_out/${T}_${x}_hbm.txt
done
find gpurun_out -path "gpurun_out/${T}_*" -name "*.csv" -exec gzip -f {} \;
du -sh gpurun_out
