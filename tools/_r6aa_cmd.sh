cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6aa
B="--no-cpu-baseline --exact-steps 0 --serial-steps 0 --probe-steps 1"
bash tools/gpu_steps.sh \
 "400|${T}_pytest_mask|python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_model.py -q -x -k 'mask or dropout or twice' --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "300|${T}_prof_c3|rocprofv3 --kernel-trace -d gpurun_out/${T}_prof_c3 -o run -- python3 bench.py --config c3 --steps 3 --warmup 2 $B" \
 "300|${T}_prof_c3m|MMT_MASK_AHEAD=1 rocprofv3 --kernel-trace -d gpurun_out/${T}_prof_c3m -o run -- python3 bench.py --config c3 --steps 3 --warmup 2 $B" \
 && for d in prof_c3 prof_c3m; do db=$(ls gpurun_out/${T}_$d/*.db | head -1); \
   python3 tools/launches.py $db gemm8_kernel --back 1 > gpurun_out/${T}_${d}_gemm8.txt; \
   python3 tools/launches.py $db attn_mask --back 1 > gpurun_out/${T}_${d}_mask.txt; \
   python3 tools/launches.py $db x --all --back 1 > gpurun_out/${T}_${d}_all.txt; \
   python3 tools/timeline.py $db 3 > gpurun_out/${T}_${d}_timeline.txt; gzip -f $db; done \
 && CFGS="c3 c1 target" ENVS="|MMT_MASK_AHEAD=1|MMT_MASK_G=1" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && CFGS="c3 c1 target" ENVS="MMT_MASK_G=1|MMT_MASK_AHEAD=1|" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
