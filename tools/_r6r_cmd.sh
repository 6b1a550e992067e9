cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6r
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
PR="rocprofv3 --kernel-trace --stats -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
bash tools/gpu_steps.sh \
 "400|${T}_mlp2|$PT tests/test_gpu_kernels.py -k 'mlp2'" \
 "300|${T}_model|MMT_MLP2_BM=64 $PT tests/test_gpu_model.py" \
 "300|${T}_prof_bm128|MMT_SIDE_STREAM=0 MMT_MLP2_BM=128 ${PR/-o run/-d gpurun_out/${T}_prof_bm128 -o run}" \
 "300|${T}_prof_bm64|MMT_SIDE_STREAM=0 MMT_MLP2_BM=64 ${PR/-o run/-d gpurun_out/${T}_prof_bm64 -o run}" \
 "600|${T}_ab|for rep in 1 2; do for v in 128 64; do MMT_MLP2_BM=\$v timeout -k 10 120 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --exact-steps 0 2>/dev/null | tail -1 > gpurun_out/${T}_ab_\${v}_\${rep}.json || exit 1; python3 -c \"import json; d=json.load(open('gpurun_out/${T}_ab_\${v}_\${rep}.json')); print('bm=\$v', d['ms_per_step'], flush=True)\"; done; done" \
 && bash tools/prof_post.sh $T && for v in bm128 bm64; do grep -E "per step|mlp2" gpurun_out/${T}_prof_${v}_summary.txt | head -3; done
