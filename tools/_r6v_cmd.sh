cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6v
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
PR="rocprofv3 --kernel-trace --stats -o run -- python3 bench.py --config target --steps 6 --warmup 2 --no-cpu-baseline --exact-steps 0 --serial-steps 0"
bash tools/gpu_steps.sh \
 "300|${T}_det|$PT tests/test_gpu_determinism.py -s -k 'hs64 or qkv2'" \
 "600|${T}_model|$PT tests/test_gpu_model.py tests/test_gpu_scale.py -k 'not full_size'" \
 "300|${T}_kern|$PT tests/test_gpu_kernels.py -k 'attention or qkv2'" \
 "300|${T}_prof_on|MMT_SIDE_STREAM=0 MMT_ATTN_QKV2=3 ${PR/-o run/-d gpurun_out/${T}_prof_on -o run}" \
 "300|${T}_prof_off|MMT_SIDE_STREAM=0 MMT_ATTN_QKV2=1 ${PR/-o run/-d gpurun_out/${T}_prof_off -o run}" \
 "900|${T}_ab|for cfg in target c3; do for rep in 1 2; do for v in 1 3; do st=20; [ \$cfg = c3 ] && st=6; MMT_ATTN_QKV2=\$v timeout -k 10 200 python -u bench.py --config \$cfg --steps \$st --warmup 2 --no-cpu-baseline --exact-steps 0 --serial-steps 0 --probe attn_bwd 2>/dev/null | tail -1 > gpurun_out/${T}_ab_\${cfg}_\${v}_\${rep}.json || exit 1; python3 -c \"import json; d=json.load(open('gpurun_out/${T}_ab_\${cfg}_\${v}_\${rep}.json')); print('\$cfg qkv2=\$v', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']], flush=True)\"; done; done; done" \
 && bash tools/prof_post.sh $T && for v in on off; do grep -E "per step|ring64|qkv2_bwd" gpurun_out/${T}_prof_${v}_summary.txt | head -5; done
