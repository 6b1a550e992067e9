cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6m
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
bash tools/gpu_steps.sh \
 "600|${T}_model|$PT tests/test_gpu_model.py" \
 "400|${T}_hs32|$PT tests/test_gpu_kernels.py -k 'hs32 or attention_fwd_bwd'" \
 "400|${T}_scale|$PT tests/test_gpu_scale.py -k 'not full_size'" \
 "500|${T}_ab|for rep in 1 2; do for v in 0 1; do MMT_ATTN_QKV2=\$v timeout -k 10 120 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --exact-steps 0 --probe attn_bwd 2>/dev/null | tail -1 > gpurun_out/${T}_ab_\${v}_\${rep}.json || exit 1; python3 -c \"import json; d=json.load(open('gpurun_out/${T}_ab_\${v}_\${rep}.json')); print('qkv2=\$v', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']], flush=True)\"; done; done"
