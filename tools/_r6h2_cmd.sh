cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6h2
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
 "600|${T}_tests|MMT_FLUSH_HOLD=1 $PT tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_scale.py tests/test_gpu_dp.py -k 'not full_size'" \
 "900|${T}_ab|for cfg in c1 target; do for rep in 1 2; do for v in 0 1; do st=100; [ \$cfg = target ] && st=20; MMT_FLUSH_HOLD=\$v timeout -k 10 200 python -u bench.py --config \$cfg --steps \$st --warmup 5 --no-cpu-baseline --exact-steps 0 --serial-steps 0 --probe '*_dw' 2>/dev/null | tail -1 > gpurun_out/${T}_ab_\${cfg}_\${v}_\${rep}.json || exit 1; python3 -c \"import json; d=json.load(open('gpurun_out/${T}_ab_\${cfg}_\${v}_\${rep}.json')); print('\$cfg hold=\$v', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']], flush=True)\"; done; done; done"
