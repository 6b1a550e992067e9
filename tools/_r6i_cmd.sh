cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "120|r6i_probe|python -u tools/probe_shapes.py 24,1,2,2 40,5,2,2 24,3,2,2" \
 "400|r6i_model|python -u -m pytest tests/test_gpu_model.py tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread" \
 "400|r6i_c4|python -u -m pytest tests/test_gpu_scale.py -x -q -s -k 'c4_fp8' --timeout 300 --timeout-method thread" \
 "400|r6i_dw|for i in 1 2; do for v in 0 1; do MMT_DW_SMALL=\$v timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --exact-steps 0 --serial-steps 0 --probe-steps 8 | tail -1 | python3 -c \"import json,sys; d=json.load(sys.stdin); print('dw_small', \$v, d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']])\"; done; done"
