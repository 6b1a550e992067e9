cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "120|r6h_probe|python -u tools/probe_shapes.py 24,1,1,1 24,1,1,1,32 48,2,1,1 96,2,1,1 24,1,2,2 72,3,1,1" \
 "300|r6h_kern|python -u -m pytest tests/test_gpu_kernels.py -k 'hs32_backward_variants' -x -q --timeout 120 --timeout-method thread" \
 "400|r6h_model|python -u -m pytest tests/test_gpu_model.py tests/test_gpu_determinism.py -x -q --timeout 200 --timeout-method thread" \
 "300|r6h_drift|python -u tools/fp8_drift.py --reps 2" \
 "300|r6h_ab|VARDIR=ab_variants LIBS='base new' CFGS='c1' REPS=2 bash tools/gpu_ab_lib.sh"
