cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6y
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
 "600|${T}_tests|$PT tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_scale.py -k 'not full_size'" \
 "300|${T}_kern|$PT tests/test_gpu_kernels.py -k mlp2" \
 "900|${T}_ab|VARDIR=ab_variants LIBS='base new' CFGS='c1 target' REPS=2 PROBES=attn_bwd bash tools/gpu_ab_lib.sh"
