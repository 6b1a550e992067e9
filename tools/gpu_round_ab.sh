# GPU tests, then an A/B of build_variants/base vs the in-tree library on whole bench steps.
# usage: CFGS="c1 target" bash tools/gpu_round_ab.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh "300|t_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit 1
grep -q " passed" gpurun_out/t_pytest.log && ! grep -q "failed" gpurun_out/t_pytest.log || exit 1
LIBS="base new" CFGS="${CFGS:-c1}" REPS=${REPS:-2} timeout -k 10 900 bash tools/gpu_ab_lib.sh
