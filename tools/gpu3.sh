cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "300|pytest_new|python -u -m pytest tests/test_gpu_train_utils.py tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread" \
 "300|bench|python -u bench.py --cpu-seconds 5"
