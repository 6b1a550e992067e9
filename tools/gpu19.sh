cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|b_side|python -u bench.py --no-cpu-baseline" \
 "200|b_noside|MMT_SIDE_STREAM=0 python -u bench.py --no-cpu-baseline" \
 "200|t_side|python -u bench.py --config target --no-cpu-baseline --steps 10" \
 "200|t_noside|MMT_SIDE_STREAM=0 python -u bench.py --config target --no-cpu-baseline --steps 10"
