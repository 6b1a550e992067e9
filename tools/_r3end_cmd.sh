cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
 "600|r3end_pytest|python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
 "200|r3end_smoke|python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r3end_bench|python -u bench.py --no-cpu-baseline --steps 100"
