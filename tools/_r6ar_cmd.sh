cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ar
bash tools/gpu_steps.sh \
 "900|${T}_pytest|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200|${T}_smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200|r6ar_bench_c3|python -u bench.py --config c3 --no-cpu-baseline --steps 10"
