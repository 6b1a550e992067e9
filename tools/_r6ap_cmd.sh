cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ap
bash tools/gpu_steps.sh \
 "900|${T}_pytest|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "200|${T}_smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
