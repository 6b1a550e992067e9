# GPU tests, GEMM microbenchmark (in-tree vs build_variants/base) on the given shapes, whole-step A/B.
# usage: ONLY="ffn2_dx,proj2" CFGS="c1 target" bash tools/gpu_ab_gemm.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh "300|t_pytest|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" || exit 1
grep -q " passed" gpurun_out/t_pytest.log && ! grep -q "failed" gpurun_out/t_pytest.log || exit 1
for lib in base new; do
  L=""; [ $lib = base ] && L="MMT_LIB_PATH=build_variants/base/libmmt_hip.so"
  env $L GEMM_BENCH_ONLY=${ONLY} timeout -k 10 200 python -u tools/gemm_bench.py --variants -1 --reps 30 2>&1 | grep variant | sed "s/^/$lib /" || exit 1
done
LIBS="base new" CFGS="${CFGS:-c1}" REPS=${REPS:-2} timeout -k 10 900 bash tools/gpu_ab_lib.sh
