# A/B of library variants on the bench's live probes.
# usage: CFGS="target c1" VARIANTS="base new" TESTS=1 bash tools/gpu_ab_attn.sh
#   variant "new" = the in-tree library; any other name = build_variants/<name>/libmmt_hip.so
cd $GRAFT_REPO_ROOT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_scale.py -x -q --timeout 200 --timeout-method thread -k "attention or model or scale" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
for cfg in ${CFGS:-target c1}; do for v in ${VARIANTS:-base new}; do
  if [ $v = new ]; then unset MMT_LIB_PATH; else export MMT_LIB_PATH=build_variants/$v/libmmt_hip.so; fi
  steps=30; [ $cfg = c4 ] && steps=4; [ $cfg = c3 ] && steps=8
  timeout -k 10 200 python -u bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline --exact-steps 0 --probe "${PROBES:-attn_fwd,attn_bwd,*_dw}" 2>/dev/null | tail -1 > gpurun_out/ab_${cfg}_${v}.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_${cfg}_${v}.json')); print('$cfg $v', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']])"
done; done
