# A/B of library builds on whole bench steps (alternating runs on one box).
# usage: LIBS="base new" CFGS="c1 target" REPS=2 bash tools/gpu_ab_lib.sh
#   a LIBS entry is a build_variants/<name> directory, or "new" for the in-tree library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${CFGS:-c1}; do for rep in $(seq ${REPS:-2}); do for v in ${LIBS:-base new}; do
  steps=100; [ $cfg = target ] && steps=20; [ $cfg = c4 ] && steps=4; [ $cfg = c3 ] && steps=8
  lib=""; [ $v != new ] && lib="MMT_LIB_PATH=${VARDIR:-build_variants}/$v/libmmt_hip.so"
  timeout -k 10 240 env $lib python -u bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline --exact-steps 0 --probe "${PROBES:-attn_fwd,attn_bwd,*_dw}" 2>/dev/null | tail -1 > gpurun_out/abl_${cfg}_${v}_${rep}.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abl_${cfg}_${v}_${rep}.json')); print('$cfg $v $rep', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']], flush=True)"
done; done; done
