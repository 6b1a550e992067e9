# A/B of GEMM pipeline variants (bench --gemm-variant V; V sets the forward/backward-data and the
# weight-gradient variants alike unless V >= 16), alternating on one box.
# usage: VARS="0 5 6" CFGS="c1 target" REPS=2 bash tools/gpu_ab_variant.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in ${CFGS:-c1}; do for rep in $(seq ${REPS:-2}); do for v in ${VARS:-0 5}; do
  steps=100; [ $cfg = target ] && steps=20; [ $cfg = c4 ] && steps=4; [ $cfg = c3 ] && steps=8
  timeout -k 10 240 python -u bench.py --config $cfg --steps $steps --warmup 5 --no-cpu-baseline --exact-steps 0 --gemm-variant $v --probe "${PROBES:-ffn0,ffn2_dx,*_dw}" 2>/dev/null | tail -1 > gpurun_out/abv_${cfg}_${v}_${rep}.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abv_${cfg}_${v}_${rep}.json')); print('$cfg v$v $rep', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']], flush=True)"
done; done; done
