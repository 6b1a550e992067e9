# A/B of environment settings on the bench's live probes (same library).
# usage: CFGS="c1" ENVS="A=1|A=2 B=3|" bash tools/gpu_ab_env.sh      ("|"-separated; empty = no extra env)
cd $GRAFT_REPO_ROOT
IFS='|' read -ra LIST <<< "${ENVS}"
for cfg in ${CFGS:-c1}; do for e in "${LIST[@]}"; do
  steps=30; [ $cfg = c4 ] && steps=4; [ $cfg = c3 ] && steps=8
  tag=$(echo "$e" | tr ' =/.' '_-__'); [ -z "$tag" ] && tag=default
  timeout -k 10 200 env $e python -u bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline --exact-steps 0 --probe "${PROBES:-attn_fwd,attn_bwd,*_dw}" 2>/dev/null | tail -1 > gpurun_out/abe_${cfg}_${tag}.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abe_${cfg}_${tag}.json')); print('$cfg [$e]', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']])"
done; done
