cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6z
bash tools/gpu_steps.sh \
 "900|${T}_ab|for rep in 1 2; do for v in base k256; do e=''; [ \$v = k256 ] && e='MMT_GEMM8_KMIN=256'; env \$e timeout -k 10 150 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --exact-steps 0 --serial-steps 0 --probe ffn0,ffn2_dx 2>/dev/null | tail -1 > gpurun_out/${T}_ab_\${v}_\${rep}.json || exit 1; python3 -c \"import json; d=json.load(open('gpurun_out/${T}_ab_\${v}_\${rep}.json')); print('c1 \$v', d['ms_per_step'], [(k['label'], k['avg_launch_us']) for k in d['kernels']], flush=True)\"; done; done"
