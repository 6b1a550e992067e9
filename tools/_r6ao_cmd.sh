cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ao
bash tools/gpu_steps.sh \
 "300|${T}_pytest|MMT_MASK_AHEAD=2 python -u -m pytest tests/test_gpu_model.py -q -x -k 'deep or multichunk' --timeout 300 --timeout-method thread -p no:cacheprovider" \
 && PROBES="attn_fwd,ffn0,*_dw" CFGS="c4 c3" ENVS="|MMT_MASK_AHEAD=2" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="attn_fwd,ffn0,*_dw" CFGS="c4 c3" ENVS="MMT_MASK_AHEAD=2| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
