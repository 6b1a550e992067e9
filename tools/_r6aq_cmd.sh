cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6aq
bash tools/gpu_steps.sh \
 "300|${T}_pytest|python -u -m pytest tests/test_gpu_determinism.py -q -x -k 'mask' --timeout 300 --timeout-method thread -p no:cacheprovider" \
 && PROBES="attn_fwd,ffn0,*_dw" CFGS="c3 c4 c1" ENVS="|MMT_MASK_G=16" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && PROBES="attn_fwd,ffn0,*_dw" CFGS="c3 c4 c1" ENVS="MMT_MASK_G=16| " bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
