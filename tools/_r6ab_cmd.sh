cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=r6ab
bash tools/gpu_steps.sh \
 "400|${T}_pytest_mask|python -u -m pytest tests/test_gpu_determinism.py tests/test_gpu_model.py tests/test_gpu_scale.py -q -x -k 'mask or dropout or twice' --timeout 300 --timeout-method thread -p no:cacheprovider" \
 && CFGS="c3 target c1" ENVS="|MMT_MASK_G=8|MMT_MASK_AHEAD=1|MMT_MASK_AHEAD=1 MMT_MASK_G=8" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab1.txt 2>&1 \
 && CFGS="c3 target c1" ENVS="MMT_MASK_AHEAD=1 MMT_MASK_G=8|MMT_MASK_AHEAD=1|MMT_MASK_G=8|" bash tools/gpu_ab_env.sh > gpurun_out/${T}_ab2.txt 2>&1
