cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
CFGS="c1" ENVS="|MMT_WGRAD_BLOCKS=96|MMT_WGRAD_BLOCKS=160|MMT_WGRAD_BLOCKS=192|MMT_LNB_CAP=512|MMT_LNB_CAP=128|MMT_GEMM_BIG_KMIN=1024|MMT_GEMM_BIG_VARIANT=1" PROBES="attn_fwd" timeout -k 10 600 bash tools/gpu_ab_env.sh || exit 1
done
CFGS="target" ENVS="|MMT_WGRAD_BLOCKS=96|MMT_WGRAD_BLOCKS=192|MMT_LNB_CAP=512|MMT_GEMM_BIG_VARIANT=1|" PROBES="attn_fwd" timeout -k 10 600 bash tools/gpu_ab_env.sh
