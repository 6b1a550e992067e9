# Kernel-trace A/B of library variants: per-kernel averages (rocprofv3 --kernel-trace --stats).
# usage: CFGS="target" VARIANTS="base new" bash tools/gpu_ab_prof.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-target}; do for v in ${VARIANTS:-base new}; do
  if [ $v = new ]; then unset MMT_LIB_PATH; else export MMT_LIB_PATH=build_variants/$v/libmmt_hip.so; fi
  steps=6; [ $cfg = c4 ] && steps=2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_${cfg}_${v} -o run -- python3 bench.py --config $cfg --steps $steps --warmup 1 --no-cpu-baseline --exact-steps 0 > gpurun_out/abp_${cfg}_${v}.log 2>&1 || exit 1
  python3 tools/profdb.py gpurun_out/abp_${cfg}_${v}/run_results.db $((steps+1)) 12 | sed "s/^/$cfg $v /"
done; done
