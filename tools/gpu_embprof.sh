cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base u8 u16 u8c1 u16c1; do
  if [ $v = base ]; then L=""; else L="MMT_LIB_PATH=build_variants/$v/libmmt_hip.so"; fi
  timeout -k 10 200 env $L MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/emb_$v -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/emb_$v.log 2>&1 || exit 1
done
