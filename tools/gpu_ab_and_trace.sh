# GPU tests, same-box A/B (build_variants/base vs in-tree) at CFGS, then a serial kernel trace of the
# in-tree library at C1 and the target shape (side stream off) for per-kernel times.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CFGS="${CFGS:-c1 target}" REPS=${REPS:-2} bash tools/gpu_round_ab.sh || exit 1
bash tools/gpu_steps.sh \
 "300|ab_c1s|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_c1s -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0" \
 "300|ab_ts|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_ts -o run -- python3 bench.py --config target --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0"
