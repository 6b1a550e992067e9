cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CFGS="c1 target" REPS=2 bash tools/gpu_round_ab.sh || exit 1
bash tools/gpu_steps.sh "300|prof_c1s_q|MMT_SIDE_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1s_q -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-steps 0"
