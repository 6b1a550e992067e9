cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu_steps.sh \
  \
 "300|r3x_gemm|GEMM_BENCH_ONLY=tgt_,ffn0_fwd,ffn2_dx,qkv1_fwd,proj2_fwd,ffn0_dx python -u tools/gemm_bench.py --variants=-1,7,8 --reps 10"
