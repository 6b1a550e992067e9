#!/bin/bash
# profiles/pmc_traffic.json from a round profile set's PMC passes (tools/gpu_prof_round.sh <tag>):
# per config, the probed families' HBM bytes per launch; self- and cross-attention rows separated
# by dispatch parity (they share a kernel and alternate: forward self first, backward cross first).
# usage: bash tools/pmc_traffic_all.sh <tag>
T=${1:?tag}
for c in c1 target c3 c4; do
  case $c in c1) t="";; target) t="_t";; *) t="_$c";; esac
  F=$(ls gpurun_out/${T}_pmc_fetch$t/*counter_collection.csv*) || exit 1
  W=$(ls gpurun_out/${T}_pmc_write$t/*counter_collection.csv*) || exit 1
  # round 5: K >= 512 forward / data-gradient launches of >= 1024 tiles run the ping-pong kernel
  # (gemm8_kernel<EPI, A_KC, B_KC>), the LayerNorm-fused N = 256 launches too (C1)
  case $c in
    c1) FF="ffn0=true, true, true, 2, 3>"; DX="ffn2_dx=, 6, 1>"; LN="ln_bwd_fused=gemm8_kernel<9, true, false>";;
    c4) FF="ffn0=gemm_f8_kernel<TileCfg<2, 4, 4, 2>, 2>"; DX="ffn2_dx=gemm8_kernel<6, true, false>"; LN="";;
    *) FF="ffn0=gemm8_kernel<2, true, true>"; DX="ffn2_dx=gemm8_kernel<6, true, false>"; LN="ln_bwd_fused=, 9, 1>";;
  esac
  args=("$FF" "*_dw=false, false, true,+slab_reduce" "attn_fwd=attn_fwd@0/2" "ca_attn_fwd=attn_fwd@1/2"
        "attn_bwd=attn_bwd_dq+attn_bwd_dkdv@1/2" "ca_attn_bwd=attn_bwd_dq+attn_bwd_dkdv@0/2" "$DX")
  # round 6: at hs 32 (C1) the self-attention backward is one kernel (attn_bwd_fused32, Q/K/V stage 2 in
  # its epilogue); the cross-attention keeps the two passes
  [ $c = c1 ] && args=("$FF" "*_dw=false, false, true,+slab_reduce" "attn_fwd=attn_fwd@0/2" "ca_attn_fwd=attn_fwd@1/2"
        "attn_bwd=attn_bwd_fused32" "ca_attn_bwd=attn_bwd_dq+attn_bwd_dkdv" "$DX")
  [ -n "$LN" ] && args+=("$LN")
  python3 tools/pmc_traffic.py $c $F $W "${args[@]}" || exit 1
done
