"""GEMM microbenchmark over the C1 shapes of the training step, per pipeline variant.

    python tools/gemm_bench.py [--variants 0,1,2,3,4] [--reps 20]

Times mmt_op_gemm (the engine's kernel) with HIP events on the current stream; prints TFLOP/s.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))

import torch  # noqa: E402

import mmt_lib as ML  # noqa: E402

R = 65536  # 4 modalities x B 64 x T 256
SHAPES = [
    # name, a_kc, b_kc, epi, M, N, K, splits
    ("ffn0_fwd", 1, 1, "bias_relu_bf16", R, 1024, 256, 1),
    ("ffn0_store", 1, 1, "store_bf16", R, 1024, 256, 1),
    ("ffn0_loop_only", 1, 1, "store_bf16", R, 1024, 256, -1),
    ("ffn0_epi_only", 1, 1, "store_bf16", R, 1024, 0, 1),
    ("ffn2dx_loop_only", 1, 0, "drelu_bf16", R, 1024, 256, -1),
    ("ffn2dx_epi_only", 1, 0, "drelu_bf16", R, 1024, 0, 1),
    ("ffn0_f32", 1, 1, "store_f32", R, 1024, 256, 1),
    ("qkv1_store", 1, 1, "store_bf16", R, 384, 256, 1),
    ("ffn2_fwd", 1, 1, "bias_resid_f32", R, 256, 1024, 1),
    ("qkv1_fwd", 1, 1, "bias_tanh_bf16", R, 384, 256, 1),
    ("proj2_fwd", 1, 1, "bias_resid_f32", R, 256, 128, 1),
    ("ffn2_dx", 1, 0, "drelu_bf16", R, 1024, 256, 1),
    ("ffn2_dx_noaux", 1, 0, "store_bf16", R, 1024, 256, 1),
    ("ffn0_dx", 1, 0, "store_f32", R, 256, 1024, 1),
    ("ffn_dw_s32", 0, 0, "atomic_f32", 1024, 256, R, 32),
    ("ffn_dw_s16", 0, 0, "atomic_f32", 1024, 256, R, 16),
    ("qkv1_dw_s32", 0, 0, "atomic_f32", 384, 256, R, 32),
    # per-modality weight grads (K = B*T = 16384), the engine groups 4 of these per launch
    ("ffn_dw16k_s8", 0, 0, "atomic_f32", 1024, 256, 16384, 8),
    ("ffn_dw16k_s16", 0, 0, "atomic_f32", 1024, 256, 16384, 16),
    ("ffn_dw16k_s32", 0, 0, "atomic_f32", 1024, 256, 16384, 32),
    ("proj_dw16k_s8", 0, 0, "atomic_f32", 128, 256, 16384, 8),
    ("proj_dw16k_s32", 0, 0, "atomic_f32", 128, 256, 16384, 32),
    ("proj_dw16k_s64", 0, 0, "atomic_f32", 128, 256, 16384, 64),
    ("ca_dw16k_s8", 0, 0, "atomic_f32", 256, 256, 16384, 8),
    ("ca_dw16k_s32", 0, 0, "atomic_f32", 256, 256, 16384, 32),
    ("ca_dw16k_s64", 0, 0, "atomic_f32", 256, 256, 16384, 64),
    # main-loop rate without atomics: one block per output tile over the whole K
    ("ffn_dw16k_s1_store", 0, 0, "store_f32", 1024, 256, 16384, 1),
    ("ffn_dw16k_s1_atomic", 0, 0, "atomic_f32", 1024, 256, 16384, 1),
    ("ffn_dw2k_s1_store", 0, 0, "store_f32", 1024, 256, 2048, 1),
    ("ffn_dw2k_s1_atomic", 0, 0, "atomic_f32", 1024, 256, 2048, 1),
    # per-CU main-loop rate: one block per output tile over a long K (16 or 64 blocks)
    ("rate_1k_16k_s1", 0, 0, "store_f32", 1024, 1024, 16384, 1),
    ("rate_1k_16k_kc", 1, 1, "store_f32", 1024, 1024, 16384, 1),
    # MFMA-bound shapes (256x256 tile): target / C4 FFN and a square reference
    ("tgt_ffn0_fwd", 1, 1, "bias_relu_bf16", R, 2048, 512, 1),
    ("tgt_ffn2_dx", 1, 0, "drelu_bf16", R, 2048, 512, 1),
    ("tgt_qkv1_fwd", 1, 1, "bias_tanh_bf16", R, 768, 512, 1),
    ("tgt_proj_dx", 1, 0, "dtanh_bf16", R, 512, 512, 1),
    ("tgt_qkv1_dx", 1, 0, "store_f32", R, 512, 768, 1),
    ("tgt_ffn0_epi_only", 1, 1, "bias_relu_bf16", R, 2048, 0, 1),
    ("tgt_ffn2dx_epi_only", 1, 0, "drelu_bf16", R, 2048, 0, 1),
    ("tgt_ffn2_fwd", 1, 1, "bias_resid_f32", R, 512, 2048, 1),
    ("c3_cakv_fwd", 1, 1, "store_bf16", 2 * R, 1024, 512, 1),
    ("c3_cakv_dx", 1, 0, "acc_f32", 2 * R, 512, 1024, 1),
    ("c4_ffn0_fwd", 1, 1, "bias_relu_bf16", R, 4096, 1024, 1),
    ("c4_ffn0_store", 1, 1, "store_bf16", R, 4096, 1024, 1),
    ("c4_ffn2_dx", 1, 0, "drelu_bf16", R, 4096, 1024, 1),
    ("c4_ffn2_fwd", 1, 1, "bias_resid_f32", R, 1024, 4096, 1),
    ("c4_ffn_dw", 0, 0, "store_f32", 4096, 1024, 16384, 1),
    ("sq4k_store", 1, 1, "store_bf16", 4096, 4096, 4096, 1),
    ("sq8k_store", 1, 1, "store_bf16", 8192, 8192, 8192, 1),
]
if os.environ.get("GEMM_BENCH_ONLY"):
    SHAPES = [s for s in SHAPES if any(k in s[0] for k in os.environ["GEMM_BENCH_ONLY"].split(","))]


def r8(x):
    return (x + 7) // 8 * 8


def run(variant, reps):
    L = ML.lib()
    assert L.mmt_gemm_set_variant(variant if variant < 0 else variant | ((variant if variant <= 6 else 0) << 4)) == 0
    out = {}
    for name, akc, bkc, epi, M, N, K, splits in SHAPES:
        if akc:
            A = torch.randn(M, r8(K), device="cuda").to(torch.bfloat16)
            lda = r8(K)
        else:
            A = torch.randn(K, r8(M), device="cuda").to(torch.bfloat16)
            lda = r8(M)
        if bkc:
            B = torch.randn(N, r8(K), device="cuda").to(torch.bfloat16)
            ldb = r8(K)
        else:
            B = torch.randn(K, r8(N), device="cuda").to(torch.bfloat16)
            ldb = r8(N)
        bias = torch.randn(N, device="cuda")
        aux = torch.randn(M, r8(N), device="cuda").to(torch.bfloat16)
        resid = torch.randn(M, N, device="cuda")
        o32 = torch.zeros(M, N, device="cuda")
        o16 = torch.zeros(M, r8(N), dtype=torch.bfloat16, device="cuda")
        s = ML.stream_ptr()

        alpha = -12345.0 if splits < 0 else 1.0  # splits -1: main loop only (debug build knob)
        sp = max(1, splits)

        def call():
            rc = L.mmt_op_gemm(s, akc, bkc, ML.EPI[epi], sp, M, N, K, ML.ptr(A), lda, ML.ptr(B), ldb, ML.ptr(bias),
                               ML.ptr(aux), r8(N), ML.ptr(resid), N, ML.ptr(o32), N, ML.ptr(o16), r8(N), alpha)
            assert rc == 0

        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        tf = 2.0 * M * N * max(K, 1) / (us * 1e-6) / 1e12
        out[name] = (us, tf)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="-1,0,6")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    for v in [int(x, 0) for x in args.variants.split(",")]:
        res = run(v, args.reps)
        for k, (us, tf) in res.items():
            print(f"variant {v}: {k:22s} {us:8.1f} us {tf:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
