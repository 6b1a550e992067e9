"""hipBLASLt (torch.matmul) reference rates on the training step's GEMM shapes, beside this build's kernel.

    python tools/blas_ref.py [--reps 20]

The library GEMM is not used by the product; its rate at the same shapes says how far the hand-written
kernel sits from what the vendor library reaches on this chip (the north-star bar is 40 % of the dense
bf16 peak, 2.5 PFLOP/s). Shapes are the grouped launches of the target (d512 / T512, B 32, 4 modalities:
R = 65,536 rows), C1 and C4.
"""
import argparse

import torch

SHAPES = [
    # name, M, N, K, transposes: "nt" = X[M,K] W[N,K]^T (forward), "nn" = dY[M,K] W[K,N] (data grad)
    ("tgt_ffn0", 65536, 2048, 512, "nt"),
    ("tgt_ffn2_fwd", 65536, 512, 2048, "nt"),
    ("tgt_ffn2_dx", 65536, 2048, 512, "nn"),
    ("tgt_qkv1", 65536, 768, 512, "nt"),
    ("tgt_proj0", 65536, 256, 512, "nt"),
    ("c1_ffn0", 65536, 1024, 256, "nt"),
    ("c4_ffn0", 65536, 4096, 1024, "nt"),
    ("sq4k", 4096, 4096, 4096, "nt"),
    ("sq8k", 8192, 8192, 8192, "nt"),
    # weight gradients dW[M,N] = dY[K,M]^T X[K,N] (K = B*T = 16,384 rows per modality), 4 modalities
    # batched as the grouped launches are ("tn", bmm over 4)
    ("tgt_ffn0_dw", 2048, 512, 16384, "tn4"),
    ("tgt_ffn2_dw", 512, 2048, 16384, "tn4"),
    ("tgt_qkv1_dw", 768, 512, 16384, "tn4"),
    ("tgt_proj0_dw", 256, 512, 16384, "tn4"),
    ("tgt_proj2_dw", 512, 256, 16384, "tn4"),
    ("c1_ffn0_dw", 1024, 256, 16384, "tn4"),
    ("c1_ffn2_dw", 256, 1024, 16384, "tn4"),
    ("c4_ffn0_dw", 4096, 1024, 16384, "tn1"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda"
    for name, M, N, K, tr in SHAPES:
        nb = 1
        if tr.startswith("tn"):
            nb = int(tr[2:])
            a = torch.randn(nb, K, M, device=dev).to(torch.bfloat16)
            w = torch.randn(nb, K, N, device=dev).to(torch.bfloat16)
        else:
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = torch.randn(N, K, device=dev).to(torch.bfloat16) if tr == "nt" else torch.randn(K, N, device=dev).to(torch.bfloat16)

        def call():
            if tr.startswith("tn"):
                return torch.bmm(a.transpose(1, 2), w)
            return a @ w.t() if tr == "nt" else a @ w

        for _ in range(3):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / args.reps * 1e3
        tf = 2.0 * nb * M * N * K / (us * 1e-6) / 1e12
        print(f"hipblaslt {name:14s} {M}x{N}x{K} {tr}: {us:8.1f} us {tf:7.1f} TF/s ({tf / 2500 * 100:5.1f} % of 2.5 PF)",
              flush=True)


if __name__ == "__main__":
    main()
