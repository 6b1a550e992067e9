"""Fused out-projection MLP (mmt_op_mlp2 / mmt_op_mlp2_bwd) against the two-GEMM pairs it replaces.

    python tools/mlp2_bench.py [--reps 20]

Shapes: the grouped launches of the target (R = 4 x 32 x 512 rows, C = 512) and C1 (R = 4 x 64 x 256, C = 256),
as one problem of R rows. HIP-event timing on the current stream; prints us per call.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))

import torch  # noqa: E402

import mmt_lib as ML  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    L = ML.lib()
    s = ML.stream_ptr()
    for name, R, C in [("target", 65536, 512), ("c1", 65536, 256)]:
        N1 = C // 2
        x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
        w0 = (torch.randn(N1, C, device="cuda") * 0.05).to(torch.bfloat16)
        w2 = (torch.randn(C, N1, device="cuda") * 0.05).to(torch.bfloat16)
        b0 = torch.randn(N1, device="cuda") * 0.1
        b2 = torch.randn(C, device="cuda") * 0.1
        resid = torch.randn(R, C, device="cuda")
        h = torch.zeros(R, N1, dtype=torch.bfloat16, device="cuda")
        out = torch.zeros(R, C, device="cuda")
        dh = torch.zeros(R, N1, dtype=torch.bfloat16, device="cuda")
        dx = torch.zeros(R, C, dtype=torch.bfloat16, device="cuda")
        db0 = torch.zeros(N1, device="cuda")
        thr = int(0.1 * 65536)

        def fused():
            assert L.mmt_op_mlp2(s, R, C, ML.ptr(x), C, ML.ptr(w0), C, ML.ptr(b0), ML.ptr(w2), N1, ML.ptr(b2), ML.ptr(h), N1,
                                 ML.ptr(resid), ML.ptr(out), None, 77, thr, 1.0 / 0.9, None, None, None, None, None) == 0

        def pair():
            assert L.mmt_op_gemm(s, 1, 1, ML.EPI["bias_tanh_bf16"], 1, R, N1, C, ML.ptr(x), C, ML.ptr(w0), C, ML.ptr(b0),
                                 None, 0, None, 0, None, 0, ML.ptr(h), N1, 1.0) == 0
            assert L.mmt_op_gemm(s, 1, 1, ML.EPI["bias_resid_f32"], 1, R, C, N1, ML.ptr(h), N1, ML.ptr(w2), N1, ML.ptr(b2),
                                 None, 0, ML.ptr(resid), C, ML.ptr(out), C, None, 0, 1.0) == 0

        def fused_bwd():
            assert L.mmt_op_mlp2_bwd(s, R, C, ML.ptr(x), C, ML.ptr(w2), N1, ML.ptr(h), N1, 1.0, ML.ptr(w0), C, ML.ptr(dh),
                                     N1, ML.ptr(db0), ML.ptr(dx)) == 0

        def pair_bwd():
            assert L.mmt_op_gemm(s, 1, 0, ML.EPI["dtanh_bf16"], 1, R, N1, C, ML.ptr(x), C, ML.ptr(w2), N1, None,
                                 ML.ptr(h), N1, None, 0, None, 0, ML.ptr(dh), N1, 1.0) == 0
            assert L.mmt_op_gemm(s, 1, 0, ML.EPI["store_bf16"], 1, R, C, N1, ML.ptr(dh), N1, ML.ptr(w0), C, None,
                                 None, 0, None, 0, None, 0, ML.ptr(dx), C, 1.0) == 0

        fl = 2.0 * 2 * R * C * N1
        for lab, fn in [("fwd fused", fused), ("fwd pair", pair), ("bwd fused", fused_bwd), ("bwd pair", pair_bwd)]:
            us = timeit(fn, args.reps)
            print(f"{name:7s} {lab:10s} {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
