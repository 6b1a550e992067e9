"""Per-block phase timing of the GEMM kernel from s_memtime stamps (diagnostic build).

    python tools/build_variant.py stamps -DMMT_GEMM_STAMPS=1
    MMT_LIB_PATH=build_variants/stamps/libmmt_hip.so python tools/gemm_stamps.py [--variants ...]

For each shape: median / p90 cycles per block of the phases prologue-issue (0-1), first stage wait
(1-2), K loop (2-3), epilogue (3-4), and the whole block, plus the per-K-step loop cost and the
fraction of the block spent outside the K loop.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))

import torch  # noqa: E402

import mmt_lib as ML  # noqa: E402

R = 65536
SHAPES = [
    # name, a_kc, b_kc, epi, M, N, K, BK of the tile it takes
    ("tgt_ffn0_fwd", 1, 1, "bias_relu_bf16", R, 2048, 512),
    ("tgt_ffn2_fwd", 1, 1, "bias_resid_f32", R, 512, 2048),
    ("tgt_ffn2_dx", 1, 0, "drelu_bf16", R, 2048, 512),
    ("c1_ffn0_fwd", 1, 1, "bias_relu_bf16", R, 1024, 256),
    ("sq4k_store", 1, 1, "store_bf16", 4096, 4096, 4096),
    ("rate_1k_16k_kc", 1, 1, "store_f32", 1024, 1024, 16384),
]


def r8(x):
    return (x + 7) // 8 * 8


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="-1")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    L = ML.lib()
    L.mmt_gemm_set_stamps.argtypes = [ctypes.c_void_p]
    for v in [int(x) for x in a.variants.split(",")]:
        assert L.mmt_gemm_set_variant(v) == 0
        for name, akc, bkc, epi, M, N, K in SHAPES:
            if a.only and not any(k in name for k in a.only.split(",")):
                continue
            A = torch.randn(M, r8(K), device="cuda").to(torch.bfloat16) if akc else \
                torch.randn(K, r8(M), device="cuda").to(torch.bfloat16)
            B = torch.randn(N, r8(K), device="cuda").to(torch.bfloat16) if bkc else \
                torch.randn(K, r8(N), device="cuda").to(torch.bfloat16)
            lda = r8(K) if akc else r8(M)
            ldb = r8(K) if bkc else r8(N)
            bias = torch.randn(N, device="cuda")
            aux = torch.randn(M, r8(N), device="cuda").to(torch.bfloat16)
            resid = torch.randn(M, N, device="cuda")
            o32 = torch.zeros(M, N, device="cuda")
            o16 = torch.zeros(M, r8(N), dtype=torch.bfloat16, device="cuda")
            st = torch.zeros(8 * 65536, dtype=torch.int64, device="cuda")
            s = ML.stream_ptr()

            def call():
                rc = L.mmt_op_gemm(s, akc, bkc, ML.EPI[epi], 1, M, N, K, ML.ptr(A), lda, ML.ptr(B), ldb, ML.ptr(bias),
                                   ML.ptr(aux), r8(N), ML.ptr(resid), N, ML.ptr(o32), N, ML.ptr(o16), r8(N), 1.0)
                assert rc == 0
            L.mmt_gemm_set_stamps(None)
            for _ in range(3):
                call()
            L.mmt_gemm_set_stamps(ctypes.c_void_p(st.data_ptr()))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call()
            e1.record()
            torch.cuda.synchronize()
            L.mmt_gemm_set_stamps(None)
            us = e0.elapsed_time(e1) * 1e3
            t = st.view(-1, 8).cpu().tolist()
            blk = [r for r in t if r[0] and r[4]]
            ph = {"prologue": [r[1] - r[0] for r in blk], "first_wait": [r[2] - r[1] for r in blk],
                  "kloop": [r[3] - r[2] for r in blk], "epilogue": [r[4] - r[3] for r in blk],
                  "block": [r[4] - r[0] for r in blk]}
            out = " ".join(f"{k} {q(vv, .5)}/{q(vv, .9)}" for k, vv in ph.items())
            frac = sum(r[3] - r[2] for r in blk) / max(1, sum(r[4] - r[0] for r in blk))
            cus = len(set((r[6], r[5] & 0xffff) for r in blk))
            print(f"variant {v}: {name:16s} {us:8.1f} us  blocks {len(blk)} on {cus} (xcc,hw_id)  "
                  f"median/p90 cycles: {out}  kloop share {frac:.2f}", flush=True)


if __name__ == "__main__":
    main()
