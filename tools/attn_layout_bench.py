"""Attention forward/backward time vs the Q/K/V memory layout (no dropout), through the C-ABI ops.

    python tools/attn_layout_bench.py

(i) the engine's layout: one interleaved [B*T, 3C] bf16 buffer, a head's 32 columns a 64-B
    segment of a 1.5-KiB row; (ii) head-major [H, T, hs] (B = 1, so row*ld + h*hstride addresses
    it): every (b, h) item reads contiguous memory. Same work: 512 (b, h) pairs x T = 256, hs = 32.
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))
import torch  # noqa: E402

import mmt_lib as ML  # noqa: E402


def run(B, H, T, hs, layout, reps=20):
    C = H * hs
    R = B * T
    dev = "cuda"
    L = ML.lib()
    s = ML.stream_ptr()
    if layout == "interleaved":
        qkv = torch.randn(R, 3 * C, device=dev).to(torch.bfloat16)
        q, q_ld = qkv[:, C:2 * C], 3 * C
        kp, vp = [qkv], [qkv[:, 2 * C:]]
        kv_ld, kv_hs = 3 * C, hs
        dq_ld = 3 * C
    else:  # head-major, B == 1
        assert B == 1
        qb = torch.randn(H, T, hs, device=dev).to(torch.bfloat16)
        kb = torch.randn(H, T, hs, device=dev).to(torch.bfloat16)
        vb = torch.randn(H, T, hs, device=dev).to(torch.bfloat16)
        q, q_ld = qb, hs
        kp, vp = [kb], [vb]
        kv_ld, kv_hs = hs, T * hs
        dq_ld = hs
    o = torch.zeros(R, C, dtype=torch.bfloat16, device=dev)
    lse = [torch.zeros(B * H * T, device=dev)]
    kpp = (ctypes.c_void_p * 1)(kp[0].data_ptr())
    vpp = (ctypes.c_void_p * 1)(vp[0].data_ptr())

    def fwd():
        rc = L.mmt_op_attention_fwd(s, B, T, H, hs, 1, ML.ptr(q), q_ld, kpp, vpp, kv_ld, kv_hs, ML.ptr(o), C,
                                    None, ML.ptr_array(lse))
        assert rc == 0

    for _ in range(3):
        fwd()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fwd()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


if __name__ == "__main__":
    for (B, H, lay) in [(64, 8, "interleaved"), (1, 512, "headmajor"), (64, 8, "interleaved"), (1, 512, "headmajor")]:
        print(f"{lay:12s} B={B} H={H}: fwd {run(B, H, 256, 32, lay):.1f} us", flush=True)
