"""Attention microbenchmark over the step's shapes, A/B of kernel variants in one process.

    python tools/attn_bench.py [--shapes target,c3,c4,c1] [--reps 10] [--rings 0,1]

Times mmt_op_attention_fwd / _bwd (the engine's kernels, one grouped problem with B = modalities x
batch) with HIP events on the current stream, for each value of the attention variant knob
(mmt_attn_set_ring), interleaved over rounds; prints us and causal-useful TFLOP/s (forward
2 B H T^2 hs per stream, backward 2.5x that: SURVEY.md §8d).
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))

import torch  # noqa: E402

import mmt_lib as ML  # noqa: E402

SHAPES = {
    # name: (B (modalities x batch), T, H, hs, streams)
    "c1": (256, 256, 8, 32, 1),
    "c1_ca": (64, 256, 8, 32, 3),  # C1's cross-attention: one query modality, 3 KV streams
    "target": (128, 512, 8, 64, 1),
    "c3": (128, 1024, 8, 64, 1),
    "c3_ca": (64, 1024, 8, 64, 7),
    "c4": (16, 4096, 16, 64, 1),
    "c4_ca": (4, 4096, 16, 64, 3),
}


def setup(B, T, H, hs, ns):
    C = H * hs
    R = B * T
    dev = "cuda"
    if ns == 1:
        qkv = torch.randn(R, 3 * C, device=dev).to(torch.bfloat16)
        q, q_ld = qkv[:, C:2 * C], 3 * C
        kptr, vptr = [qkv], [qkv[:, 2 * C:]]
        kv_ld, kv_hs = 3 * C, hs
        dqkv = torch.zeros(R, 3 * C, dtype=torch.bfloat16, device=dev)
        dq, dq_ld = dqkv[:, C:], 3 * C
        dk, dv = [dqkv], [dqkv[:, 2 * C:]]
        dkv_ld, dkv_hs = 3 * C, hs
        keep = [qkv, dqkv]
    else:
        q = torch.randn(R, C, device=dev).to(torch.bfloat16)
        q_ld = C
        kvs = [torch.randn(R, 2 * C, device=dev).to(torch.bfloat16) for _ in range(ns)]
        kptr, vptr = kvs, [kv[:, hs:] for kv in kvs]
        kv_ld, kv_hs = 2 * C, 2 * hs
        dq = torch.zeros(R, C, dtype=torch.bfloat16, device=dev)
        dq_ld = C
        dkvs = [torch.zeros(R, 2 * C, dtype=torch.bfloat16, device=dev) for _ in range(ns)]
        dk, dv = dkvs, [d[:, hs:] for d in dkvs]
        dkv_ld, dkv_hs = 2 * C, 2 * hs
        keep = [q, kvs, dkvs]
    o = torch.zeros(R, C, dtype=torch.bfloat16, device=dev)
    oj = [torch.zeros(R, C, dtype=torch.bfloat16, device=dev) for _ in range(ns)]
    lse = [torch.zeros(B * H * T, device=dev) for _ in range(ns)]
    dvec = [torch.zeros(B * H * T, device=dev) for _ in range(ns)]
    do = torch.randn(R, C, device=dev).to(torch.bfloat16)
    vp = lambda ts: (ctypes.c_void_p * ns)(*[t.data_ptr() for t in ts])  # noqa: E731
    L = ML.lib()
    s = ML.stream_ptr()

    def fwd():
        assert L.mmt_op_attention_fwd(s, B, T, H, hs, ns, ML.ptr(q), q_ld, vp(kptr), vp(vptr), kv_ld, kv_hs, ML.ptr(o), C,
                                      ML.ptr_array(oj), ML.ptr_array(lse)) == 0

    dq32 = torch.zeros(R, C, device=dev)  # fp32 dQ rows of the one-pass hs-32 multi-stream backward (the engine's dln)

    def bwd():
        assert L.mmt_op_attention_bwd_ws(s, B, T, H, hs, ns, ML.ptr(q), q_ld, vp(kptr), vp(vptr), kv_ld, kv_hs, ML.ptr(o), C,
                                      ML.ptr_array(oj), ML.ptr_array(lse), ML.ptr(do), C, ML.ptr_array(dvec),
                                      ML.ptr(dq), dq_ld, vp(dk), vp(dv), dkv_ld, dkv_hs, ML.ptr(dq32), C) == 0
    return fwd, bwd, keep + [o, oj, lse, dvec, do, dq32]


def timeit(fn, reps):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="target,c3,c4")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rings", default="0,1")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    L = ML.lib()
    L.mmt_attn_set_ring.restype = ctypes.c_int
    rings = [int(x) for x in a.rings.split(",")]
    for name in a.shapes.split(","):
        B, T, H, hs, ns = SHAPES[name]
        fwd, bwd, _keep = setup(B, T, H, hs, ns)
        fl = 2.0 * B * H * ns * T * T * hs
        fwd()
        torch.cuda.synchronize()
        res = {}
        for rd in range(a.rounds):
            for rg in rings:
                L.mmt_attn_set_ring(rg)
                tf_ = timeit(fwd, a.reps)
                tb = timeit(bwd, a.reps)
                res.setdefault(rg, []).append((tf_, tb))
        for rg in rings:
            tf_ = min(x[0] for x in res[rg])
            tb = min(x[1] for x in res[rg])
            print(f"{name:7s} ring={rg}: fwd {tf_:8.1f} us {fl / tf_ / 1e6:7.1f} TF/s | bwd {tb:8.1f} us "
                  f"{2.5 * fl / tb / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
