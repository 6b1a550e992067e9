#!/usr/bin/env python
"""bench.py — training tokens/sec of the multimodal transformer hot path on MI355X.

Metric (BASELINE.json): training tokens/sec/GPU on the 4-modality 1M-row synthetic dataset at
1/2/4/8 MI355X; `value` is the whole-job aggregate (tokens = positions x modalities, B*T*M per
rank per step). Workload C1: d_model 256, 6 layers, seq 256, 8 heads, batch 64 per GPU,
V = [900, 13, 144, 5], cross-attention on modality 0. A step is the full hot
loop of reference main.py:641-650 on HBM-resident data: device get_batch (+-1 random walk of the
900k-row training streams, start indices, window gather), forward, loss, backward, gradient
all-reduce (N > 1), fused AdamW.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|target|c3] [--no-cpu-baseline]

Multi-GPU: launched by torch.distributed.run, one rank per GPU, RCCL ("nccl") all-reduce of the
flat gradient; weak scaling (fixed batch per GPU).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "trade-aid-multimodal-transformer_amd")
sys.path.insert(0, PKG)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (M, C, H, L, T, B per GPU)
    "c1": dict(M=4, C=256, H=8, L=6, T=256, B=64),
    "target": dict(M=4, C=512, H=8, L=6, T=512, B=32),
    "c3": dict(M=8, C=512, H=8, L=12, T=1024, B=16),
}
PEAK_TFLOPS = 2500.0  # MI355X bf16 dense MFMA (MI355X_MICROARCH.md; no sparsity)
PEAK_HBM_GBS = 8000.0  # HBM3E
METRIC = "training tokens/sec/GPU, 4-modality 1M-row synthetic, at 1/2/4/8 MI355X"


def train_flops_per_row(M, C, H, L, T, V, cross, a=0.5):
    """6 x forward MACs per row (one position across all modalities), causal-useful a=1/2."""
    X = [i for i in range(M) if cross[i]] if M > 1 else []
    mac = L * (M * (2.5 * C * C + 1.5 * C * C / H + a * 2 * T * C + 8 * C * C)
               + sum(2 * C * C + (M - 1) * (2 * C * C + a * 2 * T * C) for _ in X))
    mac += sum(C * (v // 2) + (v // 2) * v for v in V)
    return 6.0 * mac


def dominant_kernel_flops(label, M, C, H, T, B, V):
    """Algorithmic flops of one grouped launch of `label` (all modalities in one launch)."""
    R = B * T
    if label == "ffn0":
        return M * 2.0 * R * C * (4 * C)
    if label == "ffn0_dw":
        return M * 2.0 * R * C * (4 * C)
    if label == "ffn2":
        return M * 2.0 * R * (4 * C) * C
    if label == "qkv1":
        return M * 2.0 * R * C * (1.5 * C)
    raise ValueError(label)


def dominant_kernel_bytes(label, M, C, H, T, B, V):
    """Algorithmic HBM bytes of one grouped launch of `label`: each operand read once, each
    output written once (bf16 activations / packed weights, fp32 bias)."""
    R = B * T
    if label == "ffn0":
        return M * (R * C * 2 + 4 * C * C * 2 + 4 * C * 4 + R * 4 * C * 2)
    if label == "ffn2":
        return M * (R * 4 * C * 2 + 4 * C * C * 2 + C * 4 + 2 * R * C * 4 + R * C * 2)
    if label == "qkv1":
        return M * (R * C * 2 + int(1.5 * C) * C * 2 + int(1.5 * C) * 4 + R * int(1.5 * C) * 2)
    raise ValueError(label)


def pmc_traffic(config, label):
    """HBM bytes per launch of `label` at `config` from the committed PMC passes
    (profiles/pmc_traffic.json: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate runs of this
    bench, FETCH_SIZE doubled per the gfx950 correction of MI355X_MICROARCH.md); None when not
    collected for this kernel and config."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(config, {}).get(label, {}).get("bytes_per_launch")
    except (OSError, ValueError, AttributeError):
        return None


def cpu_baseline(cfg, data, seconds):
    """The CPU oracle (per-head eager fp32 restatement of the reference structure) on the host
    cores, a bounded sample of the same workload: C1 shapes at a small batch, fwd+bwd+AdamW."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import mmt_oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    V = data["vocab_sizes"]
    ocfg = O.OracleConfig(cfg["C"], cfg["H"], cfg["L"], cfg["T"], V, [p[8] for p in data["params"]])
    g = torch.Generator().manual_seed(0)
    sd = O.init_params(ocfg, g)
    B = 2
    T = cfg["T"]
    idx = [torch.randint(0, v, (B, T), generator=g) for v in V]
    tgt = [torch.randint(0, v, (B, T), generator=g) for v in V]
    state = {}
    steps = 0
    t0 = time.perf_counter()
    while True:
        _, _, grads = O.forward_backward(sd, ocfg, idx, tgt)
        steps += 1
        O.adamw_step(sd, grads, state, steps, lr=3e-4)
        if time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    toks = steps * B * T * len(V)
    return {"value": toks / dt, "unit": "tokens/s", "cores": threads, "kind": "port",
            "sample": f"oracle/mmt_oracle.py eager fp32 per-head restatement, C1 shapes at batch {B}, "
                      f"{steps} fwd+bwd+AdamW steps in {dt:.1f}s on {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed steps (SURVEY.md §8d: 200)")
    ap.add_argument("--warmup", type=int, default=20, help="untimed warm-up steps (SURVEY.md §8d: 20)")
    ap.add_argument("--config", default="c1", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--dropout", type=float, default=0.1,
                    help="dropout p; SURVEY.md §8d: 0.1 for throughput runs (0.0 only for parity runs)")
    ap.add_argument("--probe", default="ffn0", help="engine launch label timed live for the roofline line")
    ap.add_argument("--gemm-variant", type=int, default=-1, help="GEMM pipeline variant (mmt_gemm_set_variant)")
    ap.add_argument("--bucket-mb", type=int, default=32, help="DP gradient all-reduce bucket size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import config_utils
    import mmt_data
    import mmt_dist
    import mmt_lib as ML
    import mmt_optim
    import training_utils as TU
    from model import MultimodalTransformer

    if args.gemm_variant >= 0:
        ML.lib().mmt_gemm_set_variant(args.gemm_variant)
    cfg = dict(CONFIGS[args.config])
    if args.batch:
        cfg["B"] = args.batch
    M, C, H, L, T, B = cfg["M"], cfg["C"], cfg["H"], cfg["L"], cfg["T"], cfg["B"]
    config_utils._config_cache = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "dropout": args.dropout,
                                  "device": str(dev), "batch_size": B, "eval_iters": 1, "learning_rate": 3e-4}
    data = mmt_data.make_synthetic(n_modalities=M)
    V = data["vocab_sizes"]
    torch.manual_seed(1234)
    model = MultimodalTransformer(M, V, data["params"]).to(dev)
    if world > 1:
        # identical replicas (broadcast from rank 0) + bucketed gradient all-reduce over RCCL,
        # issued stage by stage during the backward (overlapped with the remaining stages)
        mmt_dist.enable_data_parallel(model, bucket_bytes=args.bucket_mb << 20)
    opt = mmt_optim.AdamW(model.parameters(), lr=3e-4)
    batcher = TU.DeviceBatcher(data["train"], data["val"], V, [p[2] for p in data["params"]], data["file_lengths"],
                               data["is_percents"], T, B, dev, seed=1000 + rank)

    def step():
        xb, yb = batcher.next("train", 1)
        _, losses = model(xb, yb)
        opt.zero_grad(set_to_none=True)
        sum(losses).backward()  # DP: the gradient comes back already averaged over ranks
        opt.step()
        return losses

    for _ in range(args.warmup):
        losses = step()
    torch.cuda.synchronize()
    L_ = ML.lib()
    L_.mmt_probe_set(model._ctx, args.probe.encode())
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        # the probe's HIP events are recorded on one step in four (each event record is a queue
        # barrier, ~0.06 ms/step when every launch is bracketed)
        L_.mmt_probe_enable(model._ctx, 1 if i % 4 == 0 else 0)
        losses = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    if world > 1:
        tt = torch.tensor([dt], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    probe_ms = ctypes.c_double(0)
    probe_n = ctypes.c_int64(0)
    L_.mmt_probe_read(model._ctx, ctypes.byref(probe_ms), ctypes.byref(probe_n))
    L_.mmt_probe_set(model._ctx, None)
    final_loss = float(sum(l.item() for l in losses))

    tokens = world * B * T * M * args.steps
    value = tokens / dt
    flops_row = train_flops_per_row(M, C, H, L, T, V, [p[8] for p in data["params"]])
    achieved_step_tflops = flops_row * B * T * args.steps / dt / 1e12  # per GPU
    roof = None
    if probe_n.value > 0:
        per_launch_ms = probe_ms.value / probe_n.value
        fl = dominant_kernel_flops(args.probe, M, C, H, T, B, V)
        by = dominant_kernel_bytes(args.probe, M, C, H, T, B, V)
        sec = per_launch_ms * 1e-3
        # the binding roof at this kernel's arithmetic intensity (ridge = 2500 TFLOP/s / 8 TB/s)
        if fl / by >= PEAK_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9):
            roof = {"bound": "mfma", "achieved": round(fl / sec / 1e12, 1), "peak": PEAK_TFLOPS, "unit": "TFLOP/s"}
        else:
            roof = {"bound": "hbm", "achieved": round(by / sec / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s"}
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof.update({"traffic": pmc_traffic(args.config, args.probe), "kernel": args.probe, "launches": probe_n.value,
                     "avg_launch_us": round(per_launch_ms * 1e3, 2), "flops_per_launch": fl,
                     "algorithmic_bytes_per_launch": by, "tflops": round(fl / sec / 1e12, 1),
                     "gbs": round(by / sec / 1e9, 1)})
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": f"{args.config}: 4-modality 1M-row synthetic" if M == 4 else f"{args.config}: 8-modality",
                   "model": "multimodal-transformer", "global_batch": B * world, "seq_len": T, "n_embd": C,
                   "n_head": H, "n_layer": L, "modalities": M, "vocab_sizes": V, "dropout": args.dropout,
                   "parallelism": f"dp{world}"},
        "tokens_per_gpu_per_s": round(value / world, 1),
        "step_tflops_per_gpu": round(achieved_step_tflops, 2),
        "step_mfma_frac": round(achieved_step_tflops / PEAK_TFLOPS, 4),
        "train_flops_per_row": flops_row,
        "final_loss": round(final_loss, 4),
        "roofline": roof,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, data, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
