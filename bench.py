#!/usr/bin/env python
"""bench.py — training tokens/sec of the multimodal transformer hot path on MI355X.

Metric (BASELINE.json): training tokens/sec/GPU on the 4-modality 1M-row synthetic dataset at
1/2/4/8 MI355X; `value` is the whole-job aggregate (tokens = positions x modalities, B*T*M per
rank per step). Workload C1: d_model 256, 6 layers, seq 256, 8 heads, batch 64 per GPU,
V = [900, 13, 144, 5], cross-attention on modality 0. A step is the full hot
loop of reference main.py:641-650 on HBM-resident data: device get_batch (+-1 random walk of the
900k-row training streams, start indices, window gather), forward, loss, backward, gradient
all-reduce (N > 1), fused AdamW.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c1|target|c3|c4] [--no-cpu-baseline]

Multi-GPU: one rank per GPU, RCCL ("nccl") all-reduce of the flat gradient, weak scaling (fixed
batch per GPU). Launched by torch.distributed.run (the driver's line), or, when `--gpus N > 1` is
given without it, this process starts that launcher itself (launch_plan) before touching a GPU.

Roofline: the engine times every launch matching the probe patterns (default: all weight-gradient
GEMMs, attention forward / backward, ffn0, the ffn2 data gradient, the other data gradients) with HIP
events on the stream it runs on, over --probe-steps live steps run AFTER the timed region (the timed
steps carry no events), and reports each family's algorithmic flops / bytes per launch over that time; `roofline` is the family with the largest measured time per step, `kernels` all of them.
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
    "c4": dict(M=4, C=1024, H=16, L=24, T=4096, B=4),
}
WORKLOADS = {"c1": "C1: 4-modality 1M-row synthetic, d256 L6 T256 (BASELINE configs[1])",
             "target": "north-star target shape: 4-modality 1M-row synthetic, d512 L6 T512",
             "c3": "C3: 8-modality selective cross-attention stress, d512 L12 T1024 (BASELINE configs[3], per GPU)",
             "c4": "C4: 4-modality, d1024 L24 T4096 (BASELINE configs[4], per GPU)"}
PEAK_TFLOPS = 2500.0  # MI355X bf16 dense MFMA (MI355X_MICROARCH.md; no sparsity)
PEAK_TFLOPS_FP8 = 5000.0  # MX-fp8 dense MFMA (v_mfma_scale_f32_32x32x64_f8f6f4: 2x the bf16 rate)
# forward GEMM launch labels that run on the MX-fp8 kernel under precision fp8 (mmt_engine.hip run_forward)
FP8_LABELS = {"qkv1", "ffn0", "ffn2", "ca_q"}
PEAK_HBM_GBS = 8000.0  # HBM3E
METRIC = "training tokens/sec/GPU, 4-modality 1M-row synthetic, at 1/2/4/8 MI355X"


def train_flops_per_row(M, C, H, L, T, V, cross, a=0.5):
    """6 x forward MACs per row (one position across all modalities), causal-useful a=1/2."""
    X = [i for i in range(M) if cross[i]] if M > 1 else []
    mac = L * (M * (2.5 * C * C + 1.5 * C * C / H + a * 2 * T * C + 8 * C * C)
               + sum(2 * C * C + (M - 1) * (2 * C * C + a * 2 * T * C) for _ in X))
    mac += sum(C * (v // 2) + (v // 2) * v for v in V)
    return 6.0 * mac


PROBES = ["*_dw", "attn_fwd", "attn_bwd", "ffn0", "ffn2_dx", "*_dx"]  # engine launch labels timed live (first match)
PROBE_NAMES = {"*_dw": "weight-gradient GEMMs (all *_dw launches: split-K 256x256 / 128x128 gemm_kernel)",
               "attn_fwd": "attn_fwd_kernel (causal self-attention forward)",
               "attn_bwd": "self-attention backward (hs 32, T <= 256: attn_bwd_fused32, dQ / dK / dV in one pass with "
                           "the Q/K/V stage-2 backward in its epilogue; otherwise a dQ pass + a dK/dV pass: "
                           "attn_bwd_dq_kernel + attn_bwd_dkdv1_kernel, hs 64 on the slice rings)",
               "ffn0": "gemm_kernel ffn0 (X W0^T + b, ReLU, bf16 out)",
               "ffn2_dx": "gemm_kernel ffn2 data gradient (dY W2, ReLU' epilogue, bias-grad column sums)",
               "*_dx": "the other backward-data GEMMs (incl. the LayerNorm-backward fused ones: ffn0 / qkv1 / "
                       "cross-query / head0 dX), all on the main stream"}


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


def fp8_flops_per_row(M, C, L, cross):
    """Training flops per row that run on the MX-fp8 forward GEMMs under precision fp8: the forward of
    Q/K/V stage 1 (C x 3C/2), FFN up + down (8 C^2) per modality and the cross query (C^2) per
    cross-enabled modality (2 flops per MAC; their backward stays bf16)."""
    X = sum(1 for i in range(M) if cross[i]) if M > 1 else 0
    return 2.0 * L * (M * 9.5 * C * C + X * C * C)


def roofline_entry(label, ms, n, flops, nbytes, sampled_steps, config, peak=PEAK_TFLOPS):
    """Roofline of one probed launch family: algorithmic flops / bytes per launch (reported by the
    engine for each launch) over the live HIP-event launch time; the binding roof at the family's
    arithmetic intensity (ridge = peak / 8 TB/s: 312.5 flop/B at bf16, 625 at MX-fp8)."""
    sec = ms * 1e-3 / n
    fl, by = flops / n, nbytes / n
    if fl / by >= peak * 1e12 / (PEAK_HBM_GBS * 1e9):
        r = {"bound": "mfma", "achieved": round(fl / sec / 1e12, 1), "peak": peak, "unit": "TFLOP/s"}
    else:
        r = {"bound": "hbm", "achieved": round(by / sec / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s"}
    r["frac"] = round(r["achieved"] / r["peak"], 4)
    r.update({"traffic": pmc_traffic(config, label), "kernel": PROBE_NAMES.get(label, label), "label": label,
              "launches_per_step": round(n / sampled_steps, 2), "ms_per_step": round(ms / sampled_steps, 4),
              "avg_launch_us": round(sec * 1e6, 2), "flops_per_launch": fl, "algorithmic_bytes_per_launch": by,
              "tflops": round(fl / sec / 1e12, 1), "gbs": round(by / sec / 1e9, 1),
              "mfma_peak_tflops": peak, "mfma_frac": round(fl / sec / 1e12 / peak, 4)})
    return r


def read_probes(L_, ctx, probes, sampled, config, peaks):
    import mmt_lib as ML
    out = []
    for pi, label in enumerate(probes):
        ms, n, fl, by = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_double(0), ctypes.c_double(0)
        ML.check(L_.mmt_probe_read_at(ctx, pi, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl),
                                      ctypes.byref(by)), ctx, "mmt_probe_read_at")
        if n.value > 0 and by.value > 0:
            out.append(roofline_entry(label, ms.value, n.value, fl.value, by.value, max(1, sampled), config,
                                      peaks.get(label, PEAK_TFLOPS)))
    return out


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(cfg, data, seconds):
    """The reference's CPU training loop restated by the oracle (oracle/mmt_oracle.py: eager fp32,
    per-head modules exactly as the reference structures them; get_batch with the reference's
    per-step list walk, list->tensor conversion and window stack), on the host cores:
      * model step: C1 at the bench's batch (64), fwd + bwd + AdamW, timed over whole steps;
      * full loop: that step + one reference get_batch('train', 1) over the 1M-row, 4-modality
        training lists (report both)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import random
    import mmt_oracle as O
    # threads: OMP_NUM_THREADS when set (the GPU box sets it to 16, the CPU share one GPU's job gets
    # there; nproc shows the whole host's cores), else every core of this host
    threads = max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))
    torch.set_num_threads(threads)
    V = data["vocab_sizes"]
    ocfg = O.OracleConfig(cfg["C"], cfg["H"], cfg["L"], cfg["T"], V, [p[8] for p in data["params"]])
    g = torch.Generator().manual_seed(0)
    sd = O.init_params(ocfg, g)
    B, T = cfg["B"], cfg["T"]
    # the batcher's share: one reference get_batch (Python-loop walk of the whole training lists)
    train_lists = [list(map(int, t)) for t in data["train"]]
    t0 = time.perf_counter()
    xb, yb = O.get_batch(train_lists, data["val"], [p[2] for p in data["params"]], V, T, B, "train", 1,
                         data["file_lengths"], data["is_percents"], generator=g, rng=random.Random(0))
    t_batch = time.perf_counter() - t0
    state = {}
    # one untimed step (first-touch allocations), then at least 5 timed steps and `seconds` of work:
    # the per-step spread is reported so a noisy host shows
    _, _, grads = O.forward_backward(sd, ocfg, xb, yb)
    O.adamw_step(sd, grads, state, 1, lr=3e-4)
    steps, times = 1, []
    t0 = time.perf_counter()
    while len(times) < 5 or time.perf_counter() - t0 < seconds:
        ts = time.perf_counter()
        _, _, grads = O.forward_backward(sd, ocfg, xb, yb)
        steps += 1
        O.adamw_step(sd, grads, state, steps, lr=3e-4)
        times.append(time.perf_counter() - ts)
    times.sort()
    t_step = times[len(times) // 2]  # median step
    toks = B * T * len(V)
    return {"value": round(toks / t_step, 1), "unit": "tokens/s", "cores": threads, "kind": "port",
            "cpu": cpu_model(),
            "full_loop_value": round(toks / (t_step + t_batch), 1),
            "step_s": round(t_step, 3), "step_s_min_max": [round(times[0], 3), round(times[-1], 3)],
            "get_batch_s": round(t_batch, 3),
            "threads_reason": "OMP_NUM_THREADS (16 on the GPU box: one GPU's CPU share)" if os.environ.get(
                "OMP_NUM_THREADS") else "all host cores",
            "sample": f"oracle/mmt_oracle.py eager fp32 per-head restatement of the reference, C1 at batch {B}: "
                      f"median of {len(times)} timed fwd+bwd+AdamW steps after 1 untimed ({t_step:.2f} s/step) on "
                      f"{threads} threads; full loop adds one "
                      f"reference get_batch('train', 1) over the {len(train_lists[0])}-row x {len(V)} training lists "
                      f"({t_batch:.2f} s)"}


def launch_plan(n, argv, port):
    """Command the parent runs when `--gpus N > 1` is asked without a torch.distributed launcher:
    one rank per GPU (the driver's own launch line), started before this process touches a GPU."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed steps (SURVEY.md §8d: 200)")
    ap.add_argument("--warmup", type=int, default=20, help="untimed warm-up steps (SURVEY.md §8d: 20)")
    ap.add_argument("--config", default="c1", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--dropout", type=float, default=0.1,
                    help="dropout p; SURVEY.md §8d: 0.1 for throughput runs (0.0 only for parity runs)")
    ap.add_argument("--probe", default=",".join(PROBES),
                    help="comma-separated engine launch-label patterns timed live (roofline: the dominant one)")
    ap.add_argument("--gemm-variant", type=int, default=-1, help="GEMM pipeline variant (mmt_gemm_set_variant)")
    ap.add_argument("--bucket-mb", type=int, default=32, help="DP gradient all-reduce bucket size")
    ap.add_argument("--precision", default=None, choices=["bf16", "fp8"],
                    help="compute precision (default: fp8 for c4 as BASELINE configs[4] names it, else bf16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--probe-steps", type=int, default=8,
                    help="probed live steps after the timed region (per-family kernel times, roofline)")
    ap.add_argument("--serial-steps", type=int, default=8,
                    help="probed steps run with the side stream off after the main run (serial per-kernel rates)")
    ap.add_argument("--exact-steps", type=int, default=20,
                    help="steps timed with the bit-exact device get_batch (reference RNG streams) after the main run")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one rank per GPU, launched before this process makes any GPU call; exit with its status
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        return subprocess.call(launch_plan(args.gpus, sys.argv[1:], _free_port()), env=env)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # experiment: the whole step on a torch stream of this HIP priority (the engine's
    # side stream keeps the default one), unset = torch's default stream
    if os.environ.get("MMT_BENCH_MAIN_PRIORITY"):
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=int(os.environ["MMT_BENCH_MAIN_PRIORITY"])))
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus == world, (dist.get_world_size(), args.gpus, world)

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
    precision = args.precision or ("fp8" if args.config == "c4" else "bf16")
    config_utils._config_cache = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "dropout": args.dropout,
                                  "device": str(dev), "batch_size": B, "eval_iters": 1, "learning_rate": 3e-4,
                                  "precision": precision}
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
    probes = [p for p in args.probe.split(",") if p]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed steps carry no probe events (each event record is a queue barrier): the per-family
    # kernel times come from separate probed steps after the timed region
    t0 = time.perf_counter()
    for i in range(args.steps):
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
    peaks = {lb: PEAK_TFLOPS_FP8 for lb in FP8_LABELS} if precision == "fp8" else {}
    final_loss = float(sum(l.item() for l in losses))
    # live per-family kernel times: every launch whose label matches a probe pattern bracketed by HIP
    # events on the stream it runs on, over --probe-steps steps (side stream on, as in the timed loop;
    # the event pairs are made by mmt_probe_set, outside these steps)
    L_.mmt_probe_set(model._ctx, ",".join(probes).encode())
    L_.mmt_probe_enable(model._ctx, 1)
    for _ in range(args.probe_steps):
        step()
    torch.cuda.synchronize()
    kernels = read_probes(L_, model._ctx, probes, args.probe_steps, args.config, peaks)
    L_.mmt_probe_set(model._ctx, None)
    if args.serial_steps > 0 and world == 1:
        # the same families with the side stream off (weight gradients and keep bits on the main
        # stream): each launch has the chip to itself, so these are the per-kernel rates the live
        # figures above are shares of (untimed for the headline; one warm step first)
        ML.check(L_.mmt_set_side_stream(model._ctx, 0), model._ctx, "mmt_set_side_stream")
        step()
        torch.cuda.synchronize()
        L_.mmt_probe_set(model._ctx, ",".join(probes).encode())
        L_.mmt_probe_enable(model._ctx, 1)
        for _ in range(args.serial_steps):
            step()
        torch.cuda.synchronize()
        serial = {k["label"]: k for k in read_probes(L_, model._ctx, probes, args.serial_steps, args.config, peaks)}
        L_.mmt_probe_set(model._ctx, None)
        ML.check(L_.mmt_set_side_stream(model._ctx, 1), model._ctx, "mmt_set_side_stream")
        for k in kernels:
            sk = serial.get(k["label"])
            if sk:
                k["serial"] = {"avg_launch_us": sk["avg_launch_us"], "achieved": sk["achieved"], "frac": sk["frac"],
                               "tflops": sk["tflops"], "mfma_frac": sk["mfma_frac"], "ms_per_step": sk["ms_per_step"]}
    nonfinite = int(model.nonfinite_loss_mask(sticky=True).item())

    tokens = world * B * T * M * args.steps
    value = tokens / dt
    cross = [p[8] for p in data["params"]]
    flops_row = train_flops_per_row(M, C, H, L, T, V, cross)
    achieved_step_tflops = flops_row * B * T * args.steps / dt / 1e12  # per GPU
    # the MFMA fraction of the step: each flop priced at the peak of the unit it runs on (MX-fp8 for
    # the fp8 forward GEMMs under precision fp8, bf16 for the rest)
    f8_row = fp8_flops_per_row(M, C, L, cross) if precision == "fp8" else 0.0
    step_peak_s = (f8_row / (PEAK_TFLOPS_FP8 * 1e12) + (flops_row - f8_row) / (PEAK_TFLOPS * 1e12)) * B * T * args.steps
    step_mfma_frac = step_peak_s / dt
    # the roofline line prices the DOMINANT probed family by measured time per step
    roof = dict(max(kernels, key=lambda k: k["ms_per_step"])) if kernels else None
    if roof and "serial" in roof:
        # the live frac is this family's share of a GPU the concurrent side stream also loads; the
        # serial one (side stream off) is the kernel's own rate
        roof["frac_live"] = roof["frac"]
        roof["frac_serial"] = roof["serial"]["frac"]
        roof["achieved_serial"] = roof["serial"]["achieved"]

    # the critical path: the largest probed family on the caller's (main) stream -- the weight gradients run
    # on the side stream beside it, so the headline roofline above prices a family that is mostly off it
    main_fams = [k for k in kernels if k["label"] != "*_dw"]
    main_stream = None
    if main_fams:
        mk = max(main_fams, key=lambda k: k["ms_per_step"])
        main_stream = {key: mk.get(key) for key in ("label", "kernel", "bound", "achieved", "peak", "unit", "frac",
                                                      "ms_per_step", "launches_per_step", "avg_launch_us", "mfma_frac")}
        if "serial" in mk:
            main_stream["frac_serial"] = mk["serial"]["frac"]

    exact = None
    if args.exact_steps > 0 and world == 1:
        # the same loop fed by get_batch bit-exact with the reference (its Python `random` and torch
        # RNG streams): the device-exact batcher (MT19937 on the GPU, prefix-sum walk) over
        # args.exact_steps steps after 2 untimed ones, and the exact host batcher over 3 steps
        import random
        mmt_data.install(TU, data, model)
        config_utils._config_cache.update({"device": str(dev)})

        def exact_run(mode, n, warm):
            TU.use_device_batcher = mode == "device"
            TU.batcher_mode = "exact"
            TU._device_batcher[0] = None
            random.seed(0)
            for k in range(warm + n):
                if k == warm:
                    torch.cuda.synchronize()
                    t_ = time.perf_counter()
                xb, yb = TU.get_batch("train", 1)
                _, ls = model(xb, yb)
                opt.zero_grad(set_to_none=True)
                sum(ls).backward()
                opt.step()
            torch.cuda.synchronize()
            t_ = time.perf_counter() - t_
            TU.sync_host_state()
            return {"tokens_per_s": round(B * T * M * n / t_, 1), "ms_per_step": round(t_ / n * 1e3, 2), "steps": n}
        exact = exact_run("device", args.exact_steps, 2)
        exact["mode"] = "device-exact get_batch (Python's MT19937 on the GPU, prefix-sum walk; bit-exact batches)"
        exact["host_exact"] = exact_run("host", 3, 0)
        exact["vs_headline"] = round(exact["tokens_per_s"] / value, 4)
        TU.use_device_batcher = True
        TU.batcher_mode = "hash"
        TU._device_batcher[0] = None

    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "bf16" if precision == "bf16" else "fp8 (MX e4m3: Q/K/V stage 1, FFN, cross query) + bf16",
        "data": "synthetic",
        "config": {"workload": WORKLOADS[args.config],
                   "model": "multimodal-transformer", "global_batch": B * world, "seq_len": T, "n_embd": C,
                   "n_head": H, "n_layer": L, "modalities": M, "vocab_sizes": V, "dropout": args.dropout,
                   "parallelism": f"dp{world}"},
        "tokens_per_gpu_per_s": round(value / world, 1),
        "step_tflops_per_gpu": round(achieved_step_tflops, 2),
        "step_mfma_frac": round(step_mfma_frac, 4),
        "train_flops_per_row": flops_row,
        "final_loss": round(final_loss, 4),
        "nonfinite_loss_flags": nonfinite,
        "roofline": roof,
        "main_stream": main_stream,
        "kernels": kernels,
        "exact_batcher": exact,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cfg, data, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
