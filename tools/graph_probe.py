"""Timing probe: one training step (device get_batch + forward + backward + AdamW, as bench.py)
captured in a HIP graph (torch.cuda.graph) and replayed, against the same step launched eagerly.
The replay re-uses the captured per-step scalars (batch counter, dropout seed, AdamW step), so
this measures launch / queue overhead only — it is not a training loop.

    python tools/graph_probe.py [--config c1] [--steps 50]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c1")
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    import config_utils
    import mmt_data
    import mmt_optim
    import training_utils as TU
    from model import MultimodalTransformer
    cfg = bench.CONFIGS[a.config]
    M, C, H, L, T, B = cfg["M"], cfg["C"], cfg["H"], cfg["L"], cfg["T"], cfg["B"]
    config_utils._config_cache = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "dropout": 0.1,
                                  "device": str(dev), "batch_size": B, "eval_iters": 1, "learning_rate": 3e-4,
                                  "precision": "bf16"}
    data = mmt_data.make_synthetic(n_modalities=M)
    V = data["vocab_sizes"]
    torch.manual_seed(1234)
    model = MultimodalTransformer(M, V, data["params"]).to(dev)
    opt = mmt_optim.AdamW(model.parameters(), lr=3e-4)
    batcher = TU.DeviceBatcher(data["train"], data["val"], V, [p[2] for p in data["params"]], data["file_lengths"],
                               data["is_percents"], T, B, dev, seed=1000)

    def step():
        xb, yb = batcher.next("train", 1)
        _, losses = model(xb, yb)
        opt.zero_grad(set_to_none=False)
        sum(losses).backward()
        opt.step()
        return losses

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(5):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"eager  {eager:.3f} ms/step", flush=True)
    # host launch cost: enqueue a few steps without waiting (the GPU trails behind)
    for n in (1, 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        host = (time.perf_counter() - t0) / n * 1e3
        torch.cuda.synchronize()
        print(f"host   {host:.3f} ms/step to enqueue ({n} steps)", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"graph  {graph:.3f} ms/step  ({(1 - graph / eager) * 100:+.1f} % vs eager)", flush=True)


if __name__ == "__main__":
    main()
