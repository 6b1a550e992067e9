"""Run-to-run drift of full-size training: the C4 20-step property run of
tests/test_gpu_scale.py, repeated with the same seed, init and batch, and once from an init moved by
one ulp, in bf16 and in MX-fp8. Prints, per modality, the loss change over the 20 steps of each run and
the spread between the repeats, so the fp8-vs-bf16 band of the property test can be sized from it.

    python tools/fp8_drift.py [--config c4] [--steps 20] [--reps 2]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("trade-aid-multimodal-transformer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))

import torch  # noqa: E402

import config_utils  # noqa: E402
import test_gpu_scale as S  # noqa: E402


def run(name, prec, steps, ulp=False):
    import mmt_optim
    from model import MultimodalTransformer
    M, C, H, L, T, B, cross, _ = S.FULL[name]
    V = [900, 13, 144, 5] * (M // 4)
    config_utils._config_cache = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "dropout": 0.1,
                                  "device": "cuda", "batch_size": B, "eval_iters": 1, "precision": prec}
    torch.manual_seed(7)
    m = MultimodalTransformer(M, V, [[None] * 8 + [c] + [None] * 3 for c in cross]).to("cuda")
    if ulp:  # every parameter moved by one ulp, random sign
        with torch.no_grad():
            g = torch.Generator(device="cuda").manual_seed(1)
            sgn = torch.randint(0, 2, m.flat_params.shape, device="cuda", generator=g) * 2 - 1
            m.flat_params.copy_(torch.nextafter(m.flat_params, m.flat_params + sgn.float() * float("inf")))
    m.train()
    opt = mmt_optim.AdamW(m.parameters(), lr=3e-4)
    t = torch.arange(T + 1, device="cuda")
    seq = [((torch.arange(B, device="cuda")[:, None] * 7 + t[None, :] * (2 * i + 1)) % v) for i, v in enumerate(V)]
    idx = [s[:, :T].contiguous() for s in seq]
    tgt = [s[:, 1:].contiguous() for s in seq]
    hist = []
    for _ in range(steps):
        _, losses = m(idx, tgt)
        opt.zero_grad(set_to_none=True)
        sum(losses).backward()
        opt.step()
        hist.append(torch.stack([l.detach() for l in losses]))
    torch.cuda.synchronize()
    h = torch.stack(hist).cpu()
    del m, opt
    torch.cuda.empty_cache()
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    for prec in ("fp8", "bf16"):
        runs = [run(a.config, prec, a.steps) for _ in range(a.reps)] + [run(a.config, prec, a.steps, ulp=True)]
        start = runs[0][0]
        print(f"{prec}: start {[round(x, 4) for x in start.tolist()]}", flush=True)
        for k, h in enumerate(runs):
            d = h[-3:].mean(0) - h[0]
            tag = "ulp" if k == a.reps else f"rep{k}"
            print(f"  {tag:5s} change/start {[round(x, 5) for x in (d / start).tolist()]} "
                  f"last {[round(x, 4) for x in h[-1].tolist()]}", flush=True)
        ds = torch.stack([(h[-3:].mean(0) - h[0]) / start for h in runs])
        print(f"  spread (max - min of change/start over the {len(runs)} runs) "
              f"{[round(x, 5) for x in (ds.max(0).values - ds.min(0).values).tolist()]}", flush=True)


if __name__ == "__main__":
    main()
