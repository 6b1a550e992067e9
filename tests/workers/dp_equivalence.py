"""Worker of tests/test_gpu_dp.py (launched by torch.distributed.run, 2 ranks on one GPU, gloo).

Each rank trains on its half of one global batch with mmt_dist's bucketed, stage-overlapped
gradient averaging; rank 0 also runs the whole global batch through a second, single-process
replica. DP equivalence: N ranks x local batch b == 1 rank x batch N*b on the same
samples -> gradients, losses and the params after 2 AdamW steps agree (the only difference is
the fp32 summation order of the weight-gradient split-K accumulation). Then with dropout 0.1:
each rank draws its own masks, and the averaged gradient equals the oracle's mean of per-rank
gradients under each rank's hash masks (dropout_phase).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    import config_utils
    import mmt_dist
    import mmt_optim
    from model import MultimodalTransformer
    C, H, L, T, Bg = 64, 2, 2, 64, 8
    V = [57, 13, 24, 5]
    cross = [True, False, True, False]
    config_utils._config_cache = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "dropout": 0.0,
                                  "device": "cuda", "batch_size": Bg, "eval_iters": 1}
    params = [[None] * 8 + [c] + [None] * 3 for c in cross]
    torch.manual_seed(1234 + 17 * rank)  # different init per rank: the broadcast must fix it
    m = MultimodalTransformer(len(V), V, params).to("cuda")
    sync = mmt_dist.enable_data_parallel(m, bucket_bytes=64 << 10)
    assert len(sync.buckets) >= 3, sync.buckets
    g = torch.Generator().manual_seed(99)
    idx = [torch.randint(0, v, (Bg, T), generator=g) for v in V]
    tgt = [torch.randint(0, v, (Bg, T), generator=g) for v in V]
    b = Bg // world
    mine = slice(rank * b, (rank + 1) * b)
    opt = mmt_optim.AdamW(m.parameters(), lr=1e-3)
    ref = None
    if rank == 0:
        ref = MultimodalTransformer(len(V), V, params).to("cuda")
        with torch.no_grad():
            ref.flat_params.copy_(m.flat_params)
        ropt = mmt_optim.AdamW(ref.parameters(), lr=1e-3)
    fails = []
    p_init = m.flat_params.detach().clone()
    for it in range(2):
        _, losses = m([t[mine].cuda() for t in idx], [t[mine].cuda() for t in tgt])
        opt.zero_grad(set_to_none=True)
        sum(losses).backward()
        gdp = m.flat_params.grad.detach().clone()
        loc = torch.stack([l.detach() for l in losses])
        dist.all_reduce(loc)  # gloo on a CUDA tensor: mean of the per-rank mean losses
        loc /= world
        opt.step()
        if rank == 0:
            _, rl = ref([t.cuda() for t in idx], [t.cuda() for t in tgt])
            ropt.zero_grad(set_to_none=True)
            sum(rl).backward()
            gref = ref.flat_params.grad.detach()
            e = ((gdp - gref).norm() / gref.norm()).item()
            lerr = (loc - torch.stack([l.detach() for l in rl])).abs().max().item()
            ropt.step()
            # AdamW's early updates are ~lr * sign(g): near-zero gradient elements may flip sign under
            # a different fp32 summation order, so compare the accumulated UPDATES in L2
            upd_ref = ref.flat_params.detach() - p_init
            perr = ((m.flat_params.detach() - p_init - upd_ref).norm() / upd_ref.norm()).item()
            print(f"iter {it}: grad rel-L2 {e:.2e}  loss max-abs {lerr:.2e}  update rel-L2 {perr:.2e}", flush=True)
            if not (e < 2e-3 and lerr < 2e-3 and perr < 5e-2):
                fails.append((it, e, lerr, perr))
    # replicas stay identical across ranks
    p = m.flat_params.detach().clone()
    p0 = p.clone()
    dist.broadcast(p0, src=0)
    same = torch.equal(p, p0)
    if not same:
        fails.append(("replica drift", rank))
    fails += dropout_phase(rank, world, C, H, L, T, Bg, V, cross, params, idx, tgt)
    dist.destroy_process_group()
    if fails:
        print("FAIL", fails, flush=True)
        sys.exit(1)
    print(f"rank {rank} ok", flush=True)


def dropout_phase(rank, world, C, H, L, T, Bg, V, cross, params, idx, tgt):
    """Per-rank dropout streams: with every rank seeded identically, each rank still
    draws its own masks (the rank is folded into the seed), and the DP-averaged gradient equals the
    mean of the per-rank gradients the oracle computes on each rank's half with that rank's hash
    masks (whole-gradient rel-L2 <= 4e-2, the bf16 dropout bound of tests/test_gpu_scale.py)."""
    import config_utils
    import mmt_dist
    from model import MultimodalTransformer
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import mmt_oracle as O
    config_utils._config_cache = dict(config_utils._config_cache, dropout=0.1)
    torch.manual_seed(4321)  # identical on every rank, as bench.py / main.py --seed do
    m = MultimodalTransformer(len(V), V, params).to("cuda")
    mmt_dist.enable_data_parallel(m, bucket_bytes=64 << 10)
    m.train()
    b = Bg // world
    mine = slice(rank * b, (rank + 1) * b)
    _, losses = m([t[mine].cuda() for t in idx], [t[mine].cuda() for t in tgt])
    sum(losses).backward()
    torch.cuda.synchronize()
    seeds = [None] * world
    dist.all_gather_object(seeds, int(m.last_dropout_seed))
    out = []
    if len(set(seeds)) != world:
        out.append(("identical dropout seeds across ranks", seeds))
    if rank == 0:
        sd = {k: v.detach().cpu() for k, v in m.state_dict().items() if not k.endswith("tril")}
        cfg = O.OracleConfig(C, H, L, T, V, cross, dropout=0.1)
        acc = None
        for r in range(world):
            sl = slice(r * b, (r + 1) * b)
            _, _, g = O.forward_backward(sd, cfg, [t[sl] for t in idx], [t[sl] for t in tgt],
                                         hash_dropout=O.HashDropout(seeds[r], 0.1))
            acc = {k: v / world for k, v in g.items() if v is not None} if acc is None else \
                {k: acc[k] + g[k] / world for k in acc}
        got = {k: gg for k, gg in m.reference_grad_views() if gg is not None}
        a = torch.cat([got[k].flatten().cpu() for k in acc])
        r_ = torch.cat([acc[k].flatten() for k in acc])
        e = ((a - r_).norm() / r_.norm()).item()
        print(f"dropout DP: seeds {seeds}, grad rel-L2 vs per-rank-mask oracle {e:.3e}", flush=True)
        if not e < 4e-2:
            out.append(("dropout DP gradient", e))
    return out


if __name__ == "__main__":
    main()
