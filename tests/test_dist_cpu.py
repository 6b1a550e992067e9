"""Host logic of the data-parallel path (mmt_dist) on CPU: bucket planning and the bucketed,
stage-driven gradient averaging over a world_size-2 gloo group.

The engine itself has no CPU path; the stage ranges used here are the real ones of a context
built for the f_small fixture and for the C1 bench shape (layout only, no compute).
"""
import ctypes
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import mmt_dist
import mmt_lib as ML


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stage_ranges(C, H, L, T, V, cross):
    cfg = ML.MmtConfig()
    cfg.num_modalities = len(V)
    cfg.n_embd, cfg.n_head, cfg.n_layer, cfg.block_size = C, H, L, T
    for i, v in enumerate(V):
        cfg.vocab_sizes[i] = v
        cfg.cross_attention[i] = int(cross[i])
    lib = ML.lib()
    ctx = lib.mmt_create(ctypes.byref(cfg))
    assert ctx
    try:
        b, e = ML.c_i64(), ML.c_i64()
        out = []
        for s in range(lib.mmt_backward_stage_count(ctx)):
            assert lib.mmt_backward_stage_range(ctx, s, ctypes.byref(b), ctypes.byref(e)) == 0
            out.append((b.value, e.value))
        return out, lib.mmt_param_active_count(ctx)
    finally:
        lib.mmt_destroy(ctx)


def test_plan_buckets_cover_every_stage_once():
    ranges, active = _stage_ranges(256, 8, 6, 256, [900, 13, 144, 5], [1, 0, 0, 0])
    for bb in (1, 4 << 20, 32 << 20, 1 << 40):
        buckets = mmt_dist.plan_buckets(ranges, bb)
        covered = sorted(sl for _, slices in buckets for sl in slices)
        total = sum(e - b for b, e in covered)
        assert total == active
        for (b0, e0), (b1, e1) in zip(covered, covered[1:]):
            assert e0 <= b1
        assert buckets[-1][0] == len(ranges) - 1   # the last stage always closes a bucket
        lasts = [s for s, _ in buckets]
        assert lasts == sorted(set(lasts))
    # huge bucket -> one contiguous slice (the stages walk the layout backwards)
    one = mmt_dist.plan_buckets(ranges, 1 << 40)
    assert one == [(len(ranges) - 1, [(0, active)])]


def _worker(rank, world, port, ranges, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        grad = torch.randn(n, generator=g)
        ref = sum(torch.randn(n, generator=torch.Generator().manual_seed(100 + r)) for r in range(world)) / world
        sync = mmt_dist.GradSync(ranges, bucket_bytes=64 << 10)
        assert len(sync.buckets) > 2
        for s in range(len(ranges)):
            sync.stage_done(s, grad)
        sync.finish()
        active = max(e for _, e in ranges)
        ok = torch.allclose(grad[:active], ref[:active], atol=1e-6)
        # the inactive tail (never-used cross-attention params) is not exchanged
        tail_ok = torch.equal(grad[active:], torch.randn(n, generator=torch.Generator().manual_seed(100 + rank))[active:])
        q.put((rank, bool(ok), bool(tail_ok), len(sync.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gradsync_gloo_world2_averages_every_bucket():
    ranges, active = _stage_ranges(64, 4, 2, 32, [57, 13, 24, 5], [1, 0, 1, 0])
    n = active + 1000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, ranges, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, ok, tail_ok, nb in res:
        assert ok and tail_ok, (rank, ok, tail_ok)


def _seed_worker(rank, world, port, q):
    """enable_data_parallel on a CPU-resident model (gloo): replicas broadcast from rank 0, and each
    rank's dropout seed differs although every rank seeds torch identically."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import config_utils
        from model import MultimodalTransformer
        config_utils._config_cache = {"n_embd": 32, "n_head": 4, "n_layer": 1, "block_size": 8, "dropout": 0.1,
                                      "device": "cpu", "batch_size": 2, "eval_iters": 1}
        torch.manual_seed(1000 + rank)  # different init: the broadcast must make the replicas equal
        m = MultimodalTransformer(2, [11, 5], [[None] * 8 + [c] + [None] * 3 for c in (True, False)])
        mmt_dist.enable_data_parallel(m, bucket_bytes=1 << 10)
        p0 = m.flat_params.detach().clone()
        dist.broadcast(p0, src=0)
        torch.manual_seed(7)
        seeds = [m._next_dropout_seed(torch.device("cpu")) for _ in range(3)]
        allseeds = [None] * world
        dist.all_gather_object(allseeds, seeds)
        q.put((rank, bool(torch.equal(p0, m.flat_params.detach())), allseeds))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_data_parallel_per_rank_dropout_seeds_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, same, allseeds in res:
        assert same, rank
        s0, s1 = allseeds
        assert len(set(s0)) == 3 and not set(s0) & set(s1), allseeds
