"""Whole-model parity on the GPU: the HIP training step (libmmt_hip.so through model.py) against
golden vectors produced by the reference itself (tests/golden, gen_golden.py).

Compute is bf16 on MFMA with fp32 accumulation, so the stated bf16 tolerances
apply:  losses rel <= 5e-3, logits rel-L2 <= 2e-2, all gradients together rel-L2 <= 3e-2 and
every gradient tensor rel-L2 <= 1e-1 or abs-L2 <= 2e-3 of the whole gradient norm (the small,
cancellation-heavy value-path / tiny-head grads carry ~5-15 % bf16 noise),
params after AdamW steps close to the reference's (the update of a step is ~lr, compared with
an absolute bound of 0.1*lr + bf16 slack).
"""
import ctypes

import pytest
import torch

import config_utils
import mmt_lib as ML
from golden_io import MODEL_FIXTURES, model_fixture

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def build(meta, sd, dropout=0.0):
    config_utils._config_cache = {"n_embd": meta["n_embd"], "n_head": meta["n_head"], "n_layer": meta["n_layer"],
                                  "block_size": meta["block_size"], "dropout": dropout, "device": "cuda",
                                  "batch_size": meta["B"], "eval_iters": 1}
    import model as mmt_model
    params = []
    for i, v in enumerate(meta["V"]):
        p = [None] * 12
        p[8] = meta["cross"][i]
        params.append(p)
    m = mmt_model.MultimodalTransformer(len(meta["V"]), meta["V"], params).to("cuda")
    full = dict(sd)
    T = meta["block_size"]
    for k in meta["state_dict_keys"]:
        if k.endswith("tril"):
            full[k] = torch.tril(torch.ones(T, T))
    m.load_state_dict(full, strict=True)
    return m


@pytest.mark.parametrize("name", MODEL_FIXTURES)
def test_forward_backward_matches_reference(name):
    z, meta, cfg, sd, idx, tgt = model_fixture(name)
    m = build(meta, sd)
    m.train()
    idx_d = [t.cuda() for t in idx]
    tgt_d = [t.cuda() for t in tgt]
    logits, losses = m(idx_d, tgt_d)
    total = sum(losses)
    total.backward()
    torch.cuda.synchronize()
    ref_losses = torch.from_numpy(z["losses"])
    got = torch.stack([l.detach().cpu() for l in losses])
    assert torch.allclose(got, ref_losses, rtol=5e-3, atol=5e-3), (got, ref_losses)
    for i in range(cfg.M):
        assert rel(logits[i], torch.from_numpy(z[f"logits.{i}"])) < 2e-2, i
    grads = dict(m.reference_grad_views())
    none = set(meta["grad_none"])
    allg, allr = [], []
    for k, g in grads.items():
        if k not in none:
            allg.append(g.flatten().cpu())
            allr.append(torch.from_numpy(z[f"grad.{k}"]).flatten())
    gnorm = torch.cat(allr).norm().item()
    assert rel(torch.cat(allg), torch.cat(allr)) < 3e-2
    for k, g in grads.items():
        if k in none:
            assert g is None, k  # as in the reference: never-used parameters have no gradient
            continue
        if g.numel() == 0:
            continue
        ref = torch.from_numpy(z[f"grad.{k}"])
        # per tensor: 10 % relative, or an absolute error below 0.2 % of the whole gradient's norm
        # (tiny tensors whose gradient is a near-cancelling sum, e.g. a V=2 head's [2,1] weight)
        err = (g.float().cpu() - ref).norm().item()
        assert err <= 0.1 * ref.norm().item() or err <= 2e-3 * gnorm, (k, rel(g, ref), err, gnorm)


@pytest.mark.parametrize("name,p", [("f_demo", 0.3), ("f_small", 0.1), ("f_hs32", 0.2)])
def test_dropout_step_matches_oracle_masks(name, p):
    """Training-mode step with dropout p: the HIP path against the CPU oracle run with the SAME
    hash masks (oracle.HashDropout restates the kernels' counter hash bit-for-bit), at the bf16
    tolerances above. Parity of the mask law itself: tests/test_oracle.py (keep rate 1-p)."""
    import mmt_oracle as O
    z, meta, cfg, sd, idx, tgt = model_fixture(name)
    m = build(meta, sd, dropout=p)
    m.train()
    torch.manual_seed(7)
    logits, losses = m([t.cuda() for t in idx], [t.cuda() for t in tgt])
    sum(losses).backward()
    torch.cuda.synchronize()
    cfg.dropout = p
    hd = O.HashDropout(m.last_dropout_seed, p)
    r_logits, r_losses, r_grads = O.forward_backward(sd, cfg, idx, tgt, hash_dropout=hd)
    got = torch.stack([l.detach().cpu() for l in losses])
    ref = torch.stack(r_losses)
    assert torch.allclose(got, ref, rtol=5e-3, atol=5e-3), (got, ref)
    # the masks really act: the step lands far closer to the hash-masked oracle than to the
    # dropout-free one (a loss comparison is too weak at init scale on the tiny fixtures)
    cfg.dropout = 0.0
    _, _, n_grads = O.forward_backward(sd, cfg, idx, tgt)
    cfg.dropout = p
    for i in range(cfg.M):
        assert rel(logits[i], r_logits[i]) < 2e-2, i
    names = [n for n, _ in m.named_reference_tensors()]
    allg, allr = [], []
    for k, g in zip(names, _grad_views(m)):
        if r_grads.get(k) is not None and g is not None and g.numel():
            allg.append(g.flatten().cpu())
            allr.append(r_grads[k].flatten())
    assert rel(torch.cat(allg), torch.cat(allr)) < 3e-2
    alln = torch.cat([n_grads[k].flatten() for k, g in zip(names, _grad_views(m))
                      if r_grads.get(k) is not None and g is not None and g.numel()])
    assert rel(torch.cat(allg), alln) > 3 * max(rel(torch.cat(allg), torch.cat(allr)), 1e-2)
    # eval mode: no dropout, the golden (reference) logits again
    m.eval()
    with torch.no_grad():
        lg, _ = m([t.cuda() for t in idx], [t.cuda() for t in tgt])
    for i in range(cfg.M):
        assert rel(lg[i], torch.from_numpy(z[f"logits.{i}"])) < 2e-2, i


@pytest.mark.parametrize("C,H,T,cross,p", [(128, 2, 160, [False, True], 0.1), (128, 2, 300, [True, False], 0.2),
                                             (128, 2, 512, [False, False], 0.1)])
def test_dropout_fused_hs64_backward_matches_oracle(C, H, T, cross, p):
    """The one-pass hs-64 attention backward (mmt_attn_set_ring bit 5; self-attention at T <= 512)
    under dropout: the keep-bit records it reads per (query tile, key tiles 0..qt) against the
    oracle's hash masks, as the multichunk test below does for the two-pass kernels."""
    L = ML.lib()
    L.mmt_attn_set_ring.restype = ctypes.c_int
    old = L.mmt_attn_set_ring(47)
    try:
        test_dropout_multichunk_masks_match_oracle(C, H, T, cross, p)
    finally:
        L.mmt_attn_set_ring(old)


@pytest.mark.parametrize("ring", [79 | 128, 79, 15])
@pytest.mark.parametrize("C,H,T,cross,p", [(64, 2, 256, [True, False], 0.1), (64, 2, 37, [False, True], 0.2),
                                             (96, 3, 200, [True, False], 0.1), (64, 2, 31, [True, False], 0.1),
                                             (64, 2, 256, [True, False, True, False], 0.1),
                                             (64, 2, 77, [False, True, True], 0.2)])
def test_dropout_hs32_one_pass_backward_matches_oracle(C, H, T, cross, p, ring):
    """The one-pass hs-32 attention backward (mmt_attn_set_ring bit 6, default; T <= 256 and one KV
    stream, so both the self-attention and -- at two modalities -- the one-stream cross-attention take
    it; with 3-4 modalities and bit 7 the cross-attention walks 2-3 KV streams with its dQ summed in the
    engine's fp32 scratch) under dropout against the oracle's hash masks, at full and ragged T; ring 15 is the
    two-pass pair on the same cases. With the one-pass kernel the self-attention also runs the Q/K/V
    stage-2 backward in its epilogue (mmt_set_attn_qkv2 bit 0, default), so these cases check dh1 / dW2 /
    db1 from there too."""
    L = ML.lib()
    old = L.mmt_attn_set_ring(ring)
    try:
        test_dropout_multichunk_masks_match_oracle(C, H, T, cross, p)
    finally:
        L.mmt_attn_set_ring(old)


@pytest.mark.parametrize("C,H,T,cross,p", [(64, 2, 288, [True, False], 0.2), (128, 2, 160, [False, True], 0.1),
                                             (128, 2, 300, [True, False], 0.1)])
def test_dropout_multichunk_masks_match_oracle(C, H, T, cross, p, L=1):
    """Dropout at sequence lengths past one LDS chunk (hs 32: 256 rows, hs 64: 128 rows; the hs-64 dQ
    pass: 256 rows, so T = 300 takes it past one) with a ragged last tile: the keep bits of attn_mask_kernel, staged chunk by chunk in all three
    attention kernels, against the oracle's hash masks (random init, the oracle as reference)."""
    import mmt_oracle as O
    import model as mmt_model
    V = [13, 7, 5, 11][:len(cross)]
    ocfg = O.OracleConfig(C, H, L, T, V, cross)
    g = torch.Generator().manual_seed(5)
    sd = O.init_params(ocfg, g)
    config_utils._config_cache = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "dropout": p,
                                  "device": "cuda", "batch_size": 2, "eval_iters": 1}
    params = [[None] * 8 + [c] + [None] * 3 for c in cross]
    m = mmt_model.MultimodalTransformer(len(V), V, params).to("cuda")
    full = {k: v for k, v in m.state_dict().items() if k.endswith("tril")}
    full.update(sd)
    m.load_state_dict(full, strict=True)
    m.train()
    idx = [torch.randint(0, v, (2, T), generator=g) for v in V]
    tgt = [torch.randint(0, v, (2, T), generator=g) for v in V]
    logits, losses = m([t.cuda() for t in idx], [t.cuda() for t in tgt])
    sum(losses).backward()
    torch.cuda.synchronize()
    ocfg.dropout = p
    r_logits, r_losses, r_grads = O.forward_backward(sd, ocfg, idx, tgt, hash_dropout=O.HashDropout(m.last_dropout_seed, p))
    ocfg.dropout = 0.0
    _, _, n_grads = O.forward_backward(sd, ocfg, idx, tgt)
    got = torch.stack([l.detach().cpu() for l in losses])
    assert torch.allclose(got, torch.stack(r_losses), rtol=5e-3, atol=5e-3)
    for i in range(len(V)):
        assert rel(logits[i], r_logits[i]) < 2e-2, i
    names = [n for n, _ in m.named_reference_tensors()]
    pairs = [(g_.flatten().cpu(), r_grads[k].flatten(), n_grads[k].flatten())
             for k, g_ in zip(names, _grad_views(m)) if r_grads.get(k) is not None and g_ is not None and g_.numel()]
    allg = torch.cat([a for a, _, _ in pairs])
    allr = torch.cat([b for _, b, _ in pairs])
    alln = torch.cat([c for _, _, c in pairs])
    assert rel(allg, allr) < 3e-2
    assert rel(allg, alln) > 3 * max(rel(allg, allr), 1e-2)  # the masks act


@pytest.mark.parametrize("L", [5, 12])
def test_dropout_deep_masks_match_oracle(L):
    """Keep bits of every layer against the oracle at depth: 5 layers make the later layers' bits beside
    layer 0 (one fork, joined at layer 1); from 12 layers on the engine makes layer l + 1's bits while
    layer l computes (one fork and join per layer, run_forward's mask_ahead)."""
    test_dropout_multichunk_masks_match_oracle(64, 2, 72, [True, False, True], 0.1, L=L)


@pytest.mark.parametrize("name", ["f_small", "f_hs32"])
def test_short_sequence_inference_matches_oracle(name):
    """T < block_size without targets (inference; generate's early steps): the right-padded run's
    logits at the real positions against the oracle run at that length (model.py:380-402)."""
    import mmt_oracle as O
    z, meta, cfg, sd, idx, tgt = model_fixture(name)
    m = build(meta, sd)
    m.eval()
    Ts = meta["block_size"] // 2 + 3
    short = [t[:, :Ts] for t in idx]
    with torch.no_grad():
        lg, none = m([t.cuda() for t in short])
    assert none is None
    ref, _ = O.forward(sd, cfg, short)
    for i in range(cfg.M):
        assert tuple(lg[i].shape) == tuple(ref[i].shape)
        assert rel(lg[i], ref[i]) < 2e-2, i
    with pytest.raises(NotImplementedError):
        m([t.cuda() for t in short], [t[:, :Ts].cuda() for t in tgt])


def test_generate_appends_crops_and_aligns():
    """generate (model.py:404-446): samples appended to the target modality past block_size (the
    context is cropped), the other modalities padded with their last token, prefixes unchanged."""
    z, meta, cfg, sd, idx, tgt = model_fixture("f_small")
    m = build(meta, sd)
    m.eval()
    torch.manual_seed(0)
    start = [t[:, :10].cuda() for t in idx]
    n_new = meta["block_size"] + 8 - 10
    out = m.generate(start, max_new_tokens=n_new, modality_to_generate=1)
    B = start[0].shape[0]
    for i, o in enumerate(out):
        assert tuple(o.shape) == (B, meta["block_size"] + 8), i
        assert torch.equal(o[:, :10], start[i]), i
    g = out[1][:, 10:]
    assert int(g.min()) >= 0 and int(g.max()) < meta["V"][1]
    for i in (0, 2, 3):
        assert torch.equal(out[i][:, 10:], start[i][:, -1:].expand(B, n_new)), i


def _grad_views(m):
    for _, g in m.reference_grad_views():
        yield g


@pytest.mark.parametrize("name,stock", [("f_demo", False), ("f_m1", False), ("f_tiny_v", False),
                                        ("f_demo", True), ("f_m1", True)])
def test_adamw_steps_match_reference(name, stock):
    """The fused mmt_optim.AdamW and the reference's own line, stock torch.optim.AdamW(
    m.parameters(), lr) (reference main.py:464), against the reference's parameters after 1 and 3
    steps; the never-used CrossAttention parameters of f_m1 (M == 1) must stay untouched by both
    (their .grad stays None, so no decay)."""
    import mmt_optim
    z, meta, cfg, sd, idx, tgt = model_fixture(name)
    m = build(meta, sd)
    opt = (torch.optim.AdamW if stock else mmt_optim.AdamW)(m.parameters(), lr=1e-3)
    idx_d = [t.cuda() for t in idx]
    tgt_d = [t.cuda() for t in tgt]
    for step in range(1, 4):
        _, losses = m(idx_d, tgt_d)
        opt.zero_grad(set_to_none=True)
        sum(losses).backward()
        opt.step()
        tag = {1: "after1", 3: "after3"}.get(step)
        if tag:
            # Adam normalises each gradient element, so a bf16-level gradient difference can move a
            # tiny-gradient element by up to 2*lr per step: compare the UPDATE (p_t - p_0) as a whole
            # (rel-L2) and bound every element by the largest possible Adam move.
            torch.cuda.synchronize()
            d_got, d_ref = [], []
            for k, v in m.named_reference_tensors():
                ref = torch.from_numpy(z[f"{tag}.{k}"])
                p0 = torch.from_numpy(z[f"param.{k}"])
                d_got.append((v.detach().cpu() - p0).flatten())
                d_ref.append((ref - p0).flatten())
                if v.numel():
                    assert (v.detach().cpu() - ref).abs().max().item() <= 2.05e-3 * step + 1e-6, (tag, k)
            assert rel(torch.cat(d_got), torch.cat(d_ref)) < 0.15, tag
    # unused CrossAttention parameters (M == 1) must be untouched: no decay, no update
    for k in meta["grad_none"]:
        v = dict(m.named_reference_tensors())[k]
        assert torch.equal(v.detach().cpu(), torch.from_numpy(z[f"param.{k}"])), k
    with torch.no_grad():
        _, losses = m(idx_d, tgt_d)
    got = torch.stack([l.cpu() for l in losses])
    assert torch.allclose(got, torch.from_numpy(z["losses_after3"]), rtol=5e-3, atol=5e-3)


def test_state_dict_roundtrip_reference_keys():
    z, meta, cfg, sd, idx, tgt = model_fixture("f_small")
    m = build(meta, sd)
    out = m.state_dict()
    assert list(out.keys()) == list(meta["state_dict_keys"]) or sorted(out.keys()) == sorted(meta["state_dict_keys"])
    for k, v in sd.items():
        assert torch.equal(out[k].cpu(), v), k
        assert list(out[k].shape) == meta["state_dict_shapes"][k]


@pytest.mark.parametrize("name", ["f_small", "f_hs32", "f_demo"])
def test_kv_cache_decode_matches_full_forward(name):
    """KV-cache decode (mmt_decode_step, used by generate): after a prefill forward over positions
    < P, one position per step up to block_size - 1; its logits against the full forward of the
    whole sequence (causal: the same positions) and against the CPU oracle. f_small / f_demo have
    cross-attention (multi-stream decode attention over the appended cross K/V rows)."""
    import mmt_oracle as O
    z, meta, cfg, sd, idx, tgt = model_fixture(name)
    m = build(meta, sd)
    m.eval()
    T = meta["block_size"]
    P = max(1, T // 2 - 1)
    seq = [t.cuda() for t in idx]
    with torch.no_grad():
        m([s[:, :P] for s in seq])  # prefill
        dec = [m._decode_step([s[:, t] for s in seq], t) for t in range(P, T)]
        full, _ = m(seq)
    ref, _ = O.forward(sd, cfg, idx)
    for i in range(cfg.M):
        got = torch.stack([d[i] for d in dec], dim=1).cpu()  # [B, T-P, V]
        assert rel(got, full[i][:, P:T]) < 1e-2, (i, rel(got, full[i][:, P:T]))
        assert rel(got, ref[i][:, P:T]) < 2e-2, (i, rel(got, ref[i][:, P:T]))
    with pytest.raises(Exception):
        m._decode_step([s[:, 0] for s in seq], T)  # position outside the block


@pytest.mark.parametrize("hs", [8, 16, 24, 32, 48, 64])
def test_kv_cache_decode_every_head_size(hs):
    """The decode attention kernel (attn_decode_kernel<HS>) and the single-row GEMMs at every
    supported head size, incl. hs 64 (target shape, C4) and 24 / 48: decode logits of
    positions P..T-1 after a prefill vs the full forward of the whole sequence (itself parity-checked
    against the reference) and vs the CPU oracle; 3 modalities, cross-attention on modality 0."""
    import mmt_oracle as O
    H, L, T, B = 2, 2, 40, 3
    C = H * hs
    V = [37, 5, 11]
    cross = [True, False, False]
    cfg = O.OracleConfig(C, H, L, T, V, cross)
    g = torch.Generator().manual_seed(hs)
    sd = O.init_params(cfg, g)
    for k in sd:  # non-trivial LayerNorm / bias values so every path carries signal
        if k.endswith("bias") or "ln" in k or "norm" in k:
            sd[k] = sd[k] + 0.05 * torch.randn(sd[k].shape, generator=g)
    tril = [f"blocks.{l}.{kind}.{i}.heads.{h}.tril" for l in range(L) for i in range(len(V))
            for kind in ("sa_layers", "cross_attention_layers") for h in range(H)
            if kind == "sa_layers" or cross[i]]
    meta = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "B": B, "V": V, "cross": cross,
            "state_dict_keys": list(sd.keys()) + tril}
    m = build(meta, sd)
    m.eval()
    idx = [torch.randint(0, v, (B, T), generator=g) for v in V]
    P = 7
    seq = [t.cuda() for t in idx]
    with torch.no_grad():
        m([s[:, :P] for s in seq])
        dec = [m._decode_step([s[:, t] for s in seq], t) for t in range(P, T)]
        full, _ = m(seq)
    ref, _ = O.forward(sd, cfg, idx)
    for i in range(len(V)):
        got = torch.stack([d[i] for d in dec], dim=1).cpu()
        assert rel(got, full[i][:, P:T]) < 1e-2, (hs, i, rel(got, full[i][:, P:T]))
        assert rel(got, ref[i][:, P:T]) < 2e-2, (hs, i, rel(got, ref[i][:, P:T]))


def test_decode_refuses_dropout_prefill():
    """mmt_decode_step promises eval semantics (include/mmt.h): a cache left by a training forward
    that sampled dropout is refused with MMT_ERR_STATE."""
    z, meta, cfg, sd, idx, tgt = model_fixture("f_small")
    m = build(meta, sd, dropout=0.1)
    m.train()
    seq = [t.cuda() for t in idx]
    with torch.no_grad():
        m(seq, [t.cuda() for t in tgt])
        with pytest.raises(Exception, match="dropout"):
            m._decode_step([s[:, 1] for s in seq], 1)
        m.eval()
        m([s[:, :4] for s in seq])  # an eval prefill re-arms the cache
        m._decode_step([s[:, 4] for s in seq], 4)


def test_generate_kv_cache_greedy_matches_reforward():
    """generate with the KV cache against the reference's re-forward per token (use_cache=False),
    greedy sampling on a model with peaked output heads (so argmax is stable to bf16 noise), past
    the end of the block (the cache path hands over to the re-forward once positions shift)."""
    z, meta, cfg, sd, idx, tgt = model_fixture("f_small")
    sd = dict(sd)
    for k in list(sd):
        if k.startswith("post_block.soft_score_layers.") and k.endswith(".2.weight"):
            sd[k] = sd[k] * 60.0
    m = build(meta, sd)
    m.eval()
    T = meta["block_size"]
    start = [t[:, :5].cuda() for t in idx]
    greedy = lambda probs: probs.argmax(dim=-1, keepdim=True)  # noqa: E731
    n_new = T + 3 - 5
    a = m.generate(start, max_new_tokens=n_new, modality_to_generate=2, use_cache=True, sample_fn=greedy)
    b = m.generate(start, max_new_tokens=n_new, modality_to_generate=2, use_cache=False, sample_fn=greedy)
    for i in range(cfg.M):
        assert tuple(a[i].shape) == (start[0].shape[0], T + 3)
        assert torch.equal(a[i], b[i]), i
