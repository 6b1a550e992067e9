"""Model-level parity at the BASELINE config sizes on the GPU: the HIP training step against
fixtures produced by the reference itself (tests/golden/gen_golden.py) and against the CPU oracle
(oracle/mmt_oracle.py, pinned to those fixtures by tests/test_oracle.py), run live on the same
parameters and batch:

  f_c1     C1 dims: C=256, H=8 (hs 32), L=6, T=256, V=[900,13,144,5], cross on modality 0, B=2
  f_m8     8 modalities (C3's cross grouping): C=128, H=2 (hs 64), L=2, T=128, cross on 4 of 8, so
           4 query modalities x 7 KV streams per layer, B=2
  f_t1024  f_m8's modalities at C3's sequence length T=1024 (hs 64, L=1, B=1)
  f_t4096  C4's sequence length T=4096 at hs 64 (the 32-chunk attention walk), M=4, L=1, B=1

Tolerances (SURVEY.md §8c bf16 bar, written here): losses rel <= 5e-3; logits of the last 8
positions rel-L2 <= 2e-2; whole-gradient rel-L2 vs the fp32 oracle <= 5e-2 -- or, where the
bf16 floor itself is above that, <= 1.1 x the floor. The floor is measured, not assumed: the
oracle with every matrix product's operands rounded to bf16 (fp32 accumulation; `emulate_bf16`)
is the reference algorithm computed at the precision of the build's MFMA path, and its distance
from the fp32 oracle is what any bf16-operand implementation shows. At C1's six layers it is 5.2 %
(tools/parity_attrib.py; profiles/r3_parity_attrib_*.txt): 99 % of it comes from the forward's
rounding (the FFN GEMMs' inputs, whose ReLU gates and downstream state move the gradient), only
0.5 % from the backward's. Measured on MI355X: whole gradient 5.29 % vs floor 5.21 % (f_c1),
2.98 vs 3.05 (f_m8), 2.29 vs 2.28 (f_t1024), 1.66 vs 1.63 (f_t4096).
Per tensor group (layer x component): |err| <= max(1.5 x the floor's |err|, 1 % of the group's
norm) + 1e-4 x |whole gradient| (the near-zero key-bias gradients are pure cancellation noise).
At one layer the HIP gradient is within 1.5e-2 of the bf16-emulated oracle itself (measured
0.7 % / 0.5 %). Plus the fixture's own checks (every tensor's norm within 10 %, the 2048 sampled
entries within 1.25 x the floor's sampled error) and the losses after one AdamW step (lr 1e-3).
Under dropout (hash masks, oracle reference) the whole gradient rel-L2 <= 4e-2 (f_m8: floor 3.05 %).
"""
import pytest
import torch

import config_utils
from golden_io import scale_fixture

pytestmark = pytest.mark.gpu


def build(meta, sd, dropout=0.0, precision="bf16"):
    config_utils._config_cache = {"n_embd": meta["n_embd"], "n_head": meta["n_head"], "n_layer": meta["n_layer"],
                                  "block_size": meta["block_size"], "dropout": dropout, "device": "cuda",
                                  "batch_size": meta["B"], "eval_iters": 1, "precision": precision}
    import model as mmt_model
    params = [[None] * 8 + [c] + [None] * 3 for c in meta["cross"]]
    m = mmt_model.MultimodalTransformer(len(meta["V"]), meta["V"], params).to("cuda")
    full = dict(sd)
    T = meta["block_size"]
    for k in meta["state_dict_keys"]:
        if k.endswith("tril"):
            full[k] = torch.tril(torch.ones(T, T))
    m.load_state_dict(full, strict=True)
    return m


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def _group(k):
    import re
    m = re.match(r"blocks\.(\d+)\.(\w+?)\.(\d+)\.(.*)", k)
    if not m:
        return ".".join(k.split(".")[:2])
    l, kind, _, rest = m.groups()
    return f"{l}.{kind}." + re.sub(r"kv_projections\.\d+\.", "kv.", re.sub(r"heads\.\d+\.", "", rest))


def check_against_oracle(name, meta, cfg, sd, idx, tgt, grads):
    """Whole-gradient and per-group error of `grads` vs the fp32 oracle, bounded by the bf16 floor."""
    import mmt_oracle as O
    torch.set_num_threads(16)
    _, _, rg = O.forward_backward(sd, cfg, idx, tgt)
    _, _, eg = O.forward_backward(sd, cfg, idx, tgt, emulate_bf16=True)
    names = meta["grad_names"]
    ref = torch.cat([rg[k].flatten() for k in names])
    emu = torch.cat([eg[k].flatten() for k in names])
    got = torch.cat([grads[k].flatten().float().cpu() for k in names])
    floor, err = _rel(emu, ref), _rel(got, ref)
    print(f"{name}: whole-gradient rel-L2 {err:.4f} (bf16 floor {floor:.4f}, vs emulation {_rel(got, emu):.4f})")
    assert err <= max(5e-2, 1.1 * floor), (err, floor)
    if meta["n_layer"] == 1:
        assert _rel(got, emu) < 1.5e-2, _rel(got, emu)
    total = ref.norm().item()
    groups = {}
    for k in names:
        groups.setdefault(_group(k), []).append(k)
    bad = []
    for gname, ks in groups.items():
        r = torch.cat([rg[k].flatten() for k in ks])
        e = (torch.cat([eg[k].flatten() for k in ks]) - r).norm().item()
        d = (torch.cat([grads[k].flatten().float().cpu() for k in ks]) - r).norm().item()
        if d > max(1.5 * e, 1e-2 * r.norm().item()) + 1e-4 * total:
            bad.append((gname, d / max(r.norm().item(), 1e-30), e / max(r.norm().item(), 1e-30)))
    assert not bad, bad[:5]
    return floor, _rel(emu[torch.from_numpy(z_sample_index(name))], ref[torch.from_numpy(z_sample_index(name))])


def z_sample_index(name):
    from golden_io import load
    z, _ = load(name)
    return z["sample_index"]


@pytest.mark.parametrize("name,stock", [("f_c1", False), ("f_m8", True), ("f_t1024", False), ("f_t4096", True)])
def test_scale_step_matches_reference(name, stock):
    import mmt_optim
    from test_oracle import _scale_compare
    z, meta, cfg, sd, idx, tgt = scale_fixture(name)
    m = build(meta, sd)
    m.train()
    idx_d = [t.cuda() for t in idx]
    tgt_d = [t.cuda() for t in tgt]
    opt = (torch.optim.AdamW if stock else mmt_optim.AdamW)(m.parameters(), lr=1e-3)
    logits, losses = m(idx_d, tgt_d)
    opt.zero_grad(set_to_none=True)
    sum(losses).backward()
    torch.cuda.synchronize()
    grads = {k: g for k, g in m.reference_grad_views() if g is not None}
    floor, sample_floor = check_against_oracle(name, meta, cfg, sd, idx, tgt, grads)
    _scale_compare(z, meta, logits, losses, grads, rel_tol=5e-3, grad_tol=0.1,
                   sample_tol=max(5e-2, 1.25 * sample_floor))
    assert int(m.nonfinite_loss_mask().item()) == 0
    opt.step()
    with torch.no_grad():
        _, l1 = m(idx_d, tgt_d)
    got = torch.stack([l.cpu() for l in l1])
    assert torch.allclose(got, torch.from_numpy(z["losses_after1"]), rtol=5e-3, atol=5e-3), got


def test_t4096_fp8_losses_match_reference():
    """C4's fp8 path (MX-fp8 forward GEMMs) over the 4096-long sequence: losses within 2e-2 of the
    reference's fp32 (SURVEY.md §8c fp8 bar), logits rel-L2 within 5e-2; finite gradient."""
    z, meta, cfg, sd, idx, tgt = scale_fixture("f_t4096")
    m = build(meta, sd, precision="fp8")
    assert m.precision == "fp8"
    logits, losses = m([t.cuda() for t in idx], [t.cuda() for t in tgt])
    sum(losses).backward()
    torch.cuda.synchronize()
    got = torch.stack([l.detach().cpu() for l in losses])
    ref = torch.from_numpy(z["losses"])
    assert ((got - ref).abs() / ref).max().item() <= 2e-2, (got, ref)
    for i in range(cfg.M):
        r = torch.from_numpy(z[f"logits_tail.{i}"])
        assert _rel(logits[i][:, -8:, :].cpu(), r) < 5e-2, i
    assert torch.isfinite(m.flat_params.grad).all()


def test_m8_dropout_step_matches_oracle_masks():
    """The 8-modality grouping (4 cross modalities x 7 KV streams, grouped launches of up to 8
    problems) in training mode with dropout 0.1, against the oracle run with the same hash masks."""
    import mmt_oracle as O
    z, meta, cfg, sd, idx, tgt = scale_fixture("f_m8")
    m = build(meta, sd, dropout=0.1)
    m.train()
    torch.manual_seed(3)
    logits, losses = m([t.cuda() for t in idx], [t.cuda() for t in tgt])
    sum(losses).backward()
    torch.cuda.synchronize()
    cfg.dropout = 0.1
    r_logits, r_losses, r_grads = O.forward_backward(sd, cfg, idx, tgt, hash_dropout=O.HashDropout(m.last_dropout_seed, 0.1))
    got = torch.stack([l.detach().cpu() for l in losses])
    assert torch.allclose(got, torch.stack(r_losses), rtol=5e-3, atol=5e-3), (got, r_losses)
    for i in range(cfg.M):
        assert ((logits[i].cpu() - r_logits[i]).norm() / r_logits[i].norm()).item() < 2e-2, i
    pairs = [(g.flatten().cpu(), r_grads[k].flatten()) for k, g in m.reference_grad_views()
             if g is not None and r_grads.get(k) is not None]
    a = torch.cat([p for p, _ in pairs])
    b = torch.cat([q for _, q in pairs])
    assert ((a - b).norm() / b.norm()).item() < 4e-2


def test_nonfinite_loss_flag():
    """Failure detection: a NaN in modality 3's output-head bias makes only that
    modality's loss NaN; the loss kernel raises its bit in the per-forward and the sticky flag."""
    z, meta, cfg, sd, idx, tgt = scale_fixture("f_m8")
    m = build(meta, sd)
    idx_d = [t.cuda() for t in idx]
    tgt_d = [t.cuda() for t in tgt]
    with torch.no_grad():
        m(idx_d, tgt_d)
        assert int(m.nonfinite_loss_mask().item()) == 0
        dict(m.named_reference_tensors())["post_block.soft_score_layers.3.2.bias"][0] = float("nan")
        _, losses = m(idx_d, tgt_d)
        assert torch.isnan(losses[3]).item() and torch.isfinite(losses[0]).item()
        assert int(m.nonfinite_loss_mask().item()) == 1 << 3
        assert int(m.nonfinite_loss_mask(sticky=True, clear=True).item()) == 1 << 3
        assert int(m.nonfinite_loss_mask(sticky=True).item()) == 0


# ------------------------------------------------------------------------------------------------
# full-size property runs of the BASELINE configs: no oracle can run these shapes
# (the reference's per-head tril buffers alone need 4.8 GB at C3 and 129 GB at C4), so the checks
# are size-independent: every loss finite, the non-finite flag 0, the parameters finite, and the
# loss falling over 20 AdamW steps (lr 3e-4, dropout 0.1) on a learnable batch (periodic token
# streams, targets = the next token). Measured: C3 total 31.0 -> 24.0, C4 (fp8) 16.0 -> 12.7.
# ------------------------------------------------------------------------------------------------
FULL = {
    # name: (M, C, H, L, T, B, cross, precision)
    "c3": (8, 512, 8, 12, 1024, 2, [True, True, False, False, True, True, False, False], "bf16"),
    "c4": (4, 1024, 16, 24, 4096, 1, [True, False, False, False], "fp8"),
}


def _train_full(name, prec, steps=20):
    import mmt_optim
    from model import MultimodalTransformer
    M, C, H, L, T, B, cross, _ = FULL[name]
    V = [900, 13, 144, 5] * (M // 4)
    config_utils._config_cache = {"n_embd": C, "n_head": H, "n_layer": L, "block_size": T, "dropout": 0.1,
                                  "device": "cuda", "batch_size": B, "eval_iters": 1, "precision": prec}
    torch.manual_seed(7)
    m = MultimodalTransformer(M, V, [[None] * 8 + [c] + [None] * 3 for c in cross]).to("cuda")
    m.train()
    opt = mmt_optim.AdamW(m.parameters(), lr=3e-4)
    # stream i: token (b * 7 + t * s_i) % V_i, a fixed periodic pattern per modality
    t = torch.arange(T + 1, device="cuda")
    seq = [((torch.arange(B, device="cuda")[:, None] * 7 + t[None, :] * (2 * i + 1)) % v) for i, v in enumerate(V)]
    idx = [s[:, :T].contiguous() for s in seq]
    tgt = [s[:, 1:].contiguous() for s in seq]
    hist = []
    m.nonfinite_loss_mask(sticky=True, clear=True)
    for step in range(steps):
        _, losses = m(idx, tgt)
        opt.zero_grad(set_to_none=True)
        sum(losses).backward()
        opt.step()
        hist.append(torch.stack([l.detach() for l in losses]))
    torch.cuda.synchronize()
    h = torch.stack(hist).cpu()
    flag = int(m.nonfinite_loss_mask(sticky=True).item())
    finite = bool(torch.isfinite(m.flat_params).all().item())
    del m, opt
    torch.cuda.empty_cache()
    return h, flag, finite


def test_full_size_training_property_c3():
    """C3 (bf16): finite, flag 0, and EVERY modality's loss falls (mean of the last 3 steps below the first)."""
    h, flag, finite = _train_full("c3", "bf16")
    print("c3 loss first", h[0].tolist(), "last", h[-1].tolist())
    assert torch.isfinite(h).all() and flag == 0 and finite
    last = h[-3:].mean(0)
    assert last.sum() < 0.9 * h[0].sum() and (last < h[0]).all(), (h[0], h[-1])


def test_full_size_training_property_c4_fp8_vs_bf16():
    """C4 with the MX-fp8 forward GEMMs against the SAME 20 steps in bf16 (same seed, init, batch and dropout
    masks): the fp8 run must learn what the bf16 run learns, per modality.
    Band (stated here, two-sided): every modality's change over the 20 steps in fp8 within 3 % of its start
    loss of the bf16 one; where the bf16 loss falls clearly (by > 2 % of its start), the fp8 loss must also
    fall by at least half as much.
    Why 3 %: the 20-step run is chaotic in both precisions. tools/fp8_drift.py (profiles/r6_fp8_drift.txt)
    repeats it with the same seed (the gradients differ run to run only in the last bits: the order of the
    float atomics of the bias / LayerNorm column sums, tests/test_gpu_determinism.py) and once from an init
    moved by one ulp: the change/start of one modality spreads by up to 1.46 % in fp8 and 1.08 % in bf16
    over those runs, so fp8 - bf16 differences up to ~2 % are noise (measured: at most 1.83 %); the band is
    the sum of the two spreads rounded up. The earlier one-sided 1 % form read a fp8-only divergence into
    two runs of that noise."""
    h8, flag8, fin8 = _train_full("c4", "fp8")
    h16, flag16, fin16 = _train_full("c4", "bf16")
    d8 = h8[-3:].mean(0) - h8[0]
    d16 = h16[-3:].mean(0) - h16[0]
    print("c4 fp8  first", h8[0].tolist(), "last", h8[-1].tolist(), "change", d8.tolist())
    print("c4 bf16 first", h16[0].tolist(), "last", h16[-1].tolist(), "change", d16.tolist())
    for h, flag, fin in ((h8, flag8, fin8), (h16, flag16, fin16)):
        assert torch.isfinite(h).all() and flag == 0 and fin
        assert h[-3:].mean(0).sum() < 0.9 * h[0].sum(), (h[0], h[-1])
    # both runs start from the same parameters: the first losses differ by the fp8 forward's rounding only
    assert ((h8[0] - h16[0]).abs() / h16[0]).max() < 2e-2, (h8[0], h16[0])
    for i in range(h8.shape[1]):
        start = h16[0, i].item()
        assert abs(d8[i] - d16[i]) <= 0.03 * start, (i, d8[i].item(), d16[i].item())
        if d16[i] < -0.02 * start:
            assert d8[i] < 0.5 * d16[i], (i, d8[i].item(), d16[i].item())
