"""GPU parity of the training-loop kernels around the model (SURVEY.md §8a rows get_batch,
calculate_evaluation_metrics, estimate_loss), through the C-ABI:

  * mmt_eval_direction (calculate_evaluation_metrics, reference training_utils.py:215-330)
    against the reference's own outputs (tests/golden/eval_metrics.npz): win / loss / processed
    counts exact, certainty sums to fp64 rounding;
  * the device batcher (training_utils.py:333-384, data_utils.py:293-358): window gather
    bit-exact against numpy slicing; start indices always inside one file of the split with the
    reference's percent offset, and uniform over the valid positions; the +-r random walk only
    touches eligible elements (r < x < V - r), moves them by at most r with the reference's
    uniform choice over {0, +-1 .. +-r}, and is reproducible per (seed, counter);
  * estimate_loss end to end on a small synthetic dataset (finite losses, the reference's
    log-line format).
The batcher's randomness is a counter hash, not Python's `random`: distributions are pinned,
individual draws are not (documented deviation).
"""
import os

import numpy as np
import pytest
import torch

import mmt_lib as ML
from golden_io import load

pytestmark = pytest.mark.gpu


def test_eval_direction_matches_reference():
    import training_utils as TU
    z, meta = load("eval_metrics")
    vocabs = [[float(v) for v in z["vocab.0"]], [float(v) for v in z["vocab.1"]], meta["vocab2"]]
    logits = [torch.from_numpy(z[f"logits.{i}"]).cuda() for i in range(3)]
    xb = [torch.from_numpy(z[f"xb.{i}"]).cuda() for i in range(3)]
    yb = [torch.from_numpy(z[f"yb.{i}"]).cuda() for i in range(3)]
    params = [[None] * 12 for _ in range(3)]
    for i, pct in enumerate(meta["percent"]):
        params[i][3] = pct
    w, l, c, p = TU.calculate_evaluation_metrics(logits, xb, yb, 3, vocabs, params, None)
    assert w == list(z["wins"]) and l == list(z["losses"]) and p == list(z["processed"]), (w, l, p)
    np.testing.assert_allclose(c, z["certainty"], rtol=1e-6)  # reference sums fp32 .item()s


def test_eval_direction_ties_and_percent_large_vocab():
    """argmax ties resolve to the first index (torch.argmax), percent data uses the value's own
    sign; cross-checked against the oracle restatement at a larger vocabulary."""
    import mmt_oracle as O
    import training_utils as TU
    g = torch.Generator().manual_seed(3)
    B, T, V = 64, 5, 300
    logits = torch.randn(B, T, V, generator=g)
    logits[:8, -1, :] = 0.0  # all-equal rows: first index wins
    logits[8:16, -1, 10] = 5.0
    logits[8:16, -1, 20] = 5.0
    xb = torch.randint(0, V, (B, T), generator=g)
    yb = torch.randint(0, V, (B, T), generator=g)
    vocab = [float(v) for v in np.linspace(-3, 3, V)]
    for pct in (False, True):
        params = [[None] * 12]
        params[0][3] = pct
        w, l, c, p = TU.calculate_evaluation_metrics([logits.cuda()], [xb.cuda()], [yb.cuda()], 1, [vocab], params,
                                                     None)
        rw, rl, rc, rp = O.eval_metrics([logits], [xb], [yb], [vocab], [pct])
        assert (w, l, p) == (rw, rl, rp)
        np.testing.assert_allclose(c, rc, rtol=1e-6)


def _lib():
    return ML.lib()


def test_batch_gather_bit_exact():
    g = np.random.default_rng(0)
    data = [g.integers(0, 900, size=50_000).astype(np.int32) for _ in range(4)]
    dd = [torch.from_numpy(d).cuda() for d in data]
    B, T = 64, 256
    ix = torch.from_numpy(g.integers(0, 50_000 - T - 1, size=B)).cuda()
    xs = [torch.empty(B, T, dtype=torch.long, device="cuda") for _ in range(4)]
    ys = [torch.empty(B, T, dtype=torch.long, device="cuda") for _ in range(4)]
    rc = _lib().mmt_batch_gather(ML.stream_ptr(), 4, ML.ptr_array(dd), ML.ptr(ix), B, T, ML.ptr_array(xs),
                                 ML.ptr_array(ys))
    assert rc == 0
    ixh = ix.cpu().numpy()
    win = ixh[:, None] + np.arange(T + 1)[None, :]
    for m in range(4):
        np.testing.assert_array_equal(xs[m].cpu().numpy(), data[m][win][:, :T])
        np.testing.assert_array_equal(ys[m].cpu().numpy(), data[m][win][:, 1:])


@pytest.mark.parametrize("split,off", [("train", 0), ("train", 1), ("val", 1)])
def test_device_batcher_indices_stay_inside_files(split, off):
    import training_utils as TU
    n_files, per, T, B = 20, 1000, 64, 512
    fl = [per] * n_files
    n = n_files * per
    ntr = int(n * 0.9)
    tr = [np.arange(ntr, dtype=np.int64) % 977]
    va = [torch.arange(n - ntr, dtype=torch.long) % 977]
    bt = TU.DeviceBatcher(tr, va, [1000], [None], fl, bool(off), T, B, "cuda", seed=11)
    size = ntr if split == "train" else n - ntr
    lens = TU._split_file_lengths(size, split, fl)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    valid = np.maximum(0, np.array(lens) - (T + 1) - off + 1)
    counts = np.zeros(len(lens))
    for _ in range(40):
        cum, fs, nf, o = bt.maps[split]
        ix = torch.empty(B, dtype=torch.long, device="cuda")
        assert _lib().mmt_batch_indices(ML.stream_ptr(), B, ML.ptr(cum), ML.ptr(fs), nf, o, 7, bt.counter, ML.ptr(ix)) == 0
        bt.counter += 1
        ixh = ix.cpu().numpy()
        f = np.searchsorted(starts, ixh, side="right") - 1
        assert np.all(ixh >= starts[f] + off)
        assert np.all(ixh + T + 1 <= starts[f] + np.array(lens)[f])   # window [i, i+T] inside file f
        np.add.at(counts, f, 1)
    # uniform over valid positions: file frequencies follow valid counts (chi-square, loose)
    expct = counts.sum() * valid / valid.sum()
    chi2 = ((counts - expct) ** 2 / np.maximum(expct, 1)).sum()
    assert chi2 < 3 * len(lens) + 30, chi2
    # the batcher's own path: x/y are consistent windows
    xs, ys = bt.next(split, 0)
    assert torch.equal(xs[0][:, 1:], ys[0][:, :-1])


@pytest.mark.parametrize("r", [1, 2, 3])
def test_jitter_walk_law(r):
    V = 40
    n = 1 << 20
    g = np.random.default_rng(r)
    x0 = g.integers(0, V, size=n).astype(np.int32)
    t = torch.from_numpy(x0.copy()).cuda()
    assert _lib().mmt_batch_jitter(ML.stream_ptr(), ML.ptr(t), n, r, V, 1234, 5) == 0
    x1 = t.cpu().numpy()
    d = x1.astype(np.int64) - x0
    elig = (x0 > r) & (x0 < V - r)
    assert np.all(d[~elig] == 0)
    assert np.all(np.abs(d) <= r)
    assert np.all((x1 >= 0) & (x1 < V))
    de = d[elig]
    freq = np.bincount(de + r, minlength=2 * r + 1) / de.size
    np.testing.assert_allclose(freq, np.full(2 * r + 1, 1.0 / (2 * r + 1)), atol=4e-3)
    # reproducible per (seed, counter), different across counters
    t2 = torch.from_numpy(x0.copy()).cuda()
    _lib().mmt_batch_jitter(ML.stream_ptr(), ML.ptr(t2), n, r, V, 1234, 5)
    assert torch.equal(t, t2)
    t3 = torch.from_numpy(x0.copy()).cuda()
    _lib().mmt_batch_jitter(ML.stream_ptr(), ML.ptr(t3), n, r, V, 1234, 6)
    assert not torch.equal(t, t3)


def test_estimate_loss_end_to_end(tmp_path):
    import config_utils
    import mmt_data
    import training_utils as TU
    from model import MultimodalTransformer
    data = mmt_data.make_synthetic(n_rows=40_000, n_files=10)
    cfg = {"n_embd": 64, "n_head": 2, "n_layer": 1, "block_size": 32, "dropout": 0.1, "device": "cuda",
           "batch_size": 8, "eval_iters": 3, "output_file_name": "log.txt", "project_file_path": str(tmp_path) + "/"}
    config_utils._config_cache = cfg
    torch.manual_seed(0)
    m = MultimodalTransformer(4, data["vocab_sizes"], data["params"]).to("cuda")
    mmt_data.install(TU, data, m)
    TU._device_batcher[0] = None
    xb, yb = TU.get_batch("train", 1)
    assert len(xb) == 4 and xb[0].shape == (8, 32) and xb[0].device.type == "cuda"
    out = TU.estimate_loss(3, 10)
    assert set(out) == {"train", "val"} and all(np.isfinite(v) for v in out.values())
    assert m.training
    text = open(os.path.join(str(tmp_path), "output", "log.txt")).read()
    assert "DIRECTIONAL PREDICTION Train Set - Close (ranged): Correct=" in text
    assert "DIRECTIONAL PREDICTION Val Set - " in text
