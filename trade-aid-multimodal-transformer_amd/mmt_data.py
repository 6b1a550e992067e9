"""Synthetic 4-modality market dataset and the glue main.py would normally do.

The reference's data ingest (CSV loading, range/percent/bin processing, vocabulary, split:
main.py:76-376, data_utils.py, file_cache.py) runs once at startup and is outside the hot path;
this module produces the same *kind* of token streams directly with numpy so the training step
can be exercised at scale without network or CSV files:

  100 files x 10,000 rows (file boundaries exercised), per-file geometric random walk close
  price (start ~ U[20, 500], log-return ~ N(0, 0.002)), 10-minute ticks (144 per day), day of
  week 0-4. Modalities, mirroring the reference's config.py:83-86 template:
    0 close  -> range to 2 whole digits, 1 decimal (reference range_numeric_data)  V <= 900, cross on
    1 close  -> per-file percent change, 2 decimals, then 13 exponent-spaced bins     V <= 13
    2 time   -> 144 values                                                             V = 144
    3 dow    -> 5 values                                                               V = 5
Vocabularies are the sorted unique values (numerical_representation, data_utils.py:212-225);
the split is percentage-based (create_train_val_datasets, data_utils.py:228-290): the train set
is a list-like int array, the val set an int64 tensor.
"""
import numpy as np
import torch


def _range_2w1d(x):
    # restates range_numeric_data(num_whole_digits=2, decimal_places=1) for positive inputs
    p = np.floor(np.log10(np.abs(x)))
    v = np.round(x * 10.0 ** (1 - p), 1)
    return np.clip(v, 10.0, 99.9)


def _bins(pct, num_bins=6, exponent=2.2, outlier=0.1):
    # exponent-spaced symmetric bins (the shape of bin_numeric_data's output: num_bins per sign + zero)
    lim = np.percentile(np.abs(pct[pct != 0]), 100 - outlier) if np.any(pct != 0) else 1.0
    edges = lim * (np.arange(1, num_bins + 1) / num_bins) ** exponent
    mag = np.searchsorted(edges, np.abs(pct), side="left") + 1
    mag = np.minimum(mag, num_bins)
    return np.where(pct > 0, mag, np.where(pct < 0, -mag, 0)).astype(np.float64)


def make_synthetic(n_rows=1_000_000, n_files=100, seed=20251017, validation_size=0.1, n_modalities=4):
    rng = np.random.default_rng(seed)
    per = n_rows // n_files
    file_lengths = [per] * n_files
    close = np.empty(n_rows)
    for f in range(n_files):
        s = rng.uniform(20, 500)
        r = rng.normal(0.0, 0.002, size=per)
        close[f * per:(f + 1) * per] = s * np.exp(np.cumsum(r))
    pct = np.empty(n_rows)
    for f in range(n_files):
        c = close[f * per:(f + 1) * per]
        p = np.zeros(per)
        p[1:] = np.round((c[1:] - c[:-1]) / c[:-1] * 100.0, 2)
        pct[f * per:(f + 1) * per] = p
    tick = np.arange(n_rows)
    raw = [_range_2w1d(close), _bins(pct), (tick % 144).astype(np.float64), ((tick // 144) % 5).astype(np.float64)]
    names = ["Close (ranged)", "Close change (%) binned", "Time of day", "Day of week"]
    cross = [True, False, False, False]
    pct_flag = [False, True, False, False]
    if n_modalities == 8:  # C3 stress: the 4 modalities duplicated, cross [T,T,F,F,T,T,F,F]
        raw = raw + raw
        names = names + [n + " (2)" for n in names]
        cross = [True, True, False, False, True, True, False, False]
        pct_flag = pct_flag + pct_flag
    tokens, vocabs, params = [], [], []
    for i, x in enumerate(raw):
        vocab, inv = np.unique(x, return_inverse=True)
        tokens.append(inv.astype(np.int64))
        vocabs.append([float(v) for v in vocab])
        p = [None] * 12
        p[2] = True          # has_header (drives the reference jitter quirk)
        p[3] = pct_flag[i]   # convert_to_percents
        p[8] = cross[i]      # cross_attention
        p[9] = names[i]
        params.append(p)
    n_train = int(n_rows * (1 - validation_size))
    return {
        "train": [t[:n_train].copy() for t in tokens],
        "val": [torch.from_numpy(t[n_train:].copy()) for t in tokens],
        "full": tokens,
        "vocabs": vocabs,
        "params": params,
        "file_lengths": file_lengths,
        "is_percents": any(pct_flag),
        "vocab_sizes": [len(v) for v in vocabs],
    }


def install(training_utils, data, model=None):
    """What reference main.py:387-396 does: inject the dataset globals into training_utils."""
    training_utils.all_full_datasets = data["full"]
    training_utils.all_train_sets = data["train"]
    training_utils.all_val_sets = data["val"]
    training_utils.all_vocabularies = data["vocabs"]
    training_utils.all_modality_params = data["params"]
    training_utils.all_file_info = None
    training_utils.file_lengths = data["file_lengths"]
    training_utils.num_modalities = len(data["vocabs"])
    training_utils.is_percents = data["is_percents"]
    if model is not None:
        training_utils.m = model
