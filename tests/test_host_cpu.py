"""Host-side logic of the drop-in training_utils (no GPU): the product's
generate_batch_starting_indices against the reference's own outputs (bit-identical under a
seeded torch RNG: same torch.randint calls, vectorised file mapping), its argument validation,
and the vectorised host jitter against the reference's law (reference data_utils.py:342-351)."""
import numpy as np
import pytest
import torch

import training_utils as TU
from golden_io import load


def test_batch_indices_bit_identical_to_reference():
    z, meta = load("batch_indices")
    for ci, c in enumerate(meta["cases"]):
        torch.manual_seed(meta["seed"] + ci)
        ix = TU.generate_batch_starting_indices(c["data_size"], c["block_size"], c["batch_size"], c["split"],
                                                c["file_lengths"], c["is_percents"])
        np.testing.assert_array_equal(ix.numpy(), z[f"ix.{ci}"])


@pytest.mark.parametrize("args,exc", [
    ((0, 8, 4, "train", [10], False), TypeError),
    ((100, 100, 4, "train", [100], False), ValueError),
    ((100, 8, 0, "train", [100], False), TypeError),
    ((100, 8, 4, "test", [100], False), ValueError),
    ((100, 8, 4, "train", [], False), TypeError),
    ((100, 8, 4, "train", [100], 1), TypeError),
    ((100, 60, 4, "train", [50, 50], False), ValueError),
])
def test_batch_indices_validation(args, exc):
    with pytest.raises(exc):
        TU.generate_batch_starting_indices(*args)


@pytest.mark.parametrize("r", [1, 2, 3])
def test_host_jitter_law(r):
    V = 30
    rng = np.random.default_rng(r)
    x0 = rng.integers(0, V, size=300_000)
    x = x0.copy()
    TU.jitter_(x, r, V, np.random.default_rng(7))
    d = x - x0
    elig = (x0 > r) & (x0 < V - r)
    assert np.all(d[~elig] == 0) and np.all(np.abs(d) <= r)
    freq = np.bincount(d[elig] + r, minlength=2 * r + 1) / elig.sum()
    np.testing.assert_allclose(freq, 1.0 / (2 * r + 1), atol=5e-3)
    with pytest.raises(ValueError):
        TU.jitter_(x, 4, V, np.random.default_rng(0))
