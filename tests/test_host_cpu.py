"""Host-side logic of the drop-in training_utils (no GPU): the product's
generate_batch_starting_indices against the reference's own outputs (bit-identical under a
seeded torch RNG: same torch.randint calls, vectorised file mapping), its argument validation,
and the vectorised host jitter against the reference's law (reference data_utils.py:342-351)."""
import numpy as np
import pytest
import torch

import training_utils as TU
from golden_io import GOLDEN as GOLDEN_DIR, load


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


def test_host_jitter_reproduces_reference_golden():
    """The reference-held walk (tests/golden/jitter.npz: add_rand_to_data_points(data, True, 12)
    after random.seed(5), reference data_utils.py:293-358) through the product's vectorised walk."""
    import random
    z = np.load(f"{GOLDEN_DIR}/jitter.npz")
    random.seed(5)
    a = z["before"].astype(np.int64).copy()
    TU.jitter_exact_([a], [True], [12])
    np.testing.assert_array_equal(a, z["after"])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_host_jitter_bit_exact_with_python_loop(seed):
    """Several streams with rand sizes {True, None, 2, 3} (edges: values at the walk's bounds, a
    stream with no eligible element): same result and same Python `random` state afterwards as the
    reference's per-element random.choice loop (restated by the oracle)."""
    import random
    import mmt_oracle as O
    rng = np.random.default_rng(seed)
    Vs = [12, 5, 40, 9, 3]
    rs = [True, None, 2, 3, 1]
    data = [rng.integers(0, V, size=2000 + 37 * i) for i, V in enumerate(Vs)]
    random.seed(100 + seed)
    st0 = random.getstate()
    ref = [list(map(int, d)) for d in data]
    for d, r, V in zip(ref, rs, Vs):
        if r is not None:
            O.jitter_inplace(d, r, V)
    nxt = random.random()
    random.setstate(st0)
    got = [d.copy() for d in data]
    TU.jitter_exact_(got, rs, Vs)
    for g, r_ in zip(got, ref):
        np.testing.assert_array_equal(g, np.array(r_))
    assert random.random() == nxt
    with pytest.raises(ValueError):
        TU.jitter_exact_([got[0]], [4], [12])
    with pytest.raises(ValueError):
        TU.jitter_exact_([got[0]], [False], [12])  # has_header: false crashes in the reference too
