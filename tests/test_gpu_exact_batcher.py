"""Device-exact get_batch (training_utils.ExactDeviceBatcher: Python's MT19937 run on the GPU,
the +-r walk as prefix-sum kernels, csrc/mmt_batch.hip mmt_exact_gen / mmt_exact_walk) against
the exact host batcher, itself bit-exact with the reference (tests/test_batch_loop.py, fixture
f_loop; tests/test_host_cpu.py): over many training steps with evaluation draws in between, on
streams with every rand size (1, 2, 3 and None, incl. the walk's absorbing edges), every batch
is identical, and after sync_host_state() so are the walked training lists and Python's `random`
state (random.getstate() tuples equal)."""
import random

import numpy as np
import pytest
import torch

import config_utils
import training_utils as TU

pytestmark = pytest.mark.gpu


def _install(seed, n_rows, V, rand, file_lengths, B, T):
    rs = np.random.RandomState(seed)
    M = len(V)
    n_train = int(n_rows * 0.9)
    streams = [rs.randint(0, v, size=n_rows) for v in V]
    config_utils._config_cache = {"n_embd": 32, "n_head": 4, "n_layer": 1, "block_size": T, "dropout": 0.0,
                                  "device": "cuda", "batch_size": B, "eval_iters": 2,
                                  "output_file_name": "", "project_file_path": ""}
    TU.all_train_sets = [list(map(int, s[:n_train])) for s in streams]
    TU.all_val_sets = [torch.from_numpy(s[n_train:].copy()) for s in streams]
    TU.all_vocabularies = [list(range(v)) for v in V]
    params = []
    for i in range(M):
        p = [None] * 12
        p[2] = rand[i]
        p[9] = f"m{i}"
        params.append(p)
    TU.all_modality_params = params
    TU.all_file_info = None
    TU.file_lengths = file_lengths
    TU.num_modalities = M
    TU.is_percents = False


def _run(mode, steps, seed):
    TU.use_device_batcher = mode != "host"
    TU.batcher_mode = "exact" if mode == "exact" else "hash"
    TU._device_batcher[0] = None
    random.seed(seed)
    torch.manual_seed(seed)
    out = []
    for s in range(steps):
        xb, yb = TU.get_batch("train", 1)
        out.append([x.cpu().numpy() for x in xb] + [y.cpu().numpy() for y in yb])
        if s % 5 == 4:  # evaluation draws (no walk) on both splits
            for split in ("train", "val"):
                xb, yb = TU.get_batch(split, 0)
                out.append([x.cpu().numpy() for x in xb])
    TU.sync_host_state()
    return out, [np.asarray(t).copy() for t in TU.all_train_sets], random.getstate()


@pytest.mark.parametrize("rand", [[True, True, True, True], [1, 2, None, 3]])
def test_device_exact_matches_host_exact(rand):
    V = [900, 13, 144, 17]  # rand 3 walks only 3 < x < V - 3: V = 7 would leave the stream still
    try:
        _install(7, 200_000, V, rand, [60_000, 90_000, 50_000], 16, 64)
        ref = _run("host", 12, 123)
        _install(7, 200_000, V, rand, [60_000, 90_000, 50_000], 16, 64)
        got = _run("exact", 12, 123)
        assert len(got[0]) == len(ref[0])
        for c, (a, b) in enumerate(zip(got[0], ref[0])):
            for u, v in zip(a, b):
                np.testing.assert_array_equal(u, v, err_msg=f"call {c}")
        for i, (a, b) in enumerate(zip(got[1], ref[1])):
            np.testing.assert_array_equal(a, b, err_msg=f"walked stream {i}")
        assert got[2] == ref[2]  # Python's random state, as the reference loop leaves it
        _install(7, 200_000, V, rand, [60_000, 90_000, 50_000], 16, 64)  # the streams before any walk
        moved = [int((a != np.asarray(b)).sum()) for a, b in zip(got[1], TU.all_train_sets)]
        assert all((m > 0) == bool(r) for m, r in zip(moved, rand)), moved
    finally:
        TU.use_device_batcher = True
        TU.batcher_mode = "hash"
        TU._device_batcher[0] = None


def test_device_exact_refuses_foreign_random_use():
    try:
        _install(3, 20_000, [50, 9], [True, True], [20_000], 4, 16)
        TU.use_device_batcher = True
        TU.batcher_mode = "exact"
        TU._device_batcher[0] = None
        random.seed(5)
        TU.get_batch("train", 1)
        random.random()  # someone else draws from the walk's stream
        with pytest.raises(RuntimeError, match="random"):
            TU.get_batch("train", 1)
    finally:
        TU.use_device_batcher = True
        TU.batcher_mode = "hash"
        TU._device_batcher[0] = None
