"""get_batch / estimate_loss as main.py drives them, against the reference (fixture f_loop, made
by tests/golden/gen_golden.py with the reference's training_utils.py / data_utils.py / model.py):

  random.seed, torch.manual_seed; get_batch('train', 1) x2; estimate_loss (eval_iters 2: two
  train and two val batches, is_training 0); get_batch('train', 1)

The product's exact host path reproduces every batch and the walked training sets bit for bit,
i.e. the reference's consumption of Python's `random` (the +-1 walk, data_utils.py:342-351) and of
torch's CPU generator (start indices, training_utils.py:104,150). On the GPU the model runs
training forwards / backwards with dropout in between (it must not touch either stream), and
estimate_loss's result is compared with the reference's at the bf16 tolerance (loss rel 5e-3;
the directional counts of 6 predictions per modality within one).
"""
import contextlib
import io
import random
import re

import numpy as np
import pytest
import torch

import config_utils
import training_utils as TU
from golden_io import load, model_fixture


def _setup(device, dropout=0.0, mode="host"):
    z, meta = load("f_loop")
    M = len(meta["V"])
    zs, ms = load("f_small")
    config_utils._config_cache = {"n_embd": ms["n_embd"], "n_head": ms["n_head"], "n_layer": ms["n_layer"],
                                  "block_size": meta["T"], "dropout": dropout, "device": device,
                                  "batch_size": meta["B"], "eval_iters": meta["eval_iters"],
                                  "output_file_name": "", "project_file_path": ""}
    TU.all_train_sets = [list(map(int, z[f"train0.{i}"])) for i in range(M)]
    TU.all_val_sets = [torch.from_numpy(z[f"val.{i}"].copy()) for i in range(M)]
    TU.all_vocabularies = meta["vocabs"]
    TU.all_modality_params = meta["params"]
    TU.all_file_info = None
    TU.file_lengths = meta["file_lengths"]
    TU.num_modalities = M
    TU.is_percents = True
    TU.use_device_batcher = mode != "host"
    TU.batcher_mode = "exact" if mode == "exact" else "hash"
    TU._device_batcher[0] = None
    random.seed(meta["seed"])
    torch.manual_seed(meta["seed"])
    return z, meta, M


def _check(z, M, c, xb, yb):
    for i in range(M):
        np.testing.assert_array_equal(xb[i].cpu().numpy(), z[f"x{c}.{i}"], err_msg=f"call {c} x modality {i}")
        np.testing.assert_array_equal(yb[i].cpu().numpy(), z[f"y{c}.{i}"], err_msg=f"call {c} y modality {i}")


def test_host_get_batch_bit_exact_over_steps():
    z, meta, M = _setup("cpu")
    try:
        for c in range(2):
            _check(z, M, c, *TU.get_batch("train", 1))
        for split in ("train", "val"):  # estimate_loss's draws (is_training 0: no walk)
            for _ in range(meta["eval_iters"]):
                TU.get_batch(split, 0)
        _check(z, M, 2, *TU.get_batch("train", 1))
        for i in range(M):
            np.testing.assert_array_equal(np.asarray(TU.all_train_sets[i]), z[f"train_end.{i}"])
    finally:
        TU.use_device_batcher = True
        TU.batcher_mode = "hash"


def _counts(lines):
    out = []
    for ln in lines:
        m_ = re.search(r"(\d+)/(\d+) \(", ln)
        if m_:
            out.append((int(m_.group(1)), int(m_.group(2))))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["host", "exact"])
def test_gpu_loop_get_batch_and_estimate_loss_match_reference(mode):
    """mode "host": the exact host batcher; "exact": the device-exact batcher (MT19937 on the GPU,
    the walk as prefix-sum kernels): the same bit-exact batches, walked lists and Python state."""
    import model as mmt_model
    z, meta, M = _setup("cuda", dropout=0.1, mode=mode)
    zs, ms, cfg, sd, _, _ = model_fixture("f_small")
    try:
        m = mmt_model.MultimodalTransformer(M, meta["V"], meta["params"]).to("cuda")
        full = {k: v for k, v in m.state_dict().items() if k.endswith("tril")}
        full.update(sd)
        m.load_state_dict(full, strict=True)
        TU.m = m
        random.seed(meta["seed"])
        torch.manual_seed(meta["seed"])
        for c in range(2):
            xb, yb = TU.get_batch("train", 1)
            _check(z, M, c, xb, yb)
            m.train()
            _, losses = m(xb, yb)  # dropout 0.1: must not consume the CPU streams
            sum(losses).backward()
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            est = TU.estimate_loss(0, 10)
        np.testing.assert_allclose([est["train"], est["val"]], z["est"], rtol=5e-3)
        got = _counts(buf.getvalue().splitlines())
        ref = _counts(meta["printed"])
        assert len(got) == len(ref) == 2 * M
        for (a, n), (b, n_ref) in zip(got, ref):
            assert n == n_ref and abs(a - b) <= 1, (got, ref)
        _check(z, M, 2, *TU.get_batch("train", 1))
        TU.sync_host_state()
        for i in range(M):
            np.testing.assert_array_equal(np.asarray(TU.all_train_sets[i]), z[f"train_end.{i}"])
    finally:
        TU.use_device_batcher = True
        TU.batcher_mode = "hash"
        TU._device_batcher[0] = None
        TU.m = None
