"""Loader for the committed golden fixtures (tests/golden/*.npz, made by gen_golden.py)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta_json"]).decode())
    return z, meta


def model_fixture(name):
    import mmt_oracle as O
    z, meta = load(name)
    cfg = O.OracleConfig(meta["n_embd"], meta["n_head"], meta["n_layer"], meta["block_size"], meta["V"], meta["cross"])
    sd = {k[len("param."):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("param.")}
    M = cfg.M
    idx = [torch.from_numpy(z[f"idx.{i}"].copy()) for i in range(M)]
    tgt = [torch.from_numpy(z[f"tgt.{i}"].copy()) for i in range(M)]
    return z, meta, cfg, sd, idx, tgt


MODEL_FIXTURES = ["f_demo", "f_small", "f_hs32", "f_m1", "f_tiny_v"]
