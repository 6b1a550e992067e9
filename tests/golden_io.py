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
# BASELINE-config-sized fixtures: parameters are NOT stored (tens of MB); both the generator and
# the tests rebuild them with recipe_state_dict from the key list + seed kept in the fixture
SCALE_FIXTURES = ["f_c1", "f_m8", "f_t1024", "f_t4096"]


def recipe_state_dict(keys_shapes, seed):
    """Deterministic parameters for the scale fixtures, drawn key by key in state_dict order from
    one seeded torch generator: Linear / Embedding weights and biases N(0, 0.02^2) (the reference
    init, model.py:372-378, with non-zero biases so their paths are exercised), LayerNorm weights
    1 + N(0, 0.1^2) and biases N(0, 0.05^2)."""
    g = torch.Generator().manual_seed(int(seed))
    out = {}
    for k, shp in keys_shapes:
        shp = tuple(int(s) for s in shp)
        x = torch.randn(shp, generator=g, dtype=torch.float32)
        is_ln = len(shp) == 1 and any(c.startswith("ln") or "norm" in c for c in k.split("."))
        if is_ln and k.endswith(".weight"):
            out[k] = 1.0 + 0.1 * x
        elif is_ln:
            out[k] = 0.05 * x
        else:
            out[k] = 0.02 * x
    return out


def scale_fixture(name):
    """(z, meta, cfg, sd, idx, tgt) of a scale fixture, parameters rebuilt by the recipe."""
    import mmt_oracle as O
    z, meta = load(name)
    cfg = O.OracleConfig(meta["n_embd"], meta["n_head"], meta["n_layer"], meta["block_size"], meta["V"], meta["cross"])
    ks = [(k, meta["state_dict_shapes"][k]) for k in meta["state_dict_keys"] if not k.endswith("tril")]
    sd = recipe_state_dict(ks, meta["param_seed"])
    idx = [torch.from_numpy(z[f"idx.{i}"].copy()) for i in range(cfg.M)]
    tgt = [torch.from_numpy(z[f"tgt.{i}"].copy()) for i in range(cfg.M)]
    return z, meta, cfg, sd, idx, tgt


def c0_run_oracle_replay(emulate_bf16=False):
    """Replay the reference's recorded C0 demo run (f_c0run: the training batches it drew, its
    initial parameters) through the oracle: forward + backward + oracle AdamW per training step.
    Returns (per-step losses [steps, M], update rel-L2, params rel-L2) against the reference's
    recorded losses and final checkpoint."""
    import mmt_oracle as O
    z, meta = load("f_c0run")
    ma, tp = meta["config"]["model_architecture"], meta["config"]["training_parameters"]
    V = meta["V"]
    M = len(V)
    cfg = O.OracleConfig(ma["n_embd"], ma["n_head"], ma["n_layer"], tp["block_size"], V, [p[8] for p in meta["params"]])
    init = {k[len("init."):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("init.")}
    fin = {k[len("final."):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("final.")}
    p = {k: v.clone() for k, v in init.items()}
    state, losses = {}, []
    for s, c in enumerate([c for c, (_, tr) in enumerate(meta["calls"]) if tr == 1]):
        xb = [torch.from_numpy(z[f"x{c}.{i}"]) for i in range(M)]
        yb = [torch.from_numpy(z[f"y{c}.{i}"]) for i in range(M)]
        _, ls, g = O.forward_backward(p, cfg, xb, yb, emulate_bf16=emulate_bf16)
        losses.append([float(l) for l in ls])
        O.adamw_step(p, g, state, s + 1, lr=tp["learning_rate"])
    ks = sorted(fin)
    got = torch.cat([p[k].flatten() for k in ks])
    ref = torch.cat([fin[k].flatten() for k in ks])
    i0 = torch.cat([init[k].flatten() for k in ks])
    upd = (((got - i0) - (ref - i0)).norm() / (ref - i0).norm()).item()
    return np.array(losses), upd, ((got - ref).norm() / ref.norm()).item()
