"""Generate golden fixtures by importing the REFERENCE implementation (this container only).

Runs ONLY in the build container where /root/reference exists. It copies the reference to a
scratch directory under /tmp, imports its `model.py` / `training_utils.py` / `data_utils.py`,
injects the config through `config_utils._config_cache` (reference config_utils.py:8-24),
seeds torch + random, and dumps small .npz fixtures next to this script. Only the fixtures
(inputs and expected outputs) are committed; no reference source travels.

Fixtures:
  f_demo   C=32 H=4 L=2 T=4  M=2 V=[57,3]          cross=[T,F]   B=4   (demo dims, C0)
  f_small  C=64 H=4 L=2 T=32 M=4 V=[57,13,24,5]    cross=[T,F,T,F] B=4
  f_hs32   C=64 H=2 L=1 T=64  M=4 V=[57,13,24,5]   cross=[T,F,F,F] B=2  (production head size 32)
  f_m1     C=32 H=4 L=1 T=8  M=1 V=[11]            cross=[T]     B=3   (CA built but unused)
  f_tiny_v C=32 H=2 L=1 T=8  M=3 V=[2,1,7]         cross=[F,T,F] B=2   (V//2 = 1 and 0)

For each: state_dict (fp32), idx/tgt, logits, per-modality losses, grads of sum(losses),
and params after 1 and 3 AdamW steps (lr=1e-3, torch defaults) on the same batch.
Plus: eval-metric fixtures (calculate_evaluation_metrics) and batch-index fixtures
(generate_batch_starting_indices) with a seeded torch generator.

Scale fixtures (model-level parity at the BASELINE configs), parameters NOT stored
(tests/golden_io.recipe_state_dict rebuilds them from the key list and a seed):
  f_c1     C1 dims: C=256 H=8 L=6 T=256 M=4 V=[900,13,144,5] cross=[T,F,F,F] B=2
  f_m8     8 modalities (C3's grouping): C=128 H=2 (hs 64) L=2 T=128 V=[900,13,144,5]x2
           cross=[T,T,F,F,T,T,F,F] B=2 (4 query modalities x 7 KV streams)
  f_t1024  f_m8's modalities at C3's sequence length: C=128 H=2 (hs 64) L=1 T=1024 B=1
  f_t4096  C4's sequence length and head size: C=64 H=1 (hs 64) L=1 T=4096 M=4 cross=[T,F,F,F] B=1
  stored: losses, logits of the last 8 positions, per-tensor gradient L2 norms, sampled gradient
  entries (every tensor's first and last element + 2048 uniform draws over the concatenation), and
  the losses after one AdamW step (lr 1e-3) on the same batch.
Loop fixture (get_batch / estimate_loss as main.py drives them, reference training_utils.py):
  f_loop   f_small's model + a 3-file synthetic dataset, seeded Python `random` and torch: two
           get_batch('train', 1), estimate_loss (eval_iters 2), one more get_batch('train', 1);
           every batch, the estimate_loss result and its printed lines, the walked train sets.

Run fixture (the reference's own main.py, end to end):
  f_c0run  the demo config (C0) with dropout 0.0 and save_model 1, seeded, run as a script: every
           get_batch call, the RNG states and parameters before the first one, every training
           step's losses, stdout, the log file and the final checkpoint.

Usage:  python tests/golden/gen_golden.py [fixture names...]   (default: all)
"""
import json
import os
import random
import shutil
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
SCRATCH = "/tmp/mmt_ref_golden"


def _import_reference():
    if os.path.exists(SCRATCH):
        shutil.rmtree(SCRATCH)
    shutil.copytree(REF, SCRATCH)
    sys.path.insert(0, SCRATCH)
    import torch  # noqa: F401
    import config_utils
    return config_utils


CONFIGS = {
    "f_demo": dict(n_embd=32, n_head=4, n_layer=2, block_size=4, V=[57, 3], cross=[True, False], B=4),
    "f_small": dict(n_embd=64, n_head=4, n_layer=2, block_size=32, V=[57, 13, 24, 5],
                    cross=[True, False, True, False], B=4, steps=False),
    "f_hs32": dict(n_embd=64, n_head=2, n_layer=1, block_size=64, V=[57, 13, 24, 5],
                   cross=[True, False, False, False], B=2, steps=False),
    "f_m1": dict(n_embd=32, n_head=4, n_layer=1, block_size=8, V=[11], cross=[True], B=3),
    "f_tiny_v": dict(n_embd=32, n_head=2, n_layer=1, block_size=8, V=[2, 1, 7], cross=[False, True, False], B=2),
}


def _params_list(cfg):
    # legacy 12-element list layout (reference schema.py:207-250); index 8 = cross_attention
    out = []
    for i, v in enumerate(cfg["V"]):
        p = [None] * 12
        p[2] = True
        p[3] = False
        p[8] = cfg["cross"][i]
        p[9] = f"mod{i}"
        out.append(p)
    return out


def gen_model_fixture(config_utils, name, cfg, seed=1234):
    import torch
    import importlib
    config_utils._config_cache = {
        "n_embd": cfg["n_embd"], "n_head": cfg["n_head"], "n_layer": cfg["n_layer"],
        "block_size": cfg["block_size"], "dropout": 0.0, "device": "cpu",
        "batch_size": cfg["B"], "eval_iters": 1,
    }
    import model as ref_model
    importlib.reload(ref_model)
    torch.manual_seed(seed)
    random.seed(seed)
    torch.set_num_threads(1)
    M = len(cfg["V"])
    m = ref_model.MultimodalTransformer(M, list(cfg["V"]), _params_list(cfg))
    sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    B, T = cfg["B"], cfg["block_size"]
    g = torch.Generator().manual_seed(seed + 1)
    idx = [torch.randint(0, v, (B, T), generator=g) for v in cfg["V"]]
    tgt = [torch.randint(0, v, (B, T), generator=g) for v in cfg["V"]]

    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    out = {}
    for step in range(3):
        logits, losses = m(idx, tgt)
        total = sum(losses)
        opt.zero_grad(set_to_none=True)
        total.backward()
        if step == 0:
            for i in range(M):
                out[f"logits.{i}"] = logits[i].detach().numpy()
            out["losses"] = np.array([l.item() for l in losses], dtype=np.float32)
            for k, p in m.named_parameters():
                if p.grad is not None:
                    out[f"grad.{k}"] = p.grad.detach().numpy().copy()
        opt.step()
        if step == 0 and cfg.get("steps", True):
            for k, v in m.state_dict().items():
                if not k.endswith("tril"):
                    out[f"after1.{k}"] = v.detach().numpy().copy()
        if step == 2 and cfg.get("steps", True):
            for k, v in m.state_dict().items():
                if not k.endswith("tril"):
                    out[f"after3.{k}"] = v.detach().numpy().copy()
        if step == 2:
            with torch.no_grad():
                _, losses3 = m(idx, tgt)
            out["losses_after3"] = np.array([l.item() for l in losses3], dtype=np.float32)
    for k, v in sd0.items():
        if not k.endswith("tril"):
            out[f"param.{k}"] = v.numpy()
    for i in range(M):
        out[f"idx.{i}"] = idx[i].numpy()
        out[f"tgt.{i}"] = tgt[i].numpy()
    meta = dict(cfg)
    meta["state_dict_keys"] = list(sd0.keys())
    meta["state_dict_shapes"] = {k: list(v.shape) for k, v in sd0.items()}
    meta["grad_none"] = [k for k, p in m.named_parameters() if p.grad is None]
    meta["seed"] = seed
    out["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, "losses", out["losses"], "params", sum(v.numel() for k, v in sd0.items() if not k.endswith("tril")))


SCALE = {
    "f_c1": dict(n_embd=256, n_head=8, n_layer=6, block_size=256, V=[900, 13, 144, 5],
                 cross=[True, False, False, False], B=2, param_seed=31),
    "f_m8": dict(n_embd=128, n_head=2, n_layer=2, block_size=128, V=[900, 13, 144, 5, 900, 13, 144, 5],
                 cross=[True, True, False, False, True, True, False, False], B=2, param_seed=37),
    # long-sequence shapes: C3's sequence length and cross grouping, and C4's T = 4096
    # attention walk at head size 64 (32 chunks of 128 rows)
    "f_t1024": dict(n_embd=128, n_head=2, n_layer=1, block_size=1024, V=[900, 13, 144, 5, 900, 13, 144, 5],
                    cross=[True, True, False, False, True, True, False, False], B=1, param_seed=41),
    "f_t4096": dict(n_embd=64, n_head=1, n_layer=1, block_size=4096, V=[900, 13, 144, 5],
                    cross=[True, False, False, False], B=1, param_seed=43),
}


def gen_scale_fixture(config_utils, name, cfg, seed=4321):
    import importlib
    import torch
    sys.path.insert(0, os.path.dirname(HERE))
    from golden_io import recipe_state_dict
    config_utils._config_cache = {
        "n_embd": cfg["n_embd"], "n_head": cfg["n_head"], "n_layer": cfg["n_layer"],
        "block_size": cfg["block_size"], "dropout": 0.0, "device": "cpu",
        "batch_size": cfg["B"], "eval_iters": 1,
    }
    import model as ref_model
    importlib.reload(ref_model)
    torch.manual_seed(seed)
    torch.set_num_threads(8)
    M = len(cfg["V"])
    m = ref_model.MultimodalTransformer(M, list(cfg["V"]), _params_list(cfg))
    sd0 = m.state_dict()
    keys = list(sd0.keys())
    ks = [(k, list(v.shape)) for k, v in sd0.items() if not k.endswith("tril")]
    rec = recipe_state_dict(ks, cfg["param_seed"])
    full = dict(rec)
    for k in keys:
        if k.endswith("tril"):
            full[k] = sd0[k]
    m.load_state_dict(full, strict=True)
    B, T = cfg["B"], cfg["block_size"]
    g = torch.Generator().manual_seed(seed + 1)
    idx = [torch.randint(0, v, (B, T), generator=g) for v in cfg["V"]]
    tgt = [torch.randint(0, v, (B, T), generator=g) for v in cfg["V"]]
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    logits, losses = m(idx, tgt)
    opt.zero_grad(set_to_none=True)
    sum(losses).backward()
    out = {"losses": np.array([l.item() for l in losses], dtype=np.float32)}
    for i in range(M):
        out[f"logits_tail.{i}"] = logits[i][:, -8:, :].detach().numpy()
        out[f"idx.{i}"] = idx[i].numpy()
        out[f"tgt.{i}"] = tgt[i].numpy()
    names = [k for k, p in m.named_parameters() if p.grad is not None]
    grads = {k: p.grad.detach().flatten() for k, p in m.named_parameters() if p.grad is not None}
    out["grad_norm"] = np.array([grads[k].norm().item() for k in names], dtype=np.float64)
    first = np.array([grads[k][0].item() for k in names], dtype=np.float32)
    last = np.array([grads[k][-1].item() for k in names], dtype=np.float32)
    out["grad_first"], out["grad_last"] = first, last
    flat = torch.cat([grads[k] for k in names])
    gs = torch.Generator().manual_seed(seed + 2)
    pick = torch.randint(0, flat.numel(), (2048,), generator=gs)
    out["sample_index"] = pick.numpy().astype(np.int64)
    out["sample_value"] = flat[pick].numpy()
    opt.step()
    with torch.no_grad():
        _, l1 = m(idx, tgt)
    out["losses_after1"] = np.array([l.item() for l in l1], dtype=np.float32)
    meta = dict(cfg)
    meta["state_dict_keys"] = keys
    meta["state_dict_shapes"] = {k: list(v.shape) for k, v in sd0.items()}
    meta["grad_names"] = names
    meta["grad_none"] = [k for k, p in m.named_parameters() if p.grad is None]
    meta["seed"] = seed
    out["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, "losses", out["losses"], "after1", out["losses_after1"], "grad tensors", len(names))


def gen_loop_fixture(config_utils, seed=11):
    """get_batch + estimate_loss as main.py drives them (reference training_utils.py:333-520,
    data_utils.py:293-358), on f_small's model and a 3-file dataset with numeric vocabularies."""
    import contextlib
    import importlib
    import io
    import torch
    z = np.load(os.path.join(HERE, "f_small.npz"))
    meta = json.loads(bytes(z["meta_json"]).decode())
    B, T = 3, meta["block_size"]
    config_utils._config_cache = {
        "n_embd": meta["n_embd"], "n_head": meta["n_head"], "n_layer": meta["n_layer"],
        "block_size": T, "dropout": 0.0, "device": "cpu", "batch_size": B, "eval_iters": 2,
        "output_file_name": "", "project_file_path": "",
    }
    import model as ref_model
    import training_utils as tu
    importlib.reload(ref_model)
    importlib.reload(tu)
    torch.set_num_threads(1)
    V = meta["V"]
    M = len(V)
    vocabs = [[round(0.5 * i - 3.0, 1) for i in range(v)] for v in V]  # numeric, sorted (main.py:276-281)
    file_lengths = [300, 140, 260]
    n = sum(file_lengths)
    rs = np.random.RandomState(seed)
    streams = [rs.randint(0, v, size=n) for v in V]
    n_train = int(n * 0.8)
    params = []
    for i in range(M):
        p = [None] * 12
        p[2] = True        # has_header: drives the +-1 walk (reference quirk, training_utils.py:353)
        p[3] = (i == 1)    # one percent modality (metric sign rule; is_percents skips file starts)
        p[8] = meta["cross"][i]
        p[9] = f"mod{i}"
        params.append(p)
    params[2][2] = None    # one modality without jitter
    tu.all_train_sets = [list(map(int, s[:n_train])) for s in streams]
    tu.all_val_sets = [torch.tensor(s[n_train:], dtype=torch.long) for s in streams]
    tu.all_vocabularies = vocabs
    tu.all_modality_params = params
    tu.all_file_info = None
    tu.file_lengths = file_lengths
    tu.num_modalities = M
    tu.is_percents = True
    m = ref_model.MultimodalTransformer(M, V, params)
    sd = {k[len("param."):]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("param.")}
    full = dict(sd)
    for k in meta["state_dict_keys"]:
        if k.endswith("tril"):
            full[k] = torch.tril(torch.ones(T, T))
    m.load_state_dict(full, strict=True)
    tu.m = m
    random.seed(seed)
    torch.manual_seed(seed)
    out = {}
    for i in range(M):
        out[f"train0.{i}"] = np.array(tu.all_train_sets[i])
        out[f"val.{i}"] = tu.all_val_sets[i].numpy()
    calls = []
    for c in range(2):
        xb, yb = tu.get_batch("train", 1)
        calls.append(("train", xb, yb))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        est = tu.estimate_loss(0, 10)
    xb, yb = tu.get_batch("train", 1)
    calls.append(("train", xb, yb))
    for c, (_, xb, yb) in enumerate(calls):
        for i in range(M):
            out[f"x{c}.{i}"] = xb[i].numpy()
            out[f"y{c}.{i}"] = yb[i].numpy()
    for i in range(M):
        out[f"train_end.{i}"] = np.array(tu.all_train_sets[i])
    out["est"] = np.array([est["train"], est["val"]], dtype=np.float64)
    printed = [ln for ln in buf.getvalue().splitlines() if not ln.startswith("Evaluation:")]
    m_ = {"V": V, "B": B, "T": T, "file_lengths": file_lengths, "n_train": n_train, "seed": seed,
          "vocabs": vocabs, "params": params, "printed": printed, "eval_iters": 2}
    out["meta_json"] = np.frombuffer(json.dumps(m_).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "f_loop.npz"), **out)
    print("loop est", est, "\n" + "\n".join(printed))


def gen_run_fixture(seed=2025):
    """End-to-end C0 replay fixture: the reference's own main.py on its
    demo config (examples/demo_config.yaml + demo_input_schemas.yaml; dropout 0.0 and save_model 1
    so the run is deterministic and leaves a final checkpoint), seeded (Python random, numpy, torch)
    and run as a script from the scratch copy. Recorded: every get_batch call (split, is_training,
    xb, yb), the Python-random and torch CPU RNG states at the first call (after model creation),
    the model's state_dict at that moment (the initial parameters), the loss of every training
    step, the stdout lines, the log-file text, and the final saved state_dict."""
    import contextlib
    import io
    import runpy
    import torch
    import yaml
    cfg = yaml.safe_load(open(os.path.join(SCRATCH, "examples", "demo_config.yaml")))
    cfg["model_architecture"]["dropout"] = 0.0
    cfg["project_settings"]["save_model"] = 1
    with open(os.path.join(SCRATCH, "config.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    shutil.copy(os.path.join(SCRATCH, "examples", "demo_input_schemas.yaml"), os.path.join(SCRATCH, "input_schemas.yaml"))
    out_dir = os.path.join(SCRATCH, "examples", "output")
    if os.path.exists(out_dir):
        shutil.rmtree(out_dir)
    import training_utils as tu
    import model as ref_model
    for mod in ("config_utils", "training_utils", "model"):
        sys.modules.pop(mod, None)  # fresh imports under the script's own config discovery
    import config_utils as cu2
    cu2._config_cache = None
    import training_utils as tu
    import model as ref_model
    calls, steps, first = [], [], {}
    orig_get = tu.get_batch

    def rec_get_batch(split, is_training):
        if not first:
            first["py"] = random.getstate()
            first["torch"] = torch.get_rng_state().clone()
            first["sd"] = {k: v.detach().clone() for k, v in tu.m.state_dict().items() if not k.endswith("tril")}
            first["train"] = [list(map(int, t)) for t in tu.all_train_sets]
        xb, yb = orig_get(split, is_training)
        calls.append((split, int(is_training), [x.clone() for x in xb], [y.clone() for y in yb]))
        return xb, yb
    tu.get_batch = rec_get_batch
    orig_fwd = ref_model.MultimodalTransformer.forward

    def rec_forward(self, idx_list, targets_list=None):
        lg, ls = orig_fwd(self, idx_list, targets_list)
        if self.training and ls is not None:
            steps.append([float(l.item()) for l in ls])
        return lg, ls
    ref_model.MultimodalTransformer.forward = rec_forward
    cwd = os.getcwd()
    os.chdir(SCRATCH)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.set_num_threads(1)
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            runpy.run_path(os.path.join(SCRATCH, "main.py"), run_name="__main__")
    finally:
        os.chdir(cwd)
        ref_model.MultimodalTransformer.forward = orig_fwd
        tu.get_batch = orig_get
    stdout = buf.getvalue()
    log_text = open(os.path.join(out_dir, cfg["project_settings"]["output_file_name"])).read()
    final_sd = torch.load(os.path.join(SCRATCH, cfg["project_settings"]["model_file_name"]), weights_only=True)
    out = {}
    for c, (split, tr, xb, yb) in enumerate(calls):
        for i in range(len(xb)):
            out[f"x{c}.{i}"] = xb[i].numpy()
            out[f"y{c}.{i}"] = yb[i].numpy()
    out["steps"] = np.array(steps, dtype=np.float64)
    out["torch_state"] = first["torch"].numpy()
    py = first["py"]
    out["py_state"] = np.array(py[1], dtype=np.uint64)
    for k, v in first["sd"].items():
        out[f"init.{k}"] = v.numpy()
    for k, v in final_sd.items():
        if not k.endswith("tril"):
            out[f"final.{k}"] = v.numpy()
    for i, t in enumerate(first["train"]):
        out[f"train0.{i}"] = np.array(t, dtype=np.int64)
    for i, v in enumerate(tu.all_val_sets):
        out[f"val.{i}"] = v.numpy()
    meta = {"seed": seed, "config": cfg, "calls": [(sp, tr) for sp, tr, _, _ in calls],
            "py_state_version": py[0], "py_state_gauss": py[2],
            "vocabs": [list(v) for v in tu.all_vocabularies], "params": tu.all_modality_params,
            "file_lengths": list(tu.file_lengths) if tu.file_lengths is not None else None,
            "is_percents": bool(tu.is_percents), "V": [len(v) for v in tu.all_vocabularies],
            "state_dict_keys": list(final_sd.keys()), "stdout": stdout.splitlines(), "log": log_text}
    out["meta_json"] = np.frombuffer(json.dumps(meta, default=str).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "f_c0run.npz"), **out)
    print("c0 run:", len(calls), "get_batch calls,", len(steps), "training steps; first losses", steps[:2],
          "last", steps[-1])


def gen_metric_fixture(seed=77):
    """calculate_evaluation_metrics (reference training_utils.py:215-330)."""
    import torch
    import training_utils as tu
    torch.manual_seed(seed)
    B, T = 16, 6
    cases = []
    # value modality (non-percent), numeric vocab incl. duplicates of direction; percent modality; non-numeric
    vocab0 = [round(1.0 + 0.5 * i, 1) for i in range(9)]           # value data
    vocab1 = [-2.0, -1.0, -0.5, 0.0, 0.5, 1.0, 2.0]                 # percent data
    vocab2 = ["a", "b", "c"]                                         # non-numeric -> skipped
    vocabs = [vocab0, vocab1, vocab2]
    params = []
    for i, pct in enumerate([False, True, False]):
        p = [None] * 12
        p[3] = pct
        p[9] = f"m{i}"
        params.append(p)
    logits = [torch.randn(B, T, len(v)) for v in vocabs]
    # force argmax ties on a few rows of modality 0 (first max must win)
    logits[0][0, -1, :] = 0.0
    logits[0][1, -1, 2] = 5.0
    logits[0][1, -1, 6] = 5.0
    xb = [torch.randint(0, len(v), (B, T)) for v in vocabs]
    yb = [torch.randint(0, len(v), (B, T)) for v in vocabs]
    # flat direction cases: prev == actual
    yb[0][2, -1] = xb[0][2, -1]
    wins, losses, cert, proc = tu.calculate_evaluation_metrics(logits, xb, yb, 3, vocabs, params, None)
    out = {}
    for i in range(3):
        out[f"logits.{i}"] = logits[i].numpy()
        out[f"xb.{i}"] = xb[i].numpy()
        out[f"yb.{i}"] = yb[i].numpy()
    out["wins"] = np.array(wins)
    out["losses"] = np.array(losses)
    out["certainty"] = np.array(cert, dtype=np.float64)
    out["processed"] = np.array(proc)
    out["vocab.0"] = np.array(vocab0)
    out["vocab.1"] = np.array(vocab1)
    meta = {"percent": [False, True, False], "numeric": [True, True, False], "vocab2": vocab2}
    out["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "eval_metrics.npz"), **out)
    print("metrics", wins, losses, cert, proc)


def gen_index_fixture(seed=99):
    """generate_batch_starting_indices (reference training_utils.py:33-181) under a seeded torch RNG."""
    import torch
    import training_utils as tu
    cases = [
        dict(data_size=900, block_size=16, batch_size=32, split="train", file_lengths=[1000], is_percents=False),
        dict(data_size=9000, block_size=32, batch_size=64, split="train",
             file_lengths=[1000] * 10, is_percents=True),
        dict(data_size=1000, block_size=32, batch_size=64, split="val",
             file_lengths=[1000] * 10, is_percents=True),
        dict(data_size=2500, block_size=8, batch_size=50, split="val",
             file_lengths=[700, 300, 1200, 900, 400], is_percents=False),
        dict(data_size=2100, block_size=8, batch_size=50, split="train",
             file_lengths=[700, 300, 1200, 900, 400], is_percents=True),
    ]
    out = {}
    for ci, c in enumerate(cases):
        torch.manual_seed(seed + ci)
        ix = tu.generate_batch_starting_indices(c["data_size"], c["block_size"], c["batch_size"], c["split"],
                                                c["file_lengths"], c["is_percents"])
        out[f"ix.{ci}"] = ix.numpy()
    meta = {"cases": cases, "seed": seed}
    out["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "batch_indices.npz"), **out)
    print("indices", [out[f"ix.{i}"][:4] for i in range(len(cases))])


def gen_jitter_fixture(seed=5):
    """add_rand_to_data_points (reference data_utils.py:293-358) with rand_size=True (the has_header quirk)."""
    import data_utils as du
    random.seed(seed)
    data = [int(x) for x in np.random.RandomState(seed).randint(0, 12, size=400)]
    before = list(data)
    after = du.add_rand_to_data_points(data, True, 12)
    out = {"before": np.array(before), "after": np.array(after)}
    np.savez_compressed(os.path.join(HERE, "jitter.npz"), **out)
    d = np.array(after) - np.array(before)
    print("jitter changed", int((d != 0).sum()), "of", len(d))


if __name__ == "__main__":
    want = set(sys.argv[1:])
    cu = _import_reference()

    def on(name):
        return not want or name in want

    for name, cfg in CONFIGS.items():
        if on(name):
            gen_model_fixture(cu, name, cfg)
    for name, cfg in SCALE.items():
        if on(name):
            gen_scale_fixture(cu, name, cfg)
    if on("f_loop"):
        gen_loop_fixture(cu)
    if on("f_c0run"):
        gen_run_fixture()
    if on("eval_metrics"):
        gen_metric_fixture()
    if on("batch_indices"):
        gen_index_fixture()
    if on("jitter"):
        gen_jitter_fixture()
