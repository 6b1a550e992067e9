"""main.py — the training entry point, drop-in for the reference's main.py hot loop
(tsnuk/trade-AId-multimodal-transformer main.py:455-667) on the MI355X path.

    python main.py [--config config.yaml] [--synthetic [--rows N]] [--data tokens.npz]

Same configuration surface as the reference: the `config.yaml` sections project_settings,
data_splitting, training_parameters and model_architecture (read by config_utils with the
reference's defaults, config_manager.py:110-147), the same model creation / checkpoint-load
fallbacks (main.py:461-483), the same evaluation cadence and early-stopping bookkeeping
(main.py:598-625), checkpointing (main.py:627-638, 657-667), print lines and log-file lines.

Data: the reference builds its token streams with its own CSV ingest (file_cache.py,
data_utils.py, main.py:76-376), which runs once at startup and is outside this build's hot path
(SURVEY.md §2). Two sources are accepted here:
  * --synthetic: the 4-modality synthetic market dataset of SURVEY.md §8d (mmt_data);
  * --data tokens.npz: pre-tokenised streams (train_i / val_i int arrays, vocab_i, params_json,
    file_lengths, is_percents), e.g. dumped from a reference ingest run.
Inside a reference checkout the reference's own main.py can instead import this build's model,
training_utils and AdamW directly and keep its ingest unchanged.
"""
import argparse
import json
import os
import sys
from datetime import datetime

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "trade-aid-multimodal-transformer_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import config_utils  # noqa: E402
import mmt_data  # noqa: E402
import mmt_optim  # noqa: E402
import training_utils  # noqa: E402
from model import MultimodalTransformer  # noqa: E402
from training_utils import estimate_loss, get_batch  # noqa: E402


def load_tokens(path):
    """Pre-tokenised dataset (.npz, no pickles): the globals main.py:387-396 would inject."""
    z = np.load(path, allow_pickle=False)
    meta = json.loads(bytes(z["meta_json"]).decode())
    M = meta["num_modalities"]
    train = [z[f"train_{i}"].astype(np.int64) for i in range(M)]
    val = [torch.from_numpy(z[f"val_{i}"].astype(np.int64)) for i in range(M)]
    vocabs = [list(map(float, z[f"vocab_{i}"])) for i in range(M)]
    full = [np.concatenate([t, v.numpy()]) for t, v in zip(train, val)]
    return {"train": train, "val": val, "full": full, "vocabs": vocabs, "params": meta["params"],
            "file_lengths": meta["file_lengths"], "is_percents": bool(meta["is_percents"]),
            "vocab_sizes": [len(v) for v in vocabs]}


def approx_param_count(V, C, H, L, T, cross):
    """The parameter estimate the reference prints (main.py:400-449): weights only, no biases,
    LayerNorm weights only; kept so the "Parameters: x.xM" line matches."""
    M, hs = len(V), C // H
    tok = sum(v * C for v in V) + T * C
    attn = H * 3 * (C * (hs // 2) + (hs // 2) * hs) + (hs * H) * (C // 2) + (C // 2) * C
    per_layer = M * (attn + 8 * C * C + 2 * C)
    xattn = sum((M - 1) * (2 * (C * (H * hs // 2) + hs // 2 * hs)) + C * (C // 2) + (C // 2) * C + C
                for c in cross if c)
    out = sum(C + C * (v // 2) + (v // 2) * v for v in V)
    return tok + L * (per_layer + xattn) + out


def run(cfg, data, log=print):
    """The reference training loop (main.py:461-667) over an installed dataset."""
    config_utils._config_cache = cfg
    device = cfg["device"]
    M = len(data["vocab_sizes"])
    V = data["vocab_sizes"]
    params = data["params"]
    model_file_name = cfg["model_file_name"]
    log("Model Configuration:")
    log(f"  Modalities: {M}")
    log(f"  Vocabulary sizes: {V}")
    nparam = approx_param_count(V, cfg["n_embd"], cfg["n_head"], cfg["n_layer"], cfg["block_size"], [p[8] for p in params])
    log(f"  Parameters: {nparam / 1e6:.1f}M")
    log("")

    def fresh():
        mm = MultimodalTransformer(M, V, params).to(device)
        return mm, mmt_optim.AdamW(mm.parameters(), lr=cfg["learning_rate"])

    if cfg["create_new_model"] == 1:
        log("Model: Creating new transformer...")
        m, optimizer = fresh()
        log("Model: Created successfully")
    else:
        log(f"Model: Loading from {model_file_name}...")
        m, optimizer = fresh()
        try:
            m.load_state_dict(torch.load(model_file_name, weights_only=True, map_location="cpu"))
            log("Model: Loaded successfully")
            optimizer = mmt_optim.AdamW(m.parameters(), lr=cfg["learning_rate"])
            log("Optimizer: Created with loaded parameters")
        except FileNotFoundError:
            log("Model: File not found, creating new model instead")
            m, optimizer = fresh()
            log("Model: Created successfully")
        except Exception as e:  # noqa: BLE001 - the reference falls back on any load error
            log(f"Model: Loading failed ({e}), creating new model")
            m, optimizer = fresh()
            log("Model: Created successfully")

    mmt_data.install(training_utils, data, m)
    training_utils._device_batcher[0] = None

    out_name = cfg["output_file_name"]
    out_path = cfg["project_file_path"] + "output/" + out_name
    if out_name != "":
        os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
        with open(out_path, "a", encoding="utf-8") as f:
            f.write("\n--- TRAINING & EVALUATION RESULTS ---\n\n")
            f.write(f"Directional Prediction Analysis ({cfg['eval_iters']} iterations x {cfg['batch_size']} batches = "
                    f"{cfg['eval_iters'] * cfg['batch_size']:,} samples per evaluation)\n")

    max_iters, eval_interval = cfg["max_iters"], cfg["eval_interval"]
    log("")
    log("TRAINING PROGRESS")
    log(f"  - Iterations: {max_iters}")
    log(f"  - Device: {device}")
    log("  - Note: ** Intensive computation ahead **")
    log("")
    best_val, patience, no_improve = float("inf"), 1000, 0
    history = []
    for it in range(max_iters):
        if it % 100 == 0:
            log(f"Training: Iteration {it}/{max_iters}")
        if it % eval_interval == 0 or it == max_iters - 1:
            losses = estimate_loss(it, max_iters)
            now = datetime.now().strftime("%H:%M:%S")
            bad = m.nonfinite_loss_mask(sticky=True, clear=True)  # device flag of the loss kernel
            bad = int(bad.item()) if bad is not None else 0     # one sync
            if bad:
                names = [str(p[9] or f"Modality {i + 1}") for i, p in enumerate(m.all_modality_params)
                         if bad >> i & 1]
                log(f"Warning: non-finite loss since the last evaluation in: {', '.join(names)} | {now}")
            history.append((it, losses["train"], losses["val"]))
            if not (np.isnan(losses["train"]) or np.isnan(losses["val"])):
                log(f"\nLOSS METRICS: Step {it}/{max_iters} | Train: {losses['train']:.4f} | Val: {losses['val']:.4f} "
                    f"| Time: {now}")
                log("-" * 80)
                if out_name != "":
                    with open(out_path, "a", encoding="utf-8") as f:
                        f.write(f"\nSTEP {it:,}/{max_iters:,} ({it / max_iters * 100:.1f}% Complete) | Training Loss: "
                                f"{losses['train']:.6f} | Validation Loss: {losses['val']:.6f} | {now}\n\n")
            else:
                log(f"Warning: Step {it} losses are NaN, skipping save | {now}")
            if not np.isnan(losses["val"]):
                if losses["val"] < best_val:
                    best_val, no_improve = losses["val"], 0
                else:
                    no_improve += 1
                if no_improve >= patience:
                    log(f"Training: Early stopping (no improvement for {patience} evaluations)")
                    break
        if cfg["save_model"] == 1 and (it % eval_interval == 0 or it == max_iters - 1):
            os.makedirs(os.path.dirname(model_file_name) or ".", exist_ok=True)
            torch.save(m.state_dict(), model_file_name)
            log("")
            log(f"Saved: Model checkpoint ({round(os.path.getsize(model_file_name) / 1024 ** 2, 2)} MB) | "
                f"{datetime.now().strftime('%H:%M:%S')}")
            log("")
        xb_list, yb_list = get_batch("train", 1)
        logits_list, losses_list = m(xb_list, yb_list)
        if losses_list and all(l is not None for l in losses_list):
            total_loss = sum(losses_list)
            optimizer.zero_grad(set_to_none=True)
            total_loss.backward()
            optimizer.step()
        else:
            log("Warning: Training step losses not calculated, skipping backpropagation")
    # the device-exact batcher's last walk (the final step's get_batch) is still on the GPU: bring
    # Python's `random` state and the training lists up to it, as the reference's loop leaves them
    # (a no-op in the other batcher modes)
    training_utils.sync_host_state()
    log("\nTRAINING COMPLETED SUCCESSFULLY")
    if cfg["save_model"] == 1:
        os.makedirs(os.path.dirname(model_file_name) or ".", exist_ok=True)
        log(f"Final Save: Model checkpoint | {datetime.now().strftime('%H:%M:%S')}")
        torch.save(m.state_dict(), model_file_name)
        log(f"Final Save: {round(os.path.getsize(model_file_name) / 1024 ** 2, 2)} MB complete")
    return m, history


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", default="config.yaml")
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--data", default=None)
    ap.add_argument("--seed", type=int, default=None, help="opt-in seed (the reference seeds nothing)")
    a = ap.parse_args(argv)
    cfg = config_utils.load_system_config(a.config)
    if cfg["device"] == "cpu":
        raise SystemExit("this build runs the model on the MI355X only: set device: cuda (or auto) in config.yaml")
    if a.seed is not None:
        torch.manual_seed(a.seed)
        np.random.seed(a.seed)
    if a.data:
        data = load_tokens(a.data)
    elif a.synthetic:
        data = mmt_data.make_synthetic(n_rows=a.rows, n_files=max(1, min(100, a.rows // 10_000)),
                                       validation_size=cfg["validation_size"])
    else:
        raise SystemExit("no dataset: pass --synthetic or --data tokens.npz (see the module docstring)")
    run(cfg, data)


if __name__ == "__main__":
    main()
