"""Configuration accessors — same names and cache hook as the reference's config_utils.py:8-69.

`_config_cache` is the injection point (tests and the bench set it directly, as the reference's
own model import does). When empty it is filled from `config.yaml` in the current directory
with the defaults of the reference's SystemConfig.from_dict (config_manager.py:110-147) and the
`device: auto` resolution of compatibility_layer.py:124-126.
"""
import os

_config_cache = None

_DEFAULTS = {
    "project_settings": {"project_file_path": "", "output_file_name": "training_log.txt",
                         "model_file_name": "model.pth", "create_new_model": 1, "save_model": 1, "device": "cpu"},
    "data_splitting": {"validation_size": 0.1, "num_validation_files": 0},
    "training_parameters": {"batch_size": 32, "block_size": 64, "max_iters": 5000, "eval_interval": 500,
                            "eval_iters": 40, "learning_rate": 3e-4},
    "model_architecture": {"n_embd": 384, "n_head": 6, "n_layer": 6, "dropout": 0.2,
                           "fixed_values": [-0.5, -0.2, -0.1, 0, 0.1, 0.2, 0.5],
                           # build-only key (the reference ignores unknown keys): "bf16" | "fp8"
                           "precision": "bf16"},
}


def load_system_config(path="config.yaml"):
    """Flattened system configuration dict from a reference-format config.yaml."""
    import yaml
    raw = {}
    if os.path.exists(path):
        with open(path, "r", encoding="utf-8") as f:
            raw = yaml.safe_load(f) or {}
    flat = {}
    for section, defaults in _DEFAULTS.items():
        sec = raw.get(section, {}) or {}
        for k, v in defaults.items():
            flat[k] = sec.get(k, v)
    flat["create_new_model"] = int(bool(flat["create_new_model"]))
    flat["save_model"] = int(bool(flat["save_model"]))
    if flat["device"] == "auto":
        import torch
        flat["device"] = "cuda" if torch.cuda.is_available() else "cpu"
    return flat


def _get_config():
    global _config_cache
    if _config_cache is None:
        _config_cache = load_system_config()
    return _config_cache


def _get_device():
    return _get_config()["device"]


def _get_block_size():
    return _get_config()["block_size"]


def _get_batch_size():
    return _get_config()["batch_size"]


def _get_eval_iters():
    return _get_config()["eval_iters"]


def _get_n_embd():
    return _get_config()["n_embd"]


def _get_n_head():
    return _get_config()["n_head"]


def _get_n_layer():
    return _get_config()["n_layer"]


def _get_dropout():
    return _get_config()["dropout"]


def _get_fixed_values():
    return _get_config()["fixed_values"]


def _get_precision():
    """Build-only knob (no reference counterpart): "bf16" (default) or "fp8" (MX-fp8 forward
    GEMMs, BASELINE configs[4]); the MMT_PRECISION environment variable overrides the config."""
    p = os.environ.get("MMT_PRECISION") or _get_config().get("precision", "bf16")
    if p not in ("bf16", "fp8"):
        raise ValueError(f"precision must be 'bf16' or 'fp8', got {p!r}")
    return p
