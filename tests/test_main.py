"""The main.py entry (reference main.py:455-667 surface): config.yaml parsing with the
reference's defaults, the printed parameter estimate, and (GPU) a short end-to-end training run
with evaluation, log lines, checkpoint save and reload through create_new_model: 0."""
import os
import sys
import textwrap

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import main  # noqa: E402
import config_utils  # noqa: E402


def test_param_estimate_matches_reference_print():
    # the reference demo (V=[57,3], C=32, H=4, L=2, T=4, cross=[T,F]) prints "Parameters: 0.1M"
    n = main.approx_param_count([57, 3], 32, 4, 2, 4, [True, False])
    assert f"{n / 1e6:.1f}M" == "0.1M"


def test_config_yaml_surface(tmp_path):
    p = tmp_path / "config.yaml"
    p.write_text(textwrap.dedent("""
        project_settings:
          project_file_path: "./examples/"
          output_file_name: "demo_training_log.txt"
          model_file_name: "output/demo_model.pth"
          create_new_model: 1
          save_model: 0
          device: cpu
        data_splitting:
          validation_size: 0.2
          num_validation_files: 0
        training_parameters:
          batch_size: 4
          block_size: 4
          max_iters: 50
          eval_interval: 25
          learning_rate: 0.001
        model_architecture:
          n_embd: 32
          n_head: 4
          n_layer: 2
          dropout: 0.1
    """))
    cfg = config_utils.load_system_config(str(p))
    assert cfg["batch_size"] == 4 and cfg["block_size"] == 4 and cfg["n_embd"] == 32 and cfg["n_head"] == 4
    assert cfg["eval_iters"] == 40  # reference default (config_manager.py:110-147)
    assert cfg["save_model"] == 0 and cfg["create_new_model"] == 1 and cfg["validation_size"] == 0.2
    assert cfg["model_file_name"] == "output/demo_model.pth" and cfg["dropout"] == 0.1


def test_cpu_device_is_refused(tmp_path):
    p = tmp_path / "config.yaml"
    p.write_text("project_settings:\n  device: cpu\n")
    with pytest.raises(SystemExit):
        main.main(["--config", str(p), "--synthetic", "--rows", "20000"])


@pytest.mark.gpu
def test_main_trains_evaluates_saves_and_reloads(tmp_path):
    import mmt_data
    cfg = config_utils.load_system_config("/nonexistent.yaml")
    cfg.update({"device": "cuda", "batch_size": 8, "block_size": 32, "max_iters": 41, "eval_interval": 20,
                "eval_iters": 2, "learning_rate": 3e-3, "n_embd": 64, "n_head": 2, "n_layer": 1, "dropout": 0.0,
                "project_file_path": str(tmp_path) + "/", "output_file_name": "log.txt",
                "model_file_name": str(tmp_path / "ckpt" / "m.pth"), "save_model": 1, "create_new_model": 1})
    data = mmt_data.make_synthetic(n_rows=40_000, n_files=10)
    lines = []
    m, hist = main.run(dict(cfg), data, log=lines.append)
    assert "TRAINING COMPLETED SUCCESSFULLY" in "\n".join(lines)
    assert [h[0] for h in hist] == [0, 20, 40]
    assert hist[-1][1] < hist[0][1]  # training loss went down
    assert os.path.exists(cfg["model_file_name"])
    log = open(tmp_path / "output" / "log.txt").read()
    assert "STEP 20/41 (48.8% Complete) | Training Loss:" in log
    assert "DIRECTIONAL PREDICTION Val Set - Close (ranged): Correct=" in log
    # reload: create_new_model 0 picks the checkpoint up (reference main.py:466-483)
    cfg2 = dict(cfg, create_new_model=0, max_iters=0, save_model=0)
    lines2 = []
    m2, _ = main.run(cfg2, data, log=lines2.append)
    assert "Model: Loaded successfully" in lines2
    sd1, sd2 = m.state_dict(), m2.state_dict()
    k = "blocks.0.ffwd_layers.0.net.0.weight"
    assert np.allclose(sd1[k].cpu().numpy(), sd2[k].cpu().numpy())
