"""bench.py's host-side logic (no GPU): the N-rank launch plan, the roofline arithmetic and the
useful-flop formula of SURVEY.md §8d."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_launch_plan_one_rank_per_gpu():
    cmd = bench.launch_plan(8, ["--gpus", "8", "--steps", "5"], 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29512" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5:] == [os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "5"]


def test_roofline_entry_picks_binding_roof():
    # 100 launches in 25 sampled steps, 10 ms total: 0.1 ms per launch
    hbm = bench.roofline_entry("ffn0", 10.0, 100, 100 * 1e9, 100 * 1e8, 25, "c1")  # 10 flop/B
    assert hbm["bound"] == "hbm" and hbm["achieved"] == pytest.approx(1000.0) and hbm["frac"] == pytest.approx(0.125)
    assert hbm["launches_per_step"] == 4 and hbm["ms_per_step"] == pytest.approx(0.4)
    mf = bench.roofline_entry("attn_fwd", 10.0, 100, 100 * 1e11, 100 * 1e8, 25, "c1")  # 1000 flop/B
    assert mf["bound"] == "mfma" and mf["achieved"] == pytest.approx(1000.0) and mf["frac"] == pytest.approx(0.4)


def test_train_flops_formula_matches_survey():
    # C1 (V=[900,13,144,5], cross on modality 0) causal-useful 1.3956e8 / dense 1.5607e8 per row
    V = [900, 13, 144, 5]
    cross = [True, False, False, False]
    assert bench.train_flops_per_row(4, 256, 8, 6, 256, V, cross, a=0.5) == pytest.approx(1.3956e8, rel=1e-4)
    assert bench.train_flops_per_row(4, 256, 8, 6, 256, V, cross, a=1.0) == pytest.approx(1.5607e8, rel=1e-4)
