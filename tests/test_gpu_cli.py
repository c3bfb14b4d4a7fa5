"""The trainer CLI run as the README runs it (/root/reference/README.md:12: --batch-size=4 -h 196
--upsample-ratio 0.25 --eval-freq ... --viz-dir ...), as a fresh child process for 3 train steps at
--episodes 1 (BASELINE config 1's single env) and --episodes 64: finite metrics, the JSONL key set of
the reference's compute_batch_stats (train.py:992-1040) and eval (train.py:1869-1877), the
step_XXXXXX.json viz schema (train.py:1155-1209) and a best_model.pt that agent.GameMLP reloads."""

import json
import math
import subprocess
import sys

import pytest
import torch

from conftest import PKG

pytestmark = pytest.mark.gpu

# train.py:992-1040 (compute_batch_stats) -- every key the reference writes per train step
REF_STEP_KEYS = {
    "samples", "augmented_samples", "actor_loss", "critic_loss", "total_loss", "policy_loss", "entropy_loss",
    "value_loss", "actor_grad_norm", "critic_grad_norm", "grad_norm", "entropy", "peak_score", "avg_score",
    "ema_avg_score", "median_score", "avg_episode_return", "pct_512", "ema_pct_512", "pct_1024", "ema_pct_1024",
    "pct_2048", "ema_pct_2048", "reward_var", "reward_mean", "zero_reward_pct", "advantage_mean", "advantage_var",
    "advantage_l2", "adv_min", "adv_max", "G_norm_mean", "G_norm_std", "G_norm_min", "G_norm_max", "G_raw_std",
    "V_std", "A_std", "var_reduction", "explained_var", "ema_explained_var", "kl_total", "kl_average", "kl_max",
    "actor_lr", "critic_lr", "current_beta"}
REF_EVAL_KEYS = {"eval/max_score", "eval/avg_score", "eval/median_score", "eval/pct_512", "eval/pct_1024",
                 "eval/pct_2048"}
VIZ_REWARD_KEYS = {"points", "smoothness", "tile_bonus", "corner", "adjacency", "chain", "monotonicity",
                   "topological", "emptiness"}


@pytest.mark.parametrize("episodes", [1, 64])
def test_readme_command_runs(episodes, tmp_path):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    cmd = [sys.executable, str(PKG / "train.py"), "train", "--batch-size=4", "--steps=3", "--lr", "0.001",
           "--critic-lr", "1e-4", "-h", "196", "--gamma", "0.99", "--entropy", "0.02", "--smoothness", "0.0",
           "--tile-bonus", "0.0", "--print-freq", "1", "--corner", "0.0", "--points", "0.10", "--show-last-steps",
           "2", "--viz-dir", str(tmp_path / "viz"), "--mono", "1.0", "--model-type", "mlp", "--critic", "0.2",
           "--rtg-beta", "0.99", "--wandb", "--eval-freq", "2", "--emptiness", "0.0", "--warmup-steps", "10",
           "--upsample-ratio", "0.25", "--episodes", str(episodes), "--eval-games", "8",
           "--log-dir", str(tmp_path / "logs"), "--checkpoint-dir", str(tmp_path / "ck")]
    r = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = r.stdout
    assert "Reward breakdown:" in out and "PBRS Reward Shaping" in out and "Final state:" in out
    assert "Last 2 steps" in out
    logs = list((tmp_path / "logs").glob("train_mlp_*_001.jsonl"))
    assert len(logs) == 1
    rows = [json.loads(line) for line in logs[0].read_text().splitlines()]
    steps = [r_ for r_ in rows if "samples" in r_]
    evals = [r_ for r_ in rows if "eval/avg_score" in r_]
    assert [s["step"] for s in steps] == [0, 1, 2] and [e["step"] for e in evals] == [2]
    for s in steps:
        assert REF_STEP_KEYS <= set(s), REF_STEP_KEYS - set(s)
        for k in REF_STEP_KEYS:
            assert isinstance(s[k], (int, float)) and math.isfinite(s[k]), (k, s[k])
        assert s["samples"] > 0 and s["augmented_samples"] > 0  # --upsample-ratio 0.25
    assert REF_EVAL_KEYS <= set(evals[0])
    viz = sorted((tmp_path / "viz").glob("step_*.json"))
    assert viz and viz[0].name == "step_000000.json"
    v = json.loads(viz[0].read_text())
    assert set(v) == {"step", "score", "total_steps", "moves"} and len(v["moves"]) > 0
    # play_game_for_episode's step counter: the terminal move is not counted (train.py:334-343)
    assert v["total_steps"] in (len(v["moves"]), len(v["moves"]) - 1)
    mv = v["moves"][0]
    assert set(mv) == {"step", "state_before", "action", "state_after", "points_earned", "rewards", "entropy",
                       "advantage"}
    assert set(mv["rewards"]) == VIZ_REWARD_KEYS and mv["action"] in ("UP", "DOWN", "LEFT", "RIGHT")
    assert sum(m["points_earned"] for m in v["moves"]) == v["score"]
    # best_model.pt: the reference's checkpoint keys, reloadable into agent.GameMLP
    sys.path.insert(0, str(PKG))
    import agent
    ck = torch.load(tmp_path / "ck" / "best_model.pt", map_location="cpu", weights_only=True)
    assert {"model_state_dict", "config", "eval_avg_score", "train_step"} <= set(ck)
    m = agent.GameMLP(agent.MLPConfig(**ck["config"]))
    m.load_state_dict(ck["model_state_dict"])
    assert ck["config"]["hidden_dim"] == 196 and ck["train_step"] == 2
