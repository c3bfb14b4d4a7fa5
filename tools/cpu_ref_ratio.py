"""Restatement / reference CPU speed ratios, measured in the BUILD container where
the reference is importable (tools/refshim.py).  Writes profiles/<tag>/cpu_ref_ratio.json, which
bench.py reads to put the reference-equivalent CPU rate beside the restatement's own.

Legs, each timed on this host, 1 process, torch on 1 thread, `--seconds` per leg:
  random_step  random-legal game.step loop with auto-reset: reference Game2048 (valid directions
               from direction_has_step, game.py:260-330) vs oracle/pyref.time_random_steps
  train_loop   the README train loop (train.py:1669-1760, --episodes 1 --batch-size=4 -h 196
               --upsample-ratio 0.25): the reference's play_game_for_episode + calculate_advantage
               + model_optimize_step with its Muon/AdamW MultiOptimizer vs oracle/pyloop.time_train_loop

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/cpu_ref_ratio.py --tag r02
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import random
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "tools")]


def ref_random_steps(game, seconds: float, seed: int = 0x2048) -> dict:
    random.seed(seed)
    g = game.Game2048()
    g.reset()
    dirs = list(game.Direction)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(200):
            valid = [d for d in dirs if g.direction_has_step(d)]
            _, _, done, _ = g.step(random.choice(valid))
            n += 1
            if done:
                g.reset()
    dt = time.perf_counter() - t0
    return {"value": n / dt, "steps": n, "seconds": dt}


def ref_train_loop(game, train, seconds: float, hidden=196, batch_size=4, seed=0x2048, max_iters=50) -> dict:
    from torch.optim import AdamW, Muon
    from transformers import get_scheduler
    torch.manual_seed(seed)
    random.seed(seed)
    model = game.GameMLP(game.MLPConfig(hidden_dim=hidden, num_layers=2))
    with torch.no_grad():  # train.py:1559-1567
        for p in (model.action_head.weight, model.action_head.bias, model.value_head.weight, model.value_head.bias):
            p.zero_()
    o2, o1, v2, v1 = model.get_param_groups(1e-4, 1e-3)  # train.py:1587-1612
    adamw = AdamW([o1, v1], betas=(0.9, 0.999), weight_decay=0.01)
    muon = Muon([o2, v2], adjust_lr_fn="match_rms_adamw", weight_decay=0.01)
    opt = train.MultiOptimizer((muon, get_scheduler("cosine", muon, num_warmup_steps=10, num_training_steps=20000)),
                               (adamw, get_scheduler("cosine", adamw, num_warmup_steps=10, num_training_steps=20000)))
    fm, m2, mu = 0.0, 1.0, 0.0
    n = it = 0
    t0 = time.perf_counter()
    while it < max_iters and (it == 0 or time.perf_counter() - t0 < seconds):
        model.eval()
        eps = [train.play_game_for_episode(model, max_steps=None, device=None)]
        eps, aug, fm, m2, mu = train.calculate_advantage(eps, 0.99, fm, 0.10, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0,
                                                         0.0, rtg_beta=0.99, rtg_m2=m2, rtg_mu=mu, rtg_step=it + 1,
                                                         upsample_ratio=0.25)
        n += len(eps[0]["moves"])
        if aug:
            eps.append({"moves": aug, "total_points": 0, "total_steps": len(aug), "augmented": True})
        train.model_optimize_step(model=model, episodes=eps, optimizer=opt, lr_scheduler=None, kl_strength=0.02,
                                  critic_strength=0.2, device=None, batch_size=batch_size, epochs=1)
        it += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "steps": n, "iters": it, "seconds": dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r02")
    ap.add_argument("--seconds", type=float, default=15.0)
    a = ap.parse_args()
    torch.set_num_threads(1)
    from refshim import load_reference
    game, train = load_reference()
    # the restatements (imported after the reference: `train` below must be the build's module)
    sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]
    for name in ("train", "game", "logger"):
        sys.modules.pop(name, None)
    from oracle import pyloop, pyref
    res = {"host": platform.processor() or platform.machine(), "cpus_visible": os.cpu_count(), "torch_threads": 1,
           "seconds_per_leg": a.seconds}
    r_ref = ref_random_steps(game, a.seconds)
    r_port = pyref.time_random_steps(a.seconds)
    res["random_step"] = {"reference": r_ref, "port": {k: r_port[k] for k in ("value", "steps", "seconds")},
                          "port_over_reference": r_port["value"] / r_ref["value"]}
    t_ref = ref_train_loop(game, train, a.seconds)
    t_port = pyloop.time_train_loop(a.seconds)
    res["train_loop"] = {"reference": t_ref, "port": {k: t_port[k] for k in ("value", "steps", "iters", "seconds")},
                         "port_over_reference": t_port["value"] / t_ref["value"]}
    out = ROOT / "profiles" / a.tag / "cpu_ref_ratio.json"
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
