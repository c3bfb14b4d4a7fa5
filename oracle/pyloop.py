"""CPU restatement of the README train loop (train.py:1669-1760 at --episodes 1 --batch-size=4 -h 196
--upsample-ratio 0.25).  TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it
on the GPU box's host, where the reference is not present.

Per train step, like the reference on one process:
  play_game_for_episode (train.py:213-346): per move, to_model_format (game.py:92-101) on the
      board, GameMLP forward of one board (torch, CPU), masked softmax + torch.multinomial, and
      oracle/pyref.step (game.step with its 17 heuristic evaluations, game.py:952-1030);
  calculate_advantage (train.py:651-904): oracle.reward_rtg_normalize (the C restatement) and the
      D4 up-sampling of the host records (g2048/augment.py, train.py:774-881);
  model_optimize_step (train.py:414-642) over the moves in minibatches of 4 with Muon + AdamW and
      cosine schedules (train.py:1587-1612), the host implementation in 2048-ppo_amd/train.py.
"""

from __future__ import annotations

import random
import time

import numpy as np
import torch

from . import oracle as O
from . import pyref

_IDX = torch.arange(16)
_ROWCOL = torch.stack(((_IDX // 4) / 3, (_IDX % 4) / 3), dim=1)


def to_model_format(b) -> torch.Tensor:
    cells = torch.tensor(b, dtype=torch.float32).view(16, 1)
    return torch.cat((cells, _ROWCOL), dim=1).view(-1)


@torch.no_grad()
def play_game(model, rnd: random.Random, max_steps: int | None = None) -> dict:
    b = pyref.reset(rnd)
    moves = []
    total = 0
    step = 0
    while not max_steps or step < max_steps:
        legal = pyref.legal_mask(b)
        if legal == 0:
            break
        state_before = [b[0:4], b[4:8], b[8:12], b[12:16]]
        x = to_model_format(b)
        logits, value = model(x.unsqueeze(0))
        logits = logits.squeeze(0)
        invalid = [not (legal >> d & 1) for d in range(4)]
        logits[invalid] = -torch.inf
        probs = torch.softmax(logits, dim=-1)
        a = int(torch.multinomial(probs, 1).item())
        p = probs[probs > 0]
        ent = -(p * p.log()).sum().item()
        mono_b, empt_b = pyref.monotonicity(b), pyref.emptiness(b)
        pts, done, info = pyref.step(b, a, rnd)
        total += pts
        moves.append({"game_state": x, "selected_direction": a, "action_mask": invalid, "points_earned": pts,
                      "state_before": state_before, "result_state": [b[0:4], b[4:8], b[8:12], b[12:16]],
                      "monotonicity_before": mono_b, "monotonicity_after": 0.0 if done else pyref.monotonicity(b),
                      "emptiness_before": empt_b, "emptiness_after": 0.0 if done else pyref.emptiness(b),
                      "predicted_future_value": value.item(), "entropy": ent,
                      "policy_logprobs": logits.log_softmax(-1).tolist(), "done": done})
        if done:
            break
        step += 1
    return {"moves": moves, "total_points": total, "total_steps": step}


def calculate_advantage(ep: dict, state: list, step: int, gamma=0.99, wp=0.10, wm=1.0, we=0.0, beta=0.99,
                        upsample=0.25, rnd=random):
    from g2048.augment import augment_steps
    mv = ep["moves"]
    col = lambda k: np.array([m[k] for m in mv], np.float64)  # noqa: E731
    ends = np.zeros(len(mv), bool)
    ends[-1] = True
    r = O.reward_rtg_normalize(col("points_earned").astype(np.int64), col("monotonicity_before"),
                               col("monotonicity_after"), col("emptiness_before"), col("emptiness_after"),
                               col("done").astype(np.int64), col("predicted_future_value"), ends, gamma, wp, wm, we,
                               beta, state[1], state[2], step, rtg_first_moment=state[0])
    for k, m in enumerate(mv):
        m["advantage"] = float(r["adv"][k])
        m["future_reward"] = float(r["g_norm"][k])
    state[:] = list(r["moments"])
    return augment_steps(mv, upsample, rnd) if upsample > 0 else []


def time_train_loop(seconds: float, hidden: int = 196, batch_size: int = 4, seed: int = 0x2048,
                    max_iters: int = 50) -> dict:
    """README train loop on 1 process, torch on 1 thread; env-steps (moves played) per wall second,
    rollout + advantage + update included."""
    import agent
    import train as T
    from g2048.optim import build_optimizer
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        torch.manual_seed(seed)
        rnd = random.Random(seed)
        model = agent.GameMLP(agent.MLPConfig(hidden_dim=hidden, num_layers=2))
        with torch.no_grad():  # train.py:1559-1567
            for p in (model.action_head.weight, model.action_head.bias, model.value_head.weight,
                      model.value_head.bias):
                p.zero_()
        opt = build_optimizer(model, 1e-3, 1e-4, 0.9, 0.999, 0.01, 10, 20000)
        state = [0.0, 1.0, 0.0]  # first moment, m2, mu (train.py:1550-1552)
        n = it = 0
        t0 = time.perf_counter()
        while it < max_iters and (it == 0 or time.perf_counter() - t0 < seconds):
            model.eval()
            ep = play_game(model, rnd)
            aug = calculate_advantage(ep, state, it + 1, rnd=rnd)
            eps = [ep] + ([{"moves": aug}] if aug else [])
            T.model_optimize_step(model, eps, opt, None, 0.02, 0.2, batch_size=batch_size, epochs=1)
            n += len(ep["moves"])
            it += 1
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(threads)
    return {"value": n / dt, "unit": "env-steps/s", "cores": 1, "iters": it, "steps": n, "seconds": dt,
            "sample": f"{it} README train steps (1 game each, h={hidden}, minibatch {batch_size}, upsample 0.25, "
                      f"Muon+AdamW) = {n} env steps, torch 1 thread, {dt:.1f} s"}
