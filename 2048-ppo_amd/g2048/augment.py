"""D4 up-sampling of training steps (calculate_advantage's augmentation, train.py:774-881).

`augment_steps` follows the reference exactly, including its use of Python's global `random`
module (random.sample of int(N * ratio) steps, then per step a 0.5 mirror draw with a random axis
and an independent 0.5 rotation draw with a random angle), so under the same `random` state it picks
the same samples and transforms.  Boards, the action, the action mask and the old log-probs are
remapped; the model input is re-encoded (to_model_format, game.py:92-101) from the transformed board.
points_possible is permuted with the directions (the game is D4-symmetric, so this equals
preview_move_rewards on the transformed board).
"""

from __future__ import annotations

import copy
import random

import torch

_UP, _DOWN, _LEFT, _RIGHT = 0, 1, 2, 3
_ROT90 = {_UP: _RIGHT, _RIGHT: _DOWN, _DOWN: _LEFT, _LEFT: _UP}  # train.py:797-803


def mirror_grid(g, axis: str):
    if axis == "horizontal":
        return [list(reversed(row)) for row in g]
    if axis == "vertical":
        return [list(row) for row in reversed(g)]
    raise ValueError(f"Invalid direction: {axis}. Must be 'horizontal' or 'vertical'")


def rotate_grid(g, degrees: int):
    """Clockwise rotation (game.py:537-590): new[j][3-i] = old[i][j] for 90 degrees."""
    out = [list(row) for row in g]
    for _ in range((degrees // 90) % 4):
        out = [[out[3 - j][i] for j in range(4)] for i in range(4)]
    return out


def remap_mirror(d: int, axis: str) -> int:
    if axis == "horizontal" and d in (_LEFT, _RIGHT):
        return _LEFT if d == _RIGHT else _RIGHT
    if axis == "vertical" and d in (_UP, _DOWN):
        return _UP if d == _DOWN else _DOWN
    return d


def remap_rotate(d: int, degrees: int) -> int:
    for _ in range(degrees // 90):
        d = _ROT90[d]
    return d


def _permute(values, fn, arg):
    out = [None] * 4
    for k in range(4):
        out[fn(k, arg)] = values[k]
    return out


def encode_grid(g) -> torch.Tensor:
    """to_model_format of one grid (host side, float32 exact)."""
    cells = torch.tensor([c for row in g for c in row], dtype=torch.float32)
    idx = torch.arange(16)
    return torch.stack((cells, (idx // 4) / 3, (idx % 4) / 3), dim=1).reshape(-1)


def _transform(step: dict, grid_fn, dir_fn, arg) -> dict:
    s = copy.deepcopy({k: v for k, v in step.items() if k != "game_state"})
    s["state_before"] = grid_fn(step["state_before"], arg)
    s["result_state"] = grid_fn(step["result_state"], arg)
    s["game_state"] = encode_grid(s["state_before"])
    s["selected_direction"] = dir_fn(step["selected_direction"], arg)
    s["action_mask"] = _permute(step.get("action_mask", [False] * 4), dir_fn, arg)
    s["policy_logprobs"] = _permute(step.get("policy_logprobs", [0.0] * 4), dir_fn, arg)
    if isinstance(step.get("points_possible"), dict):
        keys = list(step["points_possible"].keys())
        vals = [step["points_possible"][k] for k in keys]
        s["points_possible"] = dict(zip(keys, _permute(vals, dir_fn, arg)))
    return s


def augment_steps(steps: list[dict], upsample_ratio: float, rnd=random) -> list[dict]:
    k = int(len(steps) * upsample_ratio)
    if k <= 0:
        return []
    out = []
    for step in rnd.sample(steps, min(k, len(steps))):
        if rnd.random() < 0.5:
            axis = rnd.choice(["horizontal", "vertical"])
            out.append(_transform(step, mirror_grid, remap_mirror, axis))
        if rnd.random() < 0.5:
            deg = rnd.choice([90, 180, 270])
            out.append(_transform(step, rotate_grid, remap_rotate, deg))
    return out
