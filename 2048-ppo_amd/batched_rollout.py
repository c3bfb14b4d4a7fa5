"""batched_rollout -- the module the reference imports but does not ship (train.py:30).

play_games_batched(model, num_games, max_steps, device) -> list[EpisodeData]

Called by the reference trainer when --episodes > 1 (train.py:1676-1679) and by export-demo
(train.py:2032-2034).  All `num_games` games run at once on the GPU (one libg2048 env-step launch
per move for every game, the policy forward batched over the live games); every game plays to its
end (or `max_steps` moves), exactly like play_game_for_episode (train.py:213-345).

Semantics chosen where the reference is silent (the module is missing, so this is unpinned):
  * total_steps follows play_game_for_episode: number of moves - 1 for a game that ended, the
    number of moves for one cut by max_steps.
  * spawns: Philox4x32-10 keyed from Python's `random` module state, so `random.seed(s)` makes a
    batch reproducible; action sampling: the device sampler (torch.multinomial's stream is not
    reproducible across implementations in any case).
  * info-only heuristic deltas (smoothness/corner/adjacency/chain/topological, game.py:981-1002)
    come from the g2048_info_deltas kernel, bit-identical to game.step's; they never reach the
    reward (train.py:702-719) but feed the breakdown tables and the --viz-dir export.
"""

from __future__ import annotations

import random

import torch


def _device(device) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("play_games_batched needs a ROCm GPU: libg2048 has no CPU path")
    d = torch.device(device) if device is not None else torch.device("cuda", 0)
    return d if d.type == "cuda" else torch.device("cuda", 0)


def play_games_batched(model: torch.nn.Module, num_games: int, max_steps: int | None = None, device=None):
    from g2048.episodes import play_games
    dev = _device(device)
    params = list(model.parameters())
    runner = model
    if params and params[0].device != dev:
        import copy
        runner = copy.deepcopy(model).to(dev)
    was = runner.training
    runner.eval()
    try:
        res = play_games(runner, int(num_games), max_steps, dev, seed=random.getrandbits(63), record=True)
    finally:
        runner.train(was)
    return res["episodes"]


__all__ = ["play_games_batched"]
