"""Whole-game play on the device and conversion to the reference's EpisodeData records.

`play_games` runs `num_games` envs episodically (one full game each, train.py:213-345 semantics)
with any policy module; `to_episode_data` turns the device trajectory into the list-of-dict
EpisodeData/StepData schema of train.py:123-177 for the `batched_rollout` seam (Python scalars,
game_state as a [48] float32 tensor, grids as list-of-lists).
"""

from __future__ import annotations

import torch

from . import _lib as L
from .rollout import Rollout

DIRECTION_NAMES = ["UP", "DOWN", "LEFT", "RIGHT"]


class _ModulePolicy:
    """Call a policy module (fp32, eval) the way the rollout expects."""

    def __init__(self, model):
        self.model = model

    @torch.no_grad()
    def __call__(self, obs):
        logits, value = self.model(obs.float())
        return logits.float(), value.float().reshape(-1)


@torch.no_grad()
def play_games(model, num_games: int, max_steps: int | None, device, seeds=None, seed: int = 0x5EED,
               record: bool = True, chunk: int = 64, cap: int = 1 << 15) -> dict:
    """Play `num_games` complete games (or until max_steps moves).  seeds[i] given -> game i's spawns
    follow CPython random.seed(seeds[i]) exactly (MT19937 on the device)."""
    dev = torch.device(device)
    limit = max_steps if max_steps and max_steps > 0 else cap
    T = -(-limit // chunk) * chunk
    # grow the buffer geometrically rather than allocating `cap` steps up front
    T_alloc = min(T, 2048)
    policy = _ModulePolicy(model)
    ro = Rollout(num_games, T_alloc, dev, seed=seed, episodic=True, obs_dtype=torch.float32, mt_seeds=seeds)
    ro.reset()
    t = 0
    while True:
        if t == ro.T and t < T:
            ro = _grow(ro, min(T, 2 * ro.T))
        end = min(t + chunk, ro.T)
        for s in range(t, end):
            ro._step(s, policy)
        t = end
        if t >= limit or bool(((ro.buf.flags[t] & L.FLAG_LEGAL) == 0).all()):
            break
    ro.counter.add_(2 * t)
    n_moves_cap = min(t, limit)
    return _summarise(ro, n_moves_cap, limit, record)


def _grow(ro: Rollout, new_T: int) -> Rollout:
    old = ro.buf
    nro = Rollout(ro.n, new_T, old.device, seed=ro.seed, env_base=ro.env_base, episodic=True,
                  obs_dtype=old.obs.dtype)
    nro.mt_state, nro.counter = ro.mt_state, ro.counter
    nb = nro.buf
    T = old.T
    for name in ("boards", "flags"):
        getattr(nb, name)[:T + 1].copy_(getattr(old, name))
    for name in ("actions", "logp", "entropy", "value", "points", "max_tile", "pot"):
        getattr(nb, name)[:T].copy_(getattr(old, name))
    return nro


def _summarise(ro: Rollout, T: int, limit: int, record: bool) -> dict:
    b = ro.buf
    sf = b.step_flags[:T]
    active = (sf & L.FLAG_INACTIVE) == 0                     # a move was made at step t
    n_moves = active.sum(0)                                   # [N]
    scores = torch.where(active, b.points[:T], 0).sum(0)
    final = b.boards[n_moves, torch.arange(ro.n, device=b.device)]  # board after the last move
    maxexp = final.max(dim=1).values.to(torch.int64)
    out = {"scores": scores.tolist(), "moves": n_moves.tolist(),
           "max_tiles": [0 if e == 0 else 1 << e for e in maxexp.tolist()], "T": T, "rollout": ro,
           "limit": limit}
    if record:
        out["episodes"] = to_episode_data(ro, T, n_moves, limit)
    return out


def to_episode_data(ro: Rollout, T: int, n_moves: torch.Tensor, limit: int) -> list[dict]:
    """Device trajectory -> list[EpisodeData] (train.py:123-177, 299-344)."""
    b = ro.buf
    n = ro.n
    boards = b.boards[:T + 1].cpu().numpy()
    obs = torch.empty(T, n, 48, dtype=torch.float32, device=b.device)
    for t in range(T):
        L.obs_encode(b.boards[t], obs[t])
    prev = torch.zeros(T, n, 4, dtype=torch.int32, device=b.device)
    for t in range(T):
        L.preview_points(b.boards[t], prev[t])
    # the info-only heuristic deltas of every step (game.py:981-1002), on the device
    info = torch.zeros(T * n, 5, dtype=torch.float64, device=b.device)
    anchor = torch.zeros(T * n, dtype=torch.int8, device=b.device)
    if T > 0:
        L.info_deltas(b.boards[:T].reshape(T * n, 16), b.actions[:T].reshape(T * n), info, anchor)
    info = info.view(T, n, 5).cpu().numpy()
    anchor = anchor.view(T, n).cpu().numpy()
    obs = obs.cpu()
    prev = prev.cpu().numpy()
    sf = b.step_flags[:T].cpu().numpy()
    legal = b.flags[:T].cpu().numpy()
    acts = b.actions[:T].cpu().numpy()
    logp = b.logp[:T].cpu().numpy()
    ent = b.entropy[:T].cpu().numpy()
    val = b.value[:T].cpu().numpy()
    pts = b.points[:T].cpu().numpy()
    mxt = b.max_tile[:T].cpu().numpy()
    pot = b.pot[:T].cpu().numpy()
    nm = n_moves.tolist()
    from agent import Direction  # noqa: F401  (the keys of points_possible)
    dirs = [Direction.UP, Direction.DOWN, Direction.LEFT, Direction.RIGHT]
    episodes = []
    for e in range(n):
        moves = []
        total = 0
        k = nm[e]
        for t in range(k):
            done = bool(sf[t, e] & L.FLAG_DONE)
            grid_b = boards[t, e].reshape(4, 4).tolist()
            grid_a = boards[t + 1, e].reshape(4, 4).tolist()
            p4 = prev[t, e].tolist()
            mexp_b = int(boards[t, e].max())
            total += int(pts[t, e])
            moves.append({
                "predicted_future_value": float(val[t, e]),
                "selected_direction": int(acts[t, e]),
                "game_state": obs[t, e],
                "state_before": grid_b,
                "result_state": grid_a,
                "max_points_possible": max(p4),
                "points_earned": int(pts[t, e]),
                "points_possible": dict(zip(dirs, p4)),
                "action_mask": [not (legal[t, e] >> a & 1) for a in range(4)],
                "smoothness_delta": float(info[t, e, 0]), "corner_delta": float(info[t, e, 1]),
                "adjacency_delta": float(info[t, e, 2]), "chain_delta": float(info[t, e, 3]),
                "topological_delta": float(info[t, e, 4]),
                "topological_anchor": (int(anchor[t, e]) // 4, int(anchor[t, e]) % 4),
                "max_tile_created": int(mxt[t, e]),
                "max_exponent_before": mexp_b,
                "max_exponent_after": max(mexp_b, int(mxt[t, e])),
                "monotonicity_before": int(pot[t, e, 0]),
                "monotonicity_after": 0.0 if done else int(pot[t, e, 1]),   # train.py:318
                "emptiness_before": int(pot[t, e, 2]),
                "emptiness_after": 0.0 if done else int(pot[t, e, 3]),      # train.py:322
                "entropy": float(ent[t, e]),
                "policy_logprobs": [float(x) for x in logp[t, e]],
            })
        ended = k > 0 and bool(sf[k - 1, e] & L.FLAG_DONE)
        total_steps = k - 1 if ended else k  # play_game_for_episode's `step` counter (train.py:334-343)
        episodes.append({"moves": moves, "total_points": total, "total_steps": total_steps,
                         "final_state": boards[k, e].reshape(4, 4).tolist()})
    return episodes
