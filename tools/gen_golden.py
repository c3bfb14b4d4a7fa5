"""Generate the golden fixtures under tests/golden/ by running the REFERENCE code in this container.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py

Every array written here is produced by the reference's own functions (loaded read-only through
tools/refshim.py) or copied from the reference's shipped data files (docs/data/*.json, *.pt loaded
with weights_only=True).  The fixtures are data only (inputs + expected outputs); no reference
source travels with them.

Fixture files (all npz, allow_pickle=False):
  rows.npz        slide/merge table: game.py:225-257 (LEFT/RIGHT) + legality game.py:260-330
  games.npz       64 seeded games: random.seed(s); reset(); step(a) with recorded actions
                  (game.py:923-1030), incl. ~5% deliberately illegal actions (game.py:959-978)
  best_game.npz   docs/data/best_game.json (1249 moves) converted to exponents, spawn recovered
  advantage.npz   calculate_advantage (train.py:651-904) over several (gamma, weights, moments)
  mlp.npz         docs/data/best_model.pt weights + GameMLP forward (game.py:1145-1220) + obs
                  encoding to_model_format (game.py:92-101)
  sampler.npz     masked softmax / log_softmax / entropy of the rollout (train.py:266-326)
  update.npz      one model_optimize_step (train.py:414-642) with dropout 0, single minibatch
  urm.npz         GameURM forward (game.py:1355-1458), small random-init config
  urm64.npz       GameURM forward at the default GameURMConfig (h 64: BASELINE config 5), 512 boards
                  (`python tools/gen_golden.py urm64` regenerates only this file)
  mlp196.npz      GameMLP forward at the bench's train configuration (h 196, 2 blocks), 512 boards
  update196.npz   model_optimize_step at h 196, dropout 0, 4 096 rows in two minibatches of 2 048, the
                  DataLoader order recorded (`python tools/gen_golden.py update196`)
  update196e4.npz the same inputs over four epochs (eight optimizer steps): orders, the eight grad
                  norms, final weights and the final policy's outputs (`... update196e4`)
"""

from __future__ import annotations

import json
import random
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from refshim import REF, load_reference  # noqa: E402

OUT = Path(__file__).resolve().parent.parent / "tests" / "golden"
DIRS = None  # filled after load: [UP, DOWN, LEFT, RIGHT]


def flat(grid) -> list[int]:
    return [c for row in grid for c in row]


def grid_of(vals) -> list[list[int]]:
    v = [int(x) for x in vals]
    return [v[0:4], v[4:8], v[8:12], v[12:16]]


def gen_rows(game):
    G = game.Game2048
    rows = [[a, b, c, d] for a in range(13) for b in range(13) for c in range(13) for d in range(13)]
    rng = np.random.default_rng(7)
    rows += rng.integers(0, 18, size=(8192, 4)).tolist()
    # rows dense in high exponents (16, 17) so merges creating 17/18 are covered
    rows += rng.integers(14, 18, size=(1024, 4)).tolist()
    R = len(rows)
    out = {k: np.zeros((R, 4), np.int8) for k in ("left", "right")}
    pts = {k: np.zeros(R, np.int64) for k in ("left", "right")}
    mx = {k: np.zeros(R, np.int8) for k in ("left", "right")}
    legal = np.zeros((R, 2), np.uint8)
    for i, r in enumerate(rows):
        lo, lp, lm = G._merge_and_shift_left_with_score(list(r))
        ro, rp, rm = G._merge_and_shift_right_with_score(list(r))
        out["left"][i], pts["left"][i], mx["left"][i] = lo, lp, lm
        out["right"][i], pts["right"][i], mx["right"][i] = ro, rp, rm
        board = [list(r), [0] * 4, [0] * 4, [0] * 4]
        for k, d in enumerate((game.Direction.LEFT, game.Direction.RIGHT)):
            legal[i, k] = G.can_move_in_direction(board, d) or G.can_merge_in_direction(board, d)
    np.savez_compressed(
        OUT / "rows.npz",
        rows=np.array(rows, np.int8),
        left=out["left"], left_points=pts["left"], left_max=mx["left"],
        right=out["right"], right_points=pts["right"], right_max=mx["right"],
        legal_lr=legal,
    )
    print(f"rows.npz: {R} rows")


def legal_mask(game, grid) -> int:
    m = 0
    for k, d in enumerate(DIRS):
        if game.Game2048.can_move_in_direction(grid, d) or game.Game2048.can_merge_in_direction(grid, d):
            m |= 1 << k
    return m


def gen_games(game, n_games=64, max_steps=3000):
    G = game.Game2048
    rec = {k: [] for k in (
        "game", "t", "before", "action", "moved", "after", "points", "max_tile", "mono_b", "mono_a",
        "empt_b", "empt_a", "invalid", "done", "mask_before", "mask_after",
        "smooth_d", "corner_d", "adj_d", "chain_d", "topo_d", "maxexp_b", "maxexp_a")}
    init_boards = []
    for s in range(n_games):
        random.seed(s)
        g = G()
        g.reset()
        init_boards.append(flat(g.grid))
        arng = np.random.default_rng(10_000 + s)
        t = 0
        while g.has_next_step() and t < max_steps:
            before = [row[:] for row in g.grid]
            mb = legal_mask(game, before)
            legal = [k for k in range(4) if mb >> k & 1]
            illegal = [k for k in range(4) if not mb >> k & 1]
            if illegal and arng.random() < 0.05:
                a = int(arng.choice(illegal))
            else:
                a = int(arng.choice(legal))
            moved, _, _ = G.simulate_move(before, DIRS[a])
            new_state, pts, done, info = g.step(DIRS[a])
            rec["game"].append(s)
            rec["t"].append(t)
            rec["before"].append(flat(before))
            rec["action"].append(a)
            rec["moved"].append(flat(moved) if not info["invalid_move"] else flat(before))
            rec["after"].append(flat(new_state))
            rec["points"].append(pts)
            rec["max_tile"].append(info["max_tile_created"])
            rec["mono_b"].append(info["monotonicity_before"])
            rec["mono_a"].append(info["monotonicity_after"])
            rec["empt_b"].append(info["emptiness_before"])
            rec["empt_a"].append(info["emptiness_after"])
            rec["invalid"].append(int(info["invalid_move"]))
            rec["done"].append(int(done))
            rec["mask_before"].append(mb)
            rec["mask_after"].append(legal_mask(game, new_state))
            rec["smooth_d"].append(info["smoothness_delta"])
            rec["corner_d"].append(info["corner_delta"])
            rec["adj_d"].append(info["adjacency_delta"])
            rec["chain_d"].append(info["chain_delta"])
            rec["topo_d"].append(info["topological_delta"])
            rec["maxexp_b"].append(info.get("max_exponent_before", 0))
            rec["maxexp_a"].append(info.get("max_exponent_after", 0))
            t += 1
            if done:
                break
    arrays = {}
    for k, v in rec.items():
        if k in ("before", "moved", "after"):
            arrays[k] = np.array(v, np.int8)
        elif k.endswith("_d"):
            arrays[k] = np.array(v, np.float64)
        else:
            arrays[k] = np.array(v, np.int64)
    arrays["init_boards"] = np.array(init_boards, np.int8)
    np.savez_compressed(OUT / "games.npz", **arrays)
    print(f"games.npz: {len(rec['t'])} steps over {n_games} games")
    return arrays


def gen_best_game(game):
    G = game.Game2048
    data = json.loads((REF / "docs" / "data" / "best_game.json").read_text())
    names = ["UP", "DOWN", "LEFT", "RIGHT"]

    def to_exp(grid):
        return [[0 if v == 0 else int(v).bit_length() - 1 for v in row] for row in grid]

    before, after, moved, acts, pts, spawn_cell, spawn_val, k_idx = [], [], [], [], [], [], [], []
    for m in data["moves"]:
        b = to_exp(m["state_before"])
        a = to_exp(m["state_after"])
        d = names.index(m["action"])
        mv, p, _ = G.simulate_move(b, DIRS[d])
        assert p == m["points_earned"], "points mismatch in best_game.json"
        diff = [i for i in range(16) if flat(mv)[i] != flat(a)[i]]
        assert len(diff) == 1 and flat(mv)[diff[0]] == 0
        cell = diff[0]
        empties = [i for i in range(16) if flat(mv)[i] == 0]
        before.append(flat(b)); after.append(flat(a)); moved.append(flat(mv))
        acts.append(d); pts.append(p)
        spawn_cell.append(cell); spawn_val.append(flat(a)[cell]); k_idx.append(empties.index(cell))
    np.savez_compressed(
        OUT / "best_game.npz",
        before=np.array(before, np.int8), after=np.array(after, np.int8),
        moved=np.array(moved, np.int8), action=np.array(acts, np.int64),
        points=np.array(pts, np.int64), spawn_cell=np.array(spawn_cell, np.int64),
        spawn_val=np.array(spawn_val, np.int64), spawn_k=np.array(k_idx, np.int64),
        score=np.int64(data["score"]), total_steps=np.int64(data["total_steps"]),
    )
    print(f"best_game.npz: {len(acts)} moves, score {data['score']}")


ADV_CASES = [
    # gamma, w_points, w_mono, w_empt, rtg_beta, rtg_m2, rtg_mu, rtg_step
    (0.99, 0.10, 1.0, 0.0, 0.99, 1.0, 0.0, 1),       # README config, first train step
    (0.99, 0.10, 1.0, 0.0, 0.99, 2500.0, 30.0, 7),
    (0.95, 1.00, 0.0, 0.5, 0.90, 1.0e4, 80.0, 50),
    (0.90, 0.00, 0.7, 1.3, 0.999, 3.0, 1.0, 3),
    (1.00, 0.25, 0.2, 0.2, 0.5, 10.0, -2.0, 1000),
]


def gen_advantage(train, games):
    n_eps = 16
    sel = games["game"] < n_eps
    vrng = np.random.default_rng(99)
    value = vrng.normal(size=int(sel.sum())).astype(np.float32).astype(np.float64)
    out = {"episode": games["game"][sel], "points": games["points"][sel],
           "mono_b": games["mono_b"][sel], "mono_a": games["mono_a"][sel],
           "empt_b": games["empt_b"][sel], "empt_a": games["empt_a"][sel],
           "done": games["done"][sel], "value": value, "cases": np.array(ADV_CASES, np.float64)}
    for ci, (gamma, wp, wm, we, beta, m2, mu, step) in enumerate(ADV_CASES):
        episodes = []
        idx = 0
        for e in range(n_eps):
            moves = []
            while idx < len(out["episode"]) and out["episode"][idx] == e:
                done = bool(out["done"][idx])
                moves.append({
                    "points_earned": int(out["points"][idx]),
                    # train.py:318,322 zero the "after" potentials on the terminal step
                    "monotonicity_before": out["mono_b"][idx],
                    "monotonicity_after": 0.0 if done else out["mono_a"][idx],
                    "emptiness_before": out["empt_b"][idx],
                    "emptiness_after": 0.0 if done else out["empt_a"][idx],
                    "predicted_future_value": float(value[idx]),
                })
                idx += 1
            episodes.append({"moves": moves, "total_points": 0, "total_steps": len(moves), "final_state": None})
        eps, aug, fm, nm2, nmu = train.calculate_advantage(
            episodes, gamma, mu, wp, 1.0, 1.0, 1.0, 1.0, 1.0, wm, we, 1.0, 1000.0,
            rtg_beta=beta, rtg_m2=m2, rtg_mu=mu, rtg_step=int(step), upsample_ratio=0.0)
        allm = [m for ep in eps for m in ep["moves"]]
        out[f"c{ci}_reward"] = np.array([m["reward"] for m in allm])
        out[f"c{ci}_g_raw"] = np.array([m["future_reward_raw"] for m in allm])
        out[f"c{ci}_g_norm"] = np.array([m["future_reward"] for m in allm])
        out[f"c{ci}_adv"] = np.array([m["advantage"] for m in allm])
        out[f"c{ci}_moments"] = np.array([fm, nm2, nmu])
    np.savez_compressed(OUT / "advantage.npz", **out)
    print(f"advantage.npz: {len(ADV_CASES)} cases over {int(sel.sum())} steps")


def gen_mlp(game, games):
    ck = torch.load(REF / "docs" / "data" / "best_model.pt", map_location="cpu", weights_only=True)
    cfg = game.MLPConfig(**ck["config"])
    model = game.GameMLP(cfg)
    model.load_state_dict(ck["model_state_dict"])
    model.eval()
    rng = np.random.default_rng(3)
    pick = rng.choice(len(games["before"]), size=256, replace=False)
    boards = games["before"][pick]
    obs = torch.stack([game.Game2048(grid_of(b)).to_model_format() for b in boards])
    with torch.no_grad():
        logits, value = model(obs)
    arrays = {f"w::{k}": v.numpy() for k, v in ck["model_state_dict"].items()}
    arrays.update(boards=boards, obs=obs.numpy(), logits=logits.numpy(), value=value.numpy(),
                  hidden_dim=np.int64(cfg.hidden_dim), num_layers=np.int64(cfg.num_layers),
                  eval_avg_score=np.float64(ck["eval_avg_score"]), train_step=np.int64(ck["train_step"]))
    np.savez_compressed(OUT / "mlp.npz", **arrays)
    print(f"mlp.npz: best_model.pt h={cfg.hidden_dim} L={cfg.num_layers}, 256 boards")


def gen_sampler():
    g = torch.Generator().manual_seed(5)
    B = 512
    logits = torch.randn(B, 4, generator=g) * 3.0
    mask = torch.rand(B, 4, generator=g) < 0.35  # True = invalid (train.py:268)
    mask[mask.all(dim=1)] = torch.tensor([True, False, True, True])
    logp, ent, probs = [], [], []
    for i in range(B):
        al = logits[i].clone()
        al[mask[i]] = -torch.inf  # train.py:271
        p = torch.softmax(al, dim=-1)  # train.py:274
        vp = p[p > 0]
        ent.append(-(vp * vp.log()).sum().item())  # train.py:290-291
        logp.append(al.log_softmax(dim=-1))  # train.py:326
        probs.append(p)
    np.savez_compressed(OUT / "sampler.npz", logits=logits.numpy(), invalid=mask.numpy(),
                        probs=torch.stack(probs).numpy(), logp=torch.stack(logp).numpy(),
                        entropy=np.array(ent, np.float64))
    print("sampler.npz: 512 cases")


def gen_update(game, train, games):
    torch.manual_seed(1234)
    cfg = game.MLPConfig(hidden_dim=64, num_layers=2, dropout=0.0, decouple_critic=False)
    model = game.GameMLP(cfg)
    sel = np.nonzero(games["game"] < 2)[0][:160]
    boards = games["before"][sel]
    obs = torch.stack([game.Game2048(grid_of(b)).to_model_format() for b in boards])
    invalid = np.array([[not (m >> k & 1) for k in range(4)] for m in games["mask_before"][sel]])
    actions = games["action"][sel].copy()
    # the trainer only ever samples legal actions; replace the fixture's deliberate illegal ones
    for i in range(len(actions)):
        if invalid[i, actions[i]]:
            actions[i] = int(np.nonzero(~invalid[i])[0][0])
    rng = np.random.default_rng(11)
    adv = rng.normal(size=len(sel)).astype(np.float32)
    fut = rng.normal(size=len(sel)).astype(np.float32)
    with torch.no_grad():
        lg, _ = model(obs)
        lg = lg.masked_fill(torch.from_numpy(invalid), float("-inf"))
        old_lp = lg.log_softmax(-1) + torch.from_numpy(rng.normal(scale=0.05, size=(len(sel), 4)).astype(np.float32))
    moves = [{"game_state": obs[i], "selected_direction": int(actions[i]), "action_mask": invalid[i].tolist(),
              "advantage": float(adv[i]), "future_reward": float(fut[i]), "policy_logprobs": old_lp[i].tolist()}
             for i in range(len(sel))]
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    o2d, o1d, v2d, v1d = model.get_param_groups(1e-4, 1e-3)
    adamw = torch.optim.AdamW([o1d, v1d], betas=(0.9, 0.999), weight_decay=0.01)
    muon = torch.optim.Muon([o2d, v2d], adjust_lr_fn="match_rms_adamw", weight_decay=0.01)
    opt = train.MultiOptimizer(muon, adamw)
    stats = train.model_optimize_step(model=model, episodes=[{"moves": moves}], optimizer=opt,
                                      lr_scheduler=None, kl_strength=0.02, critic_strength=0.2,
                                      device=None, batch_size=len(moves), epochs=1)
    arrays = {f"init::{k}": v.numpy() for k, v in init.items()}
    arrays.update({f"final::{k}": v.detach().numpy() for k, v in model.state_dict().items()})
    arrays.update(obs=obs.numpy(), actions=actions, invalid=invalid, advantage=adv, future_reward=fut,
                  old_logprobs=old_lp.numpy(), stat_keys=np.array(sorted(stats)),
                  stat_vals=np.array([float(stats[k]) for k in sorted(stats)]),
                  hparams=np.array([1e-3, 1e-4, 0.9, 0.999, 0.01, 0.02, 0.2]))
    np.savez_compressed(OUT / "update.npz", **arrays)
    print(f"update.npz: h=64 single minibatch of {len(moves)}; stats {stats}")


def _update196_inputs(game, n=4096):
    """The inputs of update196.npz / update196e4.npz: GameMLP h 196 at torch.manual_seed(1960), n rows
    of the golden games (illegal recorded actions replaced by the first legal one), advantages and
    returns from default_rng(196), old log-probabilities = the initial policy's + N(0, 0.05)."""
    torch.manual_seed(1960)
    cfg = game.MLPConfig(hidden_dim=196, num_layers=2, dropout=0.0, decouple_critic=False)
    model = game.GameMLP(cfg)
    g = np.load(OUT / "games.npz")
    boards = g["before"][:n]
    obs = torch.stack([game.Game2048(grid_of(b)).to_model_format() for b in boards])
    assert np.array_equal(np.rint(obs[:, 0::3].numpy()).astype(np.int8), boards)  # exponent channel
    invalid = np.array([[not (m >> k & 1) for k in range(4)] for m in g["mask_before"][:n]])
    actions = g["action"][:n].copy()
    for i in range(n):  # the trainer samples legal actions only (the fixture's games hold ~5 % illegal)
        if invalid[i, actions[i]]:
            actions[i] = int(np.nonzero(~invalid[i])[0][0])
    rng = np.random.default_rng(196)
    adv = rng.normal(size=n).astype(np.float32)
    fut = rng.normal(size=n).astype(np.float32)
    with torch.no_grad():  # heads at their Kaiming init: non-uniform old policies
        lg, _ = model(obs)
        lg = lg.masked_fill(torch.from_numpy(invalid), float("-inf"))
        old_lp = lg.log_softmax(-1) + torch.from_numpy(rng.normal(scale=0.05, size=(n, 4)).astype(np.float32))
    moves = [{"game_state": obs[i], "selected_direction": int(actions[i]), "action_mask": invalid[i].tolist(),
              "advantage": float(adv[i]), "future_reward": float(fut[i]), "policy_logprobs": old_lp[i].tolist()}
             for i in range(n)]
    return model, boards, obs, invalid, actions, adv, fut, old_lp, moves


def _run_recorded(train, model, moves, batch_size, epochs, lr=1e-3, clr=1e-4, wd=0.01):
    """model_optimize_step (train.py:414-642) with Muon (match_rms_adamw) + AdamW at fixed learning
    rates, the DataLoader's RandomSampler order and every clip_grad_norm_ result recorded."""
    import torch.utils.data as tud
    o2d, o1d, v2d, v1d = model.get_param_groups(clr, lr)
    adamw = torch.optim.AdamW([o1d, v1d], betas=(0.9, 0.999), weight_decay=wd)
    muon = torch.optim.Muon([o2d, v2d], adjust_lr_fn="match_rms_adamw", weight_decay=wd)
    opt = train.MultiOptimizer(muon, adamw)
    order, norms = [], []
    orig_iter, orig_clip = tud.RandomSampler.__iter__, torch.nn.utils.clip_grad_norm_

    def rec_iter(self):
        for i in orig_iter(self):
            order.append(int(i))
            yield i

    def rec_clip(params, max_norm, *a, **k):
        r = orig_clip(params, max_norm, *a, **k)
        norms.append(float(r))
        return r
    tud.RandomSampler.__iter__ = rec_iter
    torch.nn.utils.clip_grad_norm_ = rec_clip
    try:
        stats = train.model_optimize_step(model=model, episodes=[{"moves": moves}], optimizer=opt,
                                          lr_scheduler=None, kl_strength=0.02, critic_strength=0.2,
                                          device=None, batch_size=batch_size, epochs=epochs)
    finally:
        tud.RandomSampler.__iter__ = orig_iter
        torch.nn.utils.clip_grad_norm_ = orig_clip
    return stats, order, norms


def gen_update196e4(game, train):
    """update196e4.npz: the multi-step pin.  The same inputs and initial weights as update196.npz
    (asserted equal), run through model_optimize_step for FOUR epochs of two minibatches of 2 048 --
    eight consecutive optimizer steps, each epoch in its own recorded shuffle order -- so a test can
    measure how far the bf16 device update drifts from the fp32 reference over several steps.
    Stored: the 4 x 4 096 order, the eight clip_grad_norm_ results, the reference's statistics, the
    final weights, and the final policy's logits / value on the 4 096 boards (eval mode; dropout 0).
    The initial weights and inputs are update196.npz's (not stored again).
    `python tools/gen_golden.py update196e4` regenerates only this file."""
    model, boards, obs, invalid, actions, adv, fut, old_lp, moves = _update196_inputs(game)
    base = np.load(OUT / "update196.npz")
    for k, v in model.state_dict().items():
        assert np.array_equal(v.numpy(), base[f"init::{k}"]), k
    assert np.array_equal(old_lp.numpy(), base["old_logprobs"]) and np.array_equal(actions, base["actions"])
    stats, order, norms = _run_recorded(train, model, moves, 2048, 4)
    n = len(moves)
    assert len(order) == 4 * n and len(norms) == 8
    for e in range(4):
        assert sorted(order[e * n:(e + 1) * n]) == list(range(n))
    model.eval()
    with torch.no_grad():
        logits, value = model(obs)
    arrays = {f"final::{k}": v.detach().numpy() for k, v in model.state_dict().items()}
    arrays.update(order=np.array(order, np.int16).reshape(4, n), grad_norms=np.array(norms),
                  stat_keys=np.array(sorted(stats)), stat_vals=np.array([float(stats[k]) for k in sorted(stats)]),
                  logits=logits.numpy(), value=value.reshape(-1).numpy(), epochs=np.int64(4),
                  batch_size=np.int64(2048))
    np.savez_compressed(OUT / "update196e4.npz", **arrays)
    print(f"update196e4.npz: h=196, {n} rows, 4 epochs x 2 minibatches; grad norms {norms}; stats {stats}")


def gen_update196(game, train):
    """update196.npz: the reference's model_optimize_step (train.py:414-642) at the README / bench
    policy shape -- GameMLP h 196, 2 residual blocks, dropout 0 -- on 4 096 rows of the golden games
    in TWO minibatches of 2 048, one epoch; Muon (match_rms_adamw) + AdamW at fixed learning rates
    (no scheduler).  The DataLoader's shuffle order is recorded (RandomSampler, wrapped here) and
    stored as `order`, so a test can feed the same two minibatches; the per-minibatch statistics
    come from the reference's own totals (stats) plus the two grad norms (clip_grad_norm_, wrapped
    here).  `python tools/gen_golden.py update196` regenerates only this file."""
    model, boards, obs, invalid, actions, adv, fut, old_lp, moves = _update196_inputs(game)
    n = len(moves)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    lr, clr, wd = 1e-3, 1e-4, 0.01
    stats, order, norms = _run_recorded(train, model, moves, 2048, 1, lr, clr, wd)
    assert sorted(order) == list(range(n)) and len(norms) == 2
    arrays = {f"init::{k}": v.numpy() for k, v in init.items()}
    arrays.update({f"final::{k}": v.detach().numpy() for k, v in model.state_dict().items()})
    arrays.update(boards=boards, actions=actions, invalid=invalid, advantage=adv, future_reward=fut,
                  old_logprobs=old_lp.numpy(), order=np.array(order, np.int64), grad_norms=np.array(norms),
                  stat_keys=np.array(sorted(stats)), stat_vals=np.array([float(stats[k]) for k in sorted(stats)]),
                  hparams=np.array([lr, clr, 0.9, 0.999, wd, 0.02, 0.2]), batch_size=np.int64(2048))
    np.savez_compressed(OUT / "update196.npz", **arrays)
    print(f"update196.npz: h=196, {n} rows in 2 minibatches; grad norms {norms}; stats {stats}")


def gen_urm(game, games):
    torch.manual_seed(77)
    cfg = game.GameURMConfig(hidden_dim=32, num_layers=2, num_heads=4, dropout=0.0, num_loops=4,
                             num_truncated_loops=1)
    model = game.GameURM(cfg).eval()
    boards = games["before"][:64]
    obs = torch.stack([game.Game2048(grid_of(b)).to_model_format() for b in boards])
    with torch.no_grad():
        logits, value = model(obs)
    arrays = {f"w::{k}": v.numpy() for k, v in model.state_dict().items()}
    arrays.update(obs=obs.numpy(), logits=logits.numpy(), value=value.numpy(),
                  config=np.array([32, 2, 4, 4, 1, 2]), expansion=np.float64(cfg.expansion),
                  eps=np.float64(cfg.rms_norm_eps))
    np.savez_compressed(OUT / "urm.npz", **arrays)
    print("urm.npz: h=32 L=2 heads=4 loops=4/1, 64 boards")


def gen_mlp196(game):
    """mlp196.npz: the reference's GameMLP at the bench / README train configuration (h 196, 2
    residual blocks; random init under torch.manual_seed(196), heads left at their Kaiming init so
    the logits are not all zero), eval mode, on 512 boards spread over the golden games."""
    torch.manual_seed(196)
    cfg = game.MLPConfig(hidden_dim=196, num_layers=2)
    model = game.GameMLP(cfg).eval()
    before = np.load(OUT / "games.npz")["before"]
    boards = before[np.linspace(0, len(before) - 1, 512).astype(np.int64)]
    obs = torch.stack([game.Game2048(grid_of(b)).to_model_format() for b in boards])
    with torch.no_grad():
        logits, value = model(obs)
    arrays = {f"w::{k}": v.numpy() for k, v in model.state_dict().items()}
    arrays.update(boards=boards, obs=obs.numpy(), logits=logits.numpy(), value=value.numpy(),
                  hidden_dim=np.int64(196), num_layers=np.int64(2))
    np.savez_compressed(OUT / "mlp196.npz", **arrays)
    print("mlp196.npz: GameMLP h=196 L=2 random init, 512 boards")


def gen_urm64(game):
    """urm64.npz: the reference's GameURM at its DEFAULT config (GameURMConfig(): h 64, 4 heads, 2
    layers, loops 4 / 1 truncated, inter 120 -- BASELINE config 5's policy), eval mode, on 512
    boards spread over the committed golden games (tests/golden/games.npz 'before'): what the
    one-launch forward of the bench's URM leg computes."""
    torch.manual_seed(2048)
    cfg = game.GameURMConfig(dropout=0.0)
    model = game.GameURM(cfg).eval()
    before = np.load(OUT / "games.npz")["before"]
    boards = before[np.linspace(0, len(before) - 1, 512).astype(np.int64)]
    obs = torch.stack([game.Game2048(grid_of(b)).to_model_format() for b in boards])
    with torch.no_grad():
        logits, value = model(obs)
    arrays = {f"w::{k}": v.numpy() for k, v in model.state_dict().items()}
    arrays.update(obs=obs.numpy(), logits=logits.numpy(), value=value.numpy(),
                  config=np.array([cfg.hidden_dim, cfg.num_layers, cfg.num_heads, cfg.num_loops,
                                   cfg.num_truncated_loops, cfg.conv_kernel]),
                  expansion=np.float64(cfg.expansion), eps=np.float64(cfg.rms_norm_eps))
    np.savez_compressed(OUT / "urm64.npz", **arrays)
    print(f"urm64.npz: default GameURMConfig {cfg}, 512 boards")


def main():
    global DIRS
    if sys.argv[1:] in (["urm64"], ["mlp196"]):  # only that fixture (the other files unchanged)
        game, _ = load_reference()
        {"urm64": gen_urm64, "mlp196": gen_mlp196}[sys.argv[1]](game)
        return
    if sys.argv[1:] == ["update196"]:
        game, train = load_reference()
        gen_update196(game, train)
        return
    if sys.argv[1:] == ["update196e4"]:
        game, train = load_reference()
        gen_update196e4(game, train)
        return
    OUT.mkdir(parents=True, exist_ok=True)
    game, train = load_reference()
    DIRS = [game.Direction.UP, game.Direction.DOWN, game.Direction.LEFT, game.Direction.RIGHT]
    gen_rows(game)
    games = gen_games(game)
    gen_best_game(game)
    gen_advantage(train, games)
    gen_mlp(game, games)
    gen_sampler()
    gen_update(game, train, games)
    gen_urm(game, games)
    gen_urm64(game)
    gen_mlp196(game)
    gen_update196(game, train)
    gen_update196e4(game, train)


if __name__ == "__main__":
    main()
