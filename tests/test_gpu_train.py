"""GPU parity of the training path: reward/RTG scan vs calculate_advantage, sampler vs the
reference's masked softmax, seeded whole games vs the reference's spawns, the batched_rollout seam,
graph-vs-eager determinism, and short training runs."""

import math
import random

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    return torch.device("cuda:0")


def _episodes_from_fixture(a):
    eps, cur, last = [], None, None
    for i in range(len(a["episode"])):
        if a["episode"][i] != last:
            cur = {"moves": [], "total_points": 0, "total_steps": 0, "final_state": None}
            eps.append(cur)
            last = a["episode"][i]
        done = bool(a["done"][i])
        cur["moves"].append({"points_earned": int(a["points"][i]), "monotonicity_before": int(a["mono_b"][i]),
                             "monotonicity_after": 0 if done else int(a["mono_a"][i]),
                             "emptiness_before": int(a["empt_b"][i]), "emptiness_after": 0 if done else int(a["empt_a"][i]),
                             "predicted_future_value": float(a["value"][i])})
    return eps


@pytest.mark.parametrize("case", range(5))
def test_calculate_advantage_matches_reference(dev, case):
    import train
    a = golden("advantage.npz")
    gamma, wp, wm, we, beta, m2, mu, step = a["cases"][case]
    eps = _episodes_from_fixture(a)
    eps, aug, fm, nm2, nmu = train.calculate_advantage(eps, gamma, mu, wp, 1, 1, 1, 1, 1, wm, we, 1, 1000.0,
                                                       rtg_beta=beta, rtg_m2=m2, rtg_mu=mu, rtg_step=int(step),
                                                       device=dev)
    moves = [m for ep in eps for m in ep["moves"]]
    got = {k: np.array([m[k] for m in moves]) for k in ("reward", "future_reward_raw", "future_reward", "advantage")}
    # the reward is the scan kernel's device output (float64), bit-identical to the reference's floats
    assert np.array_equal(got["reward"], a[f"c{case}_reward"])
    # G_raw, G-hat and A are computed in float64 and stored fp32: a flat 1e-5 plus the fp32 storage
    # rounding itself (half an ulp, <= 2^-24 relative; cases 1 and 3 normalise to |G-hat| ~ 3e6)
    for key, ref in (("future_reward_raw", "g_raw"), ("future_reward", "g_norm"), ("advantage", "adv")):
        np.testing.assert_allclose(got[key], a[f"c{case}_{ref}"], rtol=2.0 ** -24, atol=1e-5, err_msg=key)
    np.testing.assert_allclose([fm, nm2, nmu], a[f"c{case}_moments"], rtol=1e-9)
    assert aug == []


@pytest.mark.parametrize("T,n", [(96, 4096), (64, 65536)])
def test_rtg_scan_large_time_major_vs_oracle(dev, T, n):
    """[T, N] trajectory with auto-reset episode ends and inactive tails vs the fp64 oracle; the
    second case is BASELINE config 3's full per-GPU shape (65 536 envs x T = 64: 3.1 M live steps)."""
    from g2048 import _lib as L
    g = np.random.default_rng(n)
    points = (g.integers(0, 5, size=(T, n)) * 4).astype(np.int32)
    pot = g.integers(0, 17, size=(T, n, 4)).astype(np.int8)
    flags = np.where(g.random((T, n)) < 0.02, L.FLAG_DONE, 0).astype(np.uint8)
    tail = g.integers(T // 2, T + 1, size=n)
    for e in range(n):
        flags[tail[e]:, e] = L.FLAG_INACTIVE | L.FLAG_DONE
    value = g.normal(size=(T, n)).astype(np.float32)
    gamma, wp, wm, we, beta = 0.97, 0.1, 1.0, 0.5, 0.95
    state0 = [3.0, 40.0, 3.0, 5.0]
    st = torch.tensor(state0 + [0, 1, 0, 0], dtype=torch.float64, device=dev)
    cfg = L.RewardCfg(gamma, wp, wm, we, beta)
    outs = [torch.zeros(T, n, dtype=torch.float32, device=dev) for _ in range(3)]
    part = torch.zeros(3, dtype=torch.float64, device=dev)
    ws = torch.zeros(L.rtg_workspace_bytes(n), dtype=torch.uint8, device=dev)
    td = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    L.rtg_prepare(st, cfg)
    L.reward_rtg(td(points), td(pot), td(flags), td(value), st, *outs, part, ws, cfg)
    L.rtg_finalize(st, part, cfg)
    gr, gn, ad = (o.cpu().numpy() for o in outs)
    # oracle: per env episodes in time order
    exp_gr = np.zeros((T, n))
    # episode order: env-major, time ascending, the live prefix t < tail[e] of each env
    ee = np.repeat(np.arange(n), tail)
    tt = np.arange(len(ee)) - np.repeat(np.cumsum(tail) - tail, tail)
    sel = (tt, ee)
    ends = ((flags[sel] & L.FLAG_DONE) != 0) | (tt == tail[ee] - 1)
    r = O.reward_rtg_normalize(points[sel], pot[sel][:, 0], pot[sel][:, 1], pot[sel][:, 2], pot[sel][:, 3],
                               (flags[sel] & L.FLAG_DONE) != 0, value[sel], ends, gamma, wp, wm, we, beta,
                               state0[1], state0[0], int(state0[3]), state0[2])
    np.testing.assert_allclose(gr[sel], r["g_raw"], rtol=1e-6, atol=1e-4)
    np.testing.assert_allclose(gn[sel], r["g_norm"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ad[sel], r["adv"], rtol=1e-5, atol=1e-5)
    s = st.cpu().numpy()
    np.testing.assert_allclose([s[0], s[1], s[2]], r["moments"], rtol=1e-9)
    assert s[3] == state0[3] + 1
    assert (gr[flags == (L.FLAG_INACTIVE | L.FLAG_DONE)] == 0).all()


def test_sampler_matches_reference_masked_softmax(dev):
    from g2048 import _lib as L
    g = golden("sampler.npz")
    n = len(g["logits"])
    legal = np.array([sum(1 << a for a in range(4) if not g["invalid"][i, a]) for i in range(n)], np.uint8)
    lg = torch.from_numpy(g["logits"]).to(dev)
    fl = torch.from_numpy(legal).to(dev)
    act = torch.zeros(n, dtype=torch.uint8, device=dev)
    lp = torch.zeros(n, 4, dtype=torch.float32, device=dev)
    ent = torch.zeros(n, dtype=torch.float32, device=dev)
    L.sample_actions(lg, fl, act, lp, ent, L.make_rng(L.RNG_PHILOX, 77, 12, 5))
    torch.cuda.synchronize()
    lpn, en, an = lp.cpu().numpy(), ent.cpu().numpy(), act.cpu().numpy()
    fin = np.isfinite(g["logp"])
    assert np.array_equal(np.isfinite(lpn), fin)
    np.testing.assert_allclose(lpn[fin], g["logp"][fin], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(en, g["entropy"], rtol=1e-5, atol=1e-5)
    # inverse CDF of the same Philox uniform (stream 1), away from CDF boundaries
    u = (O.philox_draws(77, 12, n, 1, env_base=5)[:, 0] >> 8).astype(np.float64) / 2**24
    cdf = np.cumsum(np.where(g["invalid"], 0.0, g["probs"]), axis=1)
    expect = np.array([int(np.argmax(u[i] < cdf[i])) for i in range(n)])
    near = np.abs(cdf - u[:, None]).min(axis=1) < 1e-5
    assert np.array_equal(an[~near], expect[~near])
    assert all(legal[i] >> an[i] & 1 for i in range(n))


def test_sampler_distribution(dev):
    from g2048 import _lib as L
    n = 1 << 20
    logits = torch.tensor([[0.0, 1.0, -1.0, 2.0]], device=dev).repeat(n, 1)
    fl = torch.full((n,), 0b1011, dtype=torch.uint8, device=dev)  # LEFT illegal
    act = torch.zeros(n, dtype=torch.uint8, device=dev)
    L.sample_actions(logits, fl, act, None, None, L.make_rng(L.RNG_PHILOX, 1, 0))
    freq = torch.bincount(act.long(), minlength=4).double().cpu().numpy() / n
    p = np.exp([0.0, 1.0, -np.inf, 2.0])
    p /= p.sum()
    assert freq[2] == 0
    assert np.abs(freq - p).max() < 3e-3


def test_seeded_game_matches_reference_spawns(dev):
    """play_game_for_episode(seed=s): replaying its actions through the pure-Python restatement
    after random.seed(s) reproduces every board (game.py spawns, bit-exact)."""
    import agent
    import train
    from oracle import pyref
    torch.manual_seed(0)
    model = agent.GameMLP(agent.MLPConfig(hidden_dim=32)).to(dev).eval()
    for s in (0, 1, 2):
        ep = train.play_game_for_episode(model, device=dev, seed=s)
        rnd = random.Random(s)
        b = pyref.reset(rnd)
        for m in ep["moves"]:
            assert [c for row in m["state_before"] for c in row] == b
            pts, done, info = pyref.step(b, m["selected_direction"], rnd)
            assert pts == m["points_earned"]
            assert [c for row in m["result_state"] for c in row] == b
            assert m["monotonicity_before"] == info["monotonicity_before"]
            assert m["emptiness_before"] == info["emptiness_before"]
        assert done and ep["total_steps"] == len(ep["moves"]) - 1
        assert ep["final_state"] == [b[0:4], b[4:8], b[8:12], b[12:16]]


def test_play_games_batched_schema(dev):
    import agent
    from batched_rollout import play_games_batched
    torch.manual_seed(1)
    model = agent.GameMLP(agent.MLPConfig(hidden_dim=32)).to(dev)
    random.seed(4)
    eps = play_games_batched(model, 64, max_steps=None, device=dev)
    assert len(eps) == 64
    keys = {"predicted_future_value", "selected_direction", "game_state", "state_before", "result_state",
            "points_earned", "action_mask", "policy_logprobs", "monotonicity_before", "monotonicity_after",
            "emptiness_before", "emptiness_after", "entropy", "max_tile_created", "points_possible"}
    for ep in eps:
        assert ep["moves"] and keys <= set(ep["moves"][0])
        assert ep["total_points"] == sum(m["points_earned"] for m in ep["moves"])
        assert O.legal_mask(np.array(ep["final_state"], np.int8).reshape(1, 16))[0] == 0
        m = ep["moves"][-1]
        assert m["monotonicity_after"] == 0.0 and m["emptiness_after"] == 0.0
        for m in ep["moves"][:5]:
            assert isinstance(m["predicted_future_value"], float) and m["game_state"].shape == (48,)
            assert not m["action_mask"][m["selected_direction"]]
            assert m["points_possible"][agent.Direction.UP] >= 0
    random.seed(4)
    again = play_games_batched(model, 64, max_steps=None, device=dev)
    assert [e["total_points"] for e in again] == [e["total_points"] for e in eps]
    capped = play_games_batched(model, 8, max_steps=7, device=dev)
    assert all(len(e["moves"]) <= 7 for e in capped)


def test_graph_and_eager_rollouts_identical(dev):
    import agent
    from g2048.rollout import InferencePolicy, Rollout
    torch.manual_seed(2)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=64)).to(dev)
    pol = InferencePolicy(m)
    outs = []
    for graph in (False, True, True):
        ro = Rollout(2048, 24, dev, seed=9)
        ro.reset()
        ro.collect(pol, graph=graph)
        outs.append((ro.buf.boards.clone(), ro.buf.actions.clone(), ro.buf.points.clone()))
    for o in outs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(outs[0], o))


@pytest.mark.parametrize("horizon,ratio,hidden", [(32, 0.0, 64), (0, 0.0, 64), (32, 0.25, 196), (0, 0.25, 64)])
def test_trainer_runs_and_learns_signal(dev, horizon, ratio, hidden):
    """Fixed-horizon and episodic training steps, with and without the device D4 up-sampling
    (--upsample-ratio: about ratio x samples copies; the ragged last minibatch runs padded)."""
    from g2048.trainer import TrainConfig, VecTrainer
    cfg = TrainConfig(steps=6, episodes=1024, horizon=horizon, max_steps=256 if horizon == 0 else None,
                      batch_size=8192, hidden=hidden, points=0.1, mono=1.0, rtg_beta=0.99, entropy=0.02, critic=0.2,
                      warmup_steps=1, lr=1e-3, critic_lr=1e-4, upsample_ratio=ratio)
    tr = VecTrainer(cfg, dev)
    ms = [tr.train_step(s) for s in range(4)]
    for m in ms:
        k = int(m["samples"] * ratio)
        assert (m["augmented_samples"] == 0) if ratio == 0 else abs(m["augmented_samples"] - k) < 6 * k ** 0.5 + 2
    for m in ms:
        for k, v in m.items():
            assert v is None or not isinstance(v, float) or math.isfinite(v), k
    assert ms[-1]["samples"] > 0 and ms[-1]["episodes_finished"] > 0
    assert ms[1]["grad_norm"] > 0
    assert 0 < ms[0]["entropy"] <= math.log(4) + 1e-5
    mom = tr.rtg.moments()
    assert mom["rtg_step"] == 5
    ev = tr.evaluate(16, 200)
    assert ev["eval/max_score"] >= ev["eval/avg_score"] > 0


def test_trainer_full_config3_shape(dev):
    """BASELINE config 3 at its full per-GPU shape (65 536 envs, h = 196, T = 64, minibatch 65 536,
    up-sampling 0.25, graphs on): two train steps run, every metric finite, the update moves the
    weights, the sample count is envs x T, and the augmented count is 0.25 x samples within 6 sigma."""
    from g2048.trainer import TrainConfig, VecTrainer
    cfg = TrainConfig(steps=4, episodes=65536, horizon=64, batch_size=65536, hidden=196, points=0.1, mono=1.0,
                      rtg_beta=0.99, entropy=0.02, critic=0.2, warmup_steps=1, lr=1e-3, critic_lr=1e-4,
                      upsample_ratio=0.25)
    tr = VecTrainer(cfg, dev)
    before = [p.detach().clone() for p in tr.model.parameters()]
    ms = [tr.train_step(s) for s in range(2)]
    for m in ms:
        for k, v in m.items():
            assert v is None or not isinstance(v, float) or math.isfinite(v), k
        assert m["samples"] == 65536 * 64
        k = int(m["samples"] * 0.25)
        assert abs(m["augmented_samples"] - k) < 6 * k ** 0.5 + 2
        assert m["grad_norm"] > 0 and 0 < m["entropy"] <= math.log(4) + 1e-5
    moved = sum(float((p.detach() - q).abs().max()) > 0 for p, q in zip(tr.model.parameters(), before))
    assert moved == len(before)


def test_episodic_trainer_respects_max_steps(dev):
    """--max-steps 100 (not a multiple of the 32-step graph chunk): no game plays or trains on more
    than 100 moves (train.py:240 `step < max_steps`), and the cap binds for a random policy."""
    from g2048 import _lib as L
    from g2048.trainer import TrainConfig, VecTrainer
    cfg = TrainConfig(steps=4, episodes=512, horizon=0, max_steps=100, batch_size=4096, hidden=32, points=0.1,
                      mono=1.0, rtg_beta=0.99, entropy=0.02, critic=0.2, warmup_steps=1)
    tr = VecTrainer(cfg, dev)
    m = tr.train_step(0)
    assert 0 < m["samples"] <= 512 * 100
    for graph in (True, False):
        tr.cfg.graph = graph
        T = tr._collect_episodic()
        assert T <= 100
        sf = tr.rollout.buf.step_flags[:T]
        moves = ((sf & L.FLAG_INACTIVE) == 0).sum(0)
        assert int(moves.max()) == 100  # some random games outlast the cap
    m = tr.train_step(1)
    assert m["samples"] <= 512 * 100


def _update_once(dev, u, mode: str, order_seed: int):
    """One PPO update of GameMLP(h 64, fp32, dropout 0) from torch seed 1234 on the golden update
    data (train.py:414-642): `tensor` = PPOUpdater on device tensors (rows in the device
    permutation's order), `compat` = the list-of-dict model_optimize_step (rows in randperm's order).
    `order_seed` seeds the row order only.  Returns (flat parameters, {name: tensor}, stats)."""
    import agent
    import train
    from g2048 import _lib as L
    from g2048.dist import GradBucket
    from g2048.optim import build_optimizer
    from g2048.ppo import PPOConfig, PPOUpdater
    n = len(u["actions"])
    torch.manual_seed(1234)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=64, num_layers=2, dropout=0.0)).to(dev)
    opt = build_optimizer(m, 1e-3, 1e-4, schedule=False)
    torch.manual_seed(order_seed)
    if mode == "tensor":
        legal = np.array([sum(1 << a for a in range(4) if not u["invalid"][i, a]) for i in range(n)], np.uint8)
        boards = np.rint(u["obs"][:, 0::3]).astype(np.int8)
        up = PPOUpdater(m, opt, PPOConfig(batch_size=n, critic=0.2, amp_dtype=None), GradBucket(m.parameters()))

        def enc(b):
            o = torch.empty(b.shape[0], 48, dtype=torch.float32, device=dev)
            L.obs_encode(b.contiguous(), o)
            return o
        data = {"boards": torch.from_numpy(boards).to(dev), "actions": torch.from_numpy(u["actions"]).to(dev),
                "legal": torch.from_numpy(legal).to(dev), "logp": torch.from_numpy(u["old_logprobs"]).to(dev),
                "adv": torch.from_numpy(u["advantage"]).to(dev), "ret": torch.from_numpy(u["future_reward"]).to(dev)}
        st = {k: float(v) for k, v in up.update(data, 0.02, enc).items()}
    else:
        moves = [{"game_state": torch.from_numpy(u["obs"][i]), "selected_direction": int(u["actions"][i]),
                  "action_mask": u["invalid"][i].tolist(), "advantage": float(u["advantage"][i]),
                  "future_reward": float(u["future_reward"][i]), "policy_logprobs": u["old_logprobs"][i].tolist()}
                 for i in range(n)]
        st = train.model_optimize_step(m, [{"moves": moves}], opt, None, 0.02, 0.2, dev, n, 1)
    named = {k: v.detach().reshape(-1).cpu().numpy().copy() for k, v in m.named_parameters()}
    return np.concatenate(list(named.values())), named, st


def test_ppo_updater_gpu_matches_compat_update(dev):
    """Tensor-path PPOUpdater (fp32, one minibatch) == list-of-dict model_optimize_step on the same data.

    Where the bound comes from (round-5 analysis of the round-4 flake, 21 of 11 973 parameters off by
    <= 9.4e-6 under a fixed atol of 2e-6): the two paths see the n rows in different orders, so their
    fp32 gradient sums differ in the last bits, and torch.optim.Muon's bf16 Newton-Schulz turns that
    into bf16-rounding-sized differences of the update (lr 1e-3: ~1e-6..1e-5 absolute).  The test
    measures both facts instead of assuming a number:
      1. each path, run twice from the same seeds in this process, is BITWISE reproducible (no
         non-deterministic kernel on either side: a flake cannot come from run-to-run noise);
      2. the order noise floor: compat runs of 4 other row orders; per parameter tensor, the
         tensor-vs-compat difference must stay within 2x the largest difference between those runs
         (+ 1e-7 absolute for tensors the order does not move)."""
    u = golden("update.npz")
    t1, tn, ts = _update_once(dev, u, "tensor", 1234)
    t2, _, _ = _update_once(dev, u, "tensor", 1234)
    c1, cn, cs = _update_once(dev, u, "compat", 1234)
    c2, _, _ = _update_once(dev, u, "compat", 1234)
    det = {"tensor": bool(np.array_equal(t1, t2)), "compat": bool(np.array_equal(c1, c2))}
    orders = [_update_once(dev, u, "compat", 1000 + k)[1] for k in range(4)]
    report = {}
    for name, tv in tn.items():
        spread = max(float(np.abs(a[name] - b[name]).max()) for i, a in enumerate(orders) for b in orders[i + 1:])
        diff = float(np.abs(tv - cn[name]).max())
        report[name] = (diff, spread)
    print("determinism", det, "| per tensor (tensor-vs-compat max diff, order spread):",
          {k: (f"{d:.2e}", f"{s:.2e}") for k, (d, s) in report.items()})
    assert det["tensor"], "PPOUpdater's tensor path is not run-to-run deterministic on this device"
    assert det["compat"], "model_optimize_step is not run-to-run deterministic on this device"
    for name, (diff, spread) in report.items():
        assert diff <= 2.0 * spread + 1e-7, (name, diff, spread)
    for k in ("loss", "policy_loss", "value_loss", "entropy", "grad_norm"):
        assert math.isclose(ts[k], cs[k], rel_tol=1e-4, abs_tol=1e-6), k


def test_graphed_update_equals_eager_update(dev):
    """The hipGraph-captured PPO minibatch step (graph-safe Muon+AdamW) == the same step run eagerly."""
    import agent
    from g2048 import _lib as L
    from g2048.dist import GradBucket
    from g2048.optim import MuonAdamW
    from g2048.ppo import PPOConfig, PPOUpdater
    g = np.random.default_rng(0)
    M = 8192
    boards = g.integers(0, 10, size=(M, 16)).astype(np.int8)
    legal = O.legal_mask(boards)
    legal[legal == 0] = 1
    acts = np.array([[a for a in range(4) if m >> a & 1][0] for m in legal], np.uint8)
    data = {"boards": torch.from_numpy(boards).to(dev), "actions": torch.from_numpy(acts).to(dev),
            "legal": torch.from_numpy(legal).to(dev),
            "logp": torch.from_numpy(np.log(np.full((M, 4), 0.25, np.float32))).to(dev),
            "adv": torch.from_numpy(g.normal(size=M).astype(np.float32)).to(dev),
            "ret": torch.from_numpy(g.normal(size=M).astype(np.float32)).to(dev)}

    def enc(b):
        o = torch.empty(b.shape[0], 48, dtype=torch.float32, device=dev)
        L.obs_encode(b.contiguous(), o)
        return o
    out = []
    for graph in (False, True):
        torch.manual_seed(3)
        m = agent.GameMLP(agent.MLPConfig(hidden_dim=64, num_layers=2, dropout=0.0)).to(dev)
        opt = MuonAdamW(m, 1e-3, 1e-4)
        order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
        gen = torch.Generator(device=dev)
        gen.manual_seed(5)
        up = PPOUpdater(m, opt, PPOConfig(batch_size=2048, critic=0.2), GradBucket(order), gen, graph=graph)
        st = None
        for _ in range(3):
            st = {k: float(v) for k, v in up.update(data, 0.02, enc).items()}
        out.append((torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy(), st))
    np.testing.assert_allclose(out[0][0], out[1][0], rtol=1e-5, atol=1e-6)
    for k in ("loss", "entropy", "grad_norm", "kl_average"):
        assert math.isclose(out[0][1][k], out[1][1][k], rel_tol=1e-4, abs_tol=1e-6), k


def test_episode_scan_matches_loop(dev):
    """g2048_episode_scan == the per-step torch loop it replaced (scores / max tiles of finished games,
    running state carried across two rollouts)."""
    from g2048 import _lib as L
    g = np.random.default_rng(3)
    T, n = 40, 3000
    pts = torch.from_numpy(g.integers(0, 64, size=(T, n)).astype(np.int32)).to(dev)
    boards = torch.from_numpy(g.integers(0, 12, size=(T, n, 16)).astype(np.int8)).to(dev)
    mt = torch.from_numpy(g.integers(0, 13, size=(T, n)).astype(np.int8)).to(dev)
    fl = torch.from_numpy(np.where(g.random((T, n)) < 0.05, 0x80, 0).astype(np.uint8)
                          | np.where(g.random((T, n)) < 0.02, 0x40, 0).astype(np.uint8)).to(dev)
    rs = torch.zeros(n, dtype=torch.int64, device=dev)
    rm = torch.zeros(n, dtype=torch.int32, device=dev)
    rs2, rm2 = rs.clone(), rm.clone()
    for _ in range(2):
        sc = torch.empty(T, n, dtype=torch.int64, device=dev)
        ti = torch.empty(T, n, dtype=torch.int32, device=dev)
        L.episode_scan(pts, boards, mt, fl, rs, rm, sc, ti)
        done = ((fl & 0x80) != 0) & ((fl & 0x40) == 0)
        for t in range(T):
            rs2 += pts[t]
            rm2 = torch.maximum(rm2, torch.maximum(boards[t].max(dim=1).values.to(torch.int32), mt[t].to(torch.int32)))
            d = done[t]
            assert torch.equal(sc[t], torch.where(d, rs2, -1))
            assert torch.equal(ti[t], torch.where(d, rm2, -1))
            rs2 = torch.where(d, 0, rs2)
            rm2 = torch.where(d, 0, rm2)
        assert torch.equal(rs, rs2) and torch.equal(rm, rm2)


def _rollout_stats_torch(pts, pot, sf, value, g_raw, g_norm, adv, boards, mt, episodic, w, rs, rm):
    """The train step's rollout metrics as the torch expression the trainer used before
    g2048_rollout_stats (float32 reductions; the same 23 entries).  rs / rm: carried state (fixed
    horizon), advanced in place."""
    T, n = pts.shape
    done = ((sf & 0x80) != 0).float()
    p = pot.float()
    r = (pts.float() * w.points + w.mono * (w.gamma * p[..., 1] * (1 - done) - p[..., 0])
         + w.emptiness * (w.gamma * p[..., 3] * (1 - done) - p[..., 2]))
    fields = [r, adv, g_norm, g_raw, value]
    if episodic:
        valid = torch.nonzero(((sf & 0x40) == 0).reshape(-1)).squeeze(1)
        fields = [f.reshape(-1).index_select(0, valid) for f in fields]
    else:
        fields = [f.reshape(-1) for f in fields]
    r, a, gn, gr, v = fields
    starts = torch.zeros_like(sf, dtype=torch.bool)
    if episodic:
        starts[0] = True
    else:
        starts[1:] = (sf[:-1] & 0x20) != 0
    g0 = (g_raw * starts).sum() / starts.sum().clamp(min=1)
    if episodic:
        scores = torch.where((sf & 0x40) == 0, pts, 0).sum(0)
        tiles = boards[T].max(dim=1).values.to(torch.int32)
        fin = torch.ones_like(scores, dtype=torch.bool)
    else:
        sc = torch.empty(T, n, dtype=torch.int64, device=pts.device)
        ti = torch.empty(T, n, dtype=torch.int32, device=pts.device)
        from g2048 import _lib as L
        L.episode_scan(pts, boards, mt, sf, rs, rm, sc, ti)
        scores, tiles, fin = sc, ti, sc >= 0
    s_flat = torch.where(fin, scores, -1).reshape(-1).to(torch.int32)
    cnt = fin.sum()
    cntf = cnt.float().clamp(min=1.0)
    srt = torch.sort(s_flat).values
    med_idx = (s_flat.numel() - cnt + (cnt - 1).clamp(min=0) // 2).clamp(max=s_flat.numel() - 1)
    return torch.stack([
        torch.tensor(float(r.numel()), device=pts.device), r.mean(), r.var(unbiased=False),
        (r == 0).float().mean() * 100, a.mean(), a.var(unbiased=False), a.pow(2).sum().sqrt(), a.min(), a.max(),
        gn.mean(), gn.std(unbiased=False), gn.min(), gn.max(), gr.std(unbiased=False), v.std(unbiased=False), g0,
        torch.where(fin, scores, 0).sum().float() / cntf, srt[med_idx].float(), s_flat.max().float(),
        (fin & (tiles >= 9)).sum().float() / cntf * 100, (fin & (tiles >= 10)).sum().float() / cntf * 100,
        (fin & (tiles >= 11)).sum().float() / cntf * 100, cnt.float()]).double().cpu().numpy()


@pytest.mark.parametrize("episodic,T,n,p_done", [(False, 64, 5000, 0.03), (False, 7, 300, 0.0), (False, 33, 1000, 0.4),
                                                 (True, 50, 2000, 0.02)])
def test_rollout_stats_kernel_matches_torch(dev, episodic, T, n, p_done):
    """g2048_rollout_stats (two launches) vs the torch expression it replaced: counts, the integer
    score statistics (median by radix select, max, finished mean) and the tile percentages exactly,
    every float moment within 1e-5 relative (the kernel sums in float64, torch in float32); the
    carried running score / max tile equal episode_scan's over three consecutive rollouts; the
    workspace's key counter is left zeroed.  Edge cases: no finished game (median / max -1), many finished games,
    episodic inactive tails."""
    from g2048 import _lib as L
    from g2048.advantage import RewardWeights
    g = np.random.default_rng(T * 7 + n)
    w = RewardWeights(gamma=0.99, points=0.1, mono=1.0, emptiness=0.5, rtg_beta=0.9)
    rs = torch.randint(0, 5000, (n,), dtype=torch.int64, device=dev)
    rm = torch.randint(0, 9, (n,), dtype=torch.int32, device=dev)
    rs_ref, rm_ref = rs.clone(), rm.clone()
    ws = torch.zeros(L.rollout_stats_workspace_bytes(T, n), dtype=torch.uint8, device=dev)
    out = torch.empty(L.ROLLOUT_STATS, dtype=torch.float32, device=dev)
    for it in range(3):
        pts = torch.from_numpy(np.where(g.random((T, n)) < 0.3, 0, g.integers(0, 2048, size=(T, n))).astype(np.int32)).to(dev)
        pot = g.integers(-20, 60, size=(T, n, 4)) * (g.random((T, n, 1)) >= 0.3)  # zero rewards where pts = 0 too
        pot = torch.from_numpy(pot.astype(np.int8)).to(dev)
        fl = np.where(g.random((T, n)) < p_done, 0x80, 0) | np.where(g.random((T, n)) < 0.1, 0x20, 0)
        if episodic:  # games end at a random step; the rest of the column is inactive
            end = g.integers(1, T + 1, size=n)
            tt = np.arange(T)[:, None]
            fl = np.where(tt == end - 1, 0x80, 0) | np.where(tt >= end, 0x40, 0)
        sf = torch.from_numpy(fl.astype(np.uint8)).to(dev)
        value, g_raw, g_norm, adv = (torch.from_numpy((g.standard_normal((T, n)) * s).astype(np.float32)).to(dev)
                                     for s in (1.0, 30.0, 1.0, 1.5))
        boards = torch.from_numpy(g.integers(0, 12, size=(T + 1, n, 16)).astype(np.int8)).to(dev)
        mt = torch.from_numpy(g.integers(0, 13, size=(T, n)).astype(np.int8)).to(dev)
        bview = boards if episodic else boards[:T]
        if episodic:
            L.rollout_stats(pts, pot, sf, value, g_raw, g_norm, adv, bview, None, True, w.cfg(), None, None, ws, out)
        else:
            L.rollout_stats(pts, pot, sf, value, g_raw, g_norm, adv, bview, mt, False, w.cfg(), rs, rm, ws, out)
        ref = _rollout_stats_torch(pts, pot, sf, value, g_raw, g_norm, adv, bview, mt, episodic, w, rs_ref, rm_ref)
        got = out.double().cpu().numpy()
        exact = [0, 17, 18, 22]  # rows, median, max, finished count
        np.testing.assert_array_equal(got[exact], ref[exact], err_msg=f"rollout {it}")
        np.testing.assert_allclose(got[19:22], ref[19:22], rtol=1e-6, atol=1e-4, err_msg=f"tile % rollout {it}")
        scale = np.maximum(np.abs(ref), 1.0)
        np.testing.assert_array_less(np.abs(got - ref) / scale, 1e-5, err_msg=f"moments rollout {it}")
        if not episodic:
            assert torch.equal(rs, rs_ref) and torch.equal(rm, rm_ref)
        if p_done == 0.0 and not episodic:
            assert got[17] == -1 and got[18] == -1 and got[22] == 0
        assert int(ws[:4].view(torch.int32)[0]) == 0  # the key counter is left zeroed


@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 5_243_197])
def test_permutation_kernel_is_a_keyed_permutation(dev, n):
    """g2048_permutation (the update's epoch order, replacing torch.randperm): every index exactly
    once (the bench's 5.24 M-sample epoch included), the same key gives the same order, the device
    key equals the host seed, and another key another order."""
    from g2048 import _lib as L
    out = torch.empty(n + 5, dtype=torch.int64, device=dev).fill_(-7)
    key = torch.tensor([123456789], dtype=torch.int64, device=dev)
    L.permutation(out, n, key)
    p = out[:n].clone()
    assert torch.equal(torch.sort(p).values, torch.arange(n, device=dev))
    assert (out[n:] == -7).all()
    L.permutation(out, n, None, seed=123456789)
    assert torch.equal(out[:n], p)
    if n >= 17:
        L.permutation(out, n, None, seed=987654321)
        assert not torch.equal(out[:n], p)


def test_permutation_positions_are_uniform(dev):
    """Where index 0 lands over 2000 keys of a 16-element permutation: every position 125 +- 55 times
    (a 5-sigma band of the binomial), like torch.randperm's."""
    from g2048 import _lib as L
    out = torch.empty(16, dtype=torch.int64, device=dev)
    pos = torch.empty(2000, dtype=torch.int64, device=dev)
    for s in range(2000):
        L.permutation(out, 16, None, seed=s, counter=3)
        pos[s] = torch.nonzero(out == 0)[0, 0]
    counts = torch.bincount(pos, minlength=16).cpu().numpy()
    assert counts.min() >= 70 and counts.max() <= 180, counts


@pytest.mark.parametrize("n,k", [(3000, 750), (257, 256), (1000, 0)])
def test_augment_kernel_matches_oracle(dev, n, k):
    """g2048_augment (D4 up-sampling, train.py:774-881) vs oracle.augment_plan + augment_rows: the
    same source rows and transforms in the same order, bit-exact copies; real rows untouched."""
    from g2048 import _lib as L
    g = np.random.default_rng(n + k)
    cap = n + 2 * k
    boards = np.zeros((cap, 16), np.int8)
    boards[:n] = g.integers(0, 12, size=(n, 16))
    actions = np.zeros(cap, np.uint8)
    actions[:n] = g.integers(0, 4, size=n)
    legal = np.zeros(cap, np.uint8)
    legal[:n] = g.integers(0, 256, size=n)
    logp = np.zeros((cap, 4), np.float32)
    logp[:n] = g.normal(size=(n, 4))
    adv = np.zeros(cap, np.float32)
    adv[:n] = g.normal(size=n)
    ret = np.zeros(cap, np.float32)
    ret[:n] = g.normal(size=n)
    t = [torch.from_numpy(a.copy()).to(dev) for a in (boards, actions, legal, logp, adv, ret)]
    ws = torch.zeros(L.augment_workspace_bytes(k), dtype=torch.uint8, device=dev)
    count = torch.zeros(1, dtype=torch.int64, device=dev)
    seed, counter = 0x5EED + k, 11
    L.augment(*t, n, k, seed, counter, ws, count)
    torch.cuda.synchronize()
    plan = O.augment_plan(n, k, seed, counter)
    want = O.augment_rows(boards, actions, legal, logp, adv, ret, plan)
    c = int(count.item())
    assert c == n + len(want[0])
    got = [x.cpu().numpy() for x in t]
    for a, w, full in zip(got, want, (boards, actions, legal, logp, adv, ret)):
        assert np.array_equal(a[:n], full[:n])
        assert np.array_equal(a[n:c], w)


@pytest.mark.parametrize("hidden,layers,want", [(196, 2, []), (196, 3, ["rollout"]),
                                                (256, 2, ["rollout", "update forward", "optimizer"])])
def test_trainer_reports_kernel_fallbacks(dev, hidden, layers, want):
    """A GameMLP shape outside a fused kernel's cover (-l 3: no fused rollout; -h 256: no MFMA layer
    kernel, no one-block Newton-Schulz) is reported (warning + VecTrainer.fallbacks, printed by the
    CLI), never silent; the README model (h 196, 2 blocks) runs every fused path."""
    import warnings
    from g2048.trainer import TrainConfig, VecTrainer
    cfg = TrainConfig(steps=2, episodes=64, horizon=8, batch_size=256, hidden=hidden, num_layers=layers,
                      warmup_steps=0)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        tr = VecTrainer(cfg, dev)
    got = [m.split(":")[0] for m in tr.fallbacks]
    assert got == want, tr.fallbacks
    assert len([x for x in w if "g2048:" in str(x.message)]) == len(want)
    if not want:
        assert tr.paths["rollout"] == "policy_rollout_kernel" and tr.paths["update"] == "FusedPPOUpdater"
    m = tr.train_step(0)
    assert math.isfinite(m["loss"])
    # after the first update the labels are the updater's own decision (FusedPPOUpdater._alloc)
    after = [x.split(":")[0] for x in tr.fallbacks]
    if not want:
        assert tr.paths["update_forward"] == "fused train / KL passes + fused backward" and after == []
    else:
        assert "predicted" not in tr.paths["update_forward"]
        assert ("update" in after) == (layers != 2 or hidden == 256), tr.fallbacks
