"""Host-side logic on CPU: the PPO update against the reference's golden update step, the LR
schedule, D4 augmentation, and the flat gradient bucket."""

import math
import random

import numpy as np
import pytest
import torch

from conftest import golden


# bounds of the eight-step CPU pin (test_model_optimize_step_matches_reference_four_epochs_h196): its
# first run here reproduced the reference bit for bit (every move cosine 1.000000, final logits and
# values identical: the same torch CPU kernels in the same order); the bounds leave room for another
# CPU's thread count / vector width changing a reduction order
COS_E4_CPU = 0.9999
LOGIT_E4_CPU = 1e-4


def _golden_model():
    import agent
    u = golden("update.npz")
    torch.manual_seed(1234)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=64, num_layers=2, dropout=0.0))
    return m, u


def _moves(u):
    return [{"game_state": torch.from_numpy(u["obs"][i]), "selected_direction": int(u["actions"][i]),
             "action_mask": u["invalid"][i].tolist(), "advantage": float(u["advantage"][i]),
             "future_reward": float(u["future_reward"][i]), "policy_logprobs": u["old_logprobs"][i].tolist()}
            for i in range(len(u["actions"]))]


def test_model_optimize_step_matches_reference_update():
    """train.py:414-642 with Muon+AdamW at fixed lr, one minibatch: parameters after the step and the
    returned statistics agree with the reference run (tests/golden/update.npz)."""
    import train
    from g2048.optim import MultiOptimizer
    m, u = _golden_model()
    lr, clr, b1, b2, wd, beta, critic = u["hparams"]
    o2d, o1d, v2d, v1d = m.get_param_groups(clr, lr)
    adamw = torch.optim.AdamW([o1d, v1d], betas=(b1, b2), weight_decay=wd)
    muon = torch.optim.Muon([o2d, v2d], adjust_lr_fn="match_rms_adamw", weight_decay=wd)
    stats = train.model_optimize_step(m, [{"moves": _moves(u)}], MultiOptimizer(muon, adamw), None, beta, critic,
                                      None, batch_size=len(u["actions"]), epochs=1)
    for k, v in m.state_dict().items():
        np.testing.assert_allclose(v.numpy(), u[f"final::{k}"], rtol=1e-4, atol=2e-6, err_msg=k)
    ref = dict(zip(u["stat_keys"].tolist(), u["stat_vals"].tolist()))
    for k in ("loss", "policy_loss", "entropy_loss", "value_loss", "grad_norm", "entropy"):
        assert math.isclose(stats[k], ref[k], rel_tol=1e-4, abs_tol=1e-6), (k, stats[k], ref[k])
    assert stats["lr"] == ref["lr"] == 0.0


def test_model_optimize_step_matches_reference_update_h196(monkeypatch):
    """The same at the README / bench policy shape (tests/golden/update196.npz: h 196, 4 096 rows in the
    reference's two shuffled minibatches of 2 048, clip active): with the DataLoader's recorded order,
    the CPU restatement's parameters and statistics match the reference run (fp32; Muon's bf16
    Newton-Schulz is torch's own here, so only the reduction order of the two runs differs)."""
    import agent
    import train
    from g2048.augment import encode_grid
    from g2048.optim import MultiOptimizer
    u = golden("update196.npz")
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=196, num_layers=2, dropout=0.0))
    m.load_state_dict({k[len("init::"):]: torch.from_numpy(u[k]) for k in u.files if k.startswith("init::")})
    lr, clr, b1, b2, wd, beta, critic = (float(x) for x in u["hparams"])
    moves = [{"game_state": encode_grid(u["boards"][i].reshape(4, 4).tolist()), "selected_direction": int(u["actions"][i]),
              "action_mask": u["invalid"][i].tolist(), "advantage": float(u["advantage"][i]),
              "future_reward": float(u["future_reward"][i]), "policy_logprobs": u["old_logprobs"][i].tolist()}
             for i in range(len(u["actions"]))]
    order = torch.from_numpy(u["order"])
    real_randperm = torch.randperm
    monkeypatch.setattr(torch, "randperm", lambda n, *a, **k: order.clone() if n == len(order) else real_randperm(n, *a, **k))
    o2d, o1d, v2d, v1d = m.get_param_groups(clr, lr)
    adamw = torch.optim.AdamW([o1d, v1d], betas=(b1, b2), weight_decay=wd)
    muon = torch.optim.Muon([o2d, v2d], adjust_lr_fn="match_rms_adamw", weight_decay=wd)
    stats = train.model_optimize_step(m, [{"moves": moves}], MultiOptimizer(muon, adamw), None, beta, critic,
                                      None, batch_size=int(u["batch_size"]), epochs=1)
    for k, v in m.state_dict().items():
        want = u[f"final::{k}"] - u[f"init::{k}"]
        got = v.numpy() - u[f"init::{k}"]
        cos = float(np.dot(got.ravel(), want.ravel()) / (np.linalg.norm(got) * np.linalg.norm(want) + 1e-30))
        assert cos > 0.9995, (k, cos)  # the two fp32 runs differ by summation order only (measured >= 0.9997 on device)
        np.testing.assert_allclose(v.numpy(), u[f"final::{k}"], rtol=1e-3, atol=2e-5, err_msg=k)
    ref = dict(zip(u["stat_keys"].tolist(), u["stat_vals"].tolist()))
    for k in ("loss", "policy_loss", "entropy_loss", "value_loss", "grad_norm", "entropy"):
        assert math.isclose(stats[k], ref[k], rel_tol=1e-4, abs_tol=1e-6), (k, stats[k], ref[k])


def test_model_optimize_step_matches_reference_four_epochs_h196(monkeypatch):
    """The multi-step pin on CPU (tests/golden/update196e4.npz: update196's inputs through FOUR epochs,
    eight optimizer steps, each epoch in the reference's recorded order): the restatement's final
    parameters, statistics and final policy agree with the reference run after eight steps (fp32, the
    two runs differ in summation order only, which Muon's bf16 Newton-Schulz amplifies step by step)."""
    import agent
    import train
    from g2048.augment import encode_grid
    from g2048.optim import MultiOptimizer
    u, e = golden("update196.npz"), golden("update196e4.npz")
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=196, num_layers=2, dropout=0.0))
    m.load_state_dict({k[len("init::"):]: torch.from_numpy(u[k]) for k in u.files if k.startswith("init::")})
    lr, clr, b1, b2, wd, beta, critic = (float(x) for x in u["hparams"])
    n = len(u["actions"])
    obs = [encode_grid(u["boards"][i].reshape(4, 4).tolist()) for i in range(n)]
    moves = [{"game_state": obs[i], "selected_direction": int(u["actions"][i]),
              "action_mask": u["invalid"][i].tolist(), "advantage": float(u["advantage"][i]),
              "future_reward": float(u["future_reward"][i]), "policy_logprobs": u["old_logprobs"][i].tolist()}
             for i in range(n)]
    orders = iter([torch.from_numpy(o.astype(np.int64)) for o in e["order"]])
    real_randperm = torch.randperm
    monkeypatch.setattr(torch, "randperm", lambda k, *a, **kw: next(orders) if k == n else real_randperm(k, *a, **kw))
    o2d, o1d, v2d, v1d = m.get_param_groups(clr, lr)
    adamw = torch.optim.AdamW([o1d, v1d], betas=(b1, b2), weight_decay=wd)
    muon = torch.optim.Muon([o2d, v2d], adjust_lr_fn="match_rms_adamw", weight_decay=wd)
    stats = train.model_optimize_step(m, [{"moves": moves}], MultiOptimizer(muon, adamw), None, beta, critic,
                                      None, batch_size=int(e["batch_size"]), epochs=int(e["epochs"]))
    for k, v in m.state_dict().items():
        want = e[f"final::{k}"] - u[f"init::{k}"]
        got = v.numpy() - u[f"init::{k}"]
        cos = float(np.dot(got.ravel(), want.ravel()) / (np.linalg.norm(got) * np.linalg.norm(want) + 1e-30))
        assert cos > COS_E4_CPU, (k, cos)
    ref = dict(zip(e["stat_keys"].tolist(), e["stat_vals"].tolist()))
    for k in ("loss", "policy_loss", "entropy_loss", "value_loss", "grad_norm", "entropy"):
        assert math.isclose(stats[k], ref[k], rel_tol=1e-4, abs_tol=1e-6), (k, stats[k], ref[k])
    m.eval()
    with torch.no_grad():
        lg, val = m(torch.stack(obs))
    np.testing.assert_allclose(lg.numpy(), e["logits"], rtol=0, atol=LOGIT_E4_CPU)
    np.testing.assert_allclose(val.reshape(-1).numpy(), e["value"], rtol=0, atol=LOGIT_E4_CPU)


def test_cosine_schedule_matches_transformers():
    from transformers import get_scheduler
    from g2048.optim import cosine_with_warmup
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = get_scheduler("cosine", opt, num_warmup_steps=10, num_training_steps=100)
    f = cosine_with_warmup(10, 100)
    for step in range(120):
        assert math.isclose(opt.param_groups[0]["lr"], f(step), rel_tol=1e-12, abs_tol=1e-15), step
        opt.step()
        sch.step()


def test_augmentation_is_a_symmetry_of_the_game(games):
    """A mirrored/rotated step, with its remapped action, must be a legal transition of the
    transformed board (checked with the oracle's move)."""
    from g2048.augment import augment_steps, encode_grid
    from oracle import oracle as O
    g = games
    steps = []
    for i in range(400):
        if g["invalid"][i]:
            continue
        mask = [not (g["mask_before"][i] >> a & 1) for a in range(4)]
        steps.append({"state_before": g["before"][i].reshape(4, 4).tolist(),
                      "result_state": g["moved"][i].reshape(4, 4).tolist(),
                      "selected_direction": int(g["action"][i]), "action_mask": mask,
                      "policy_logprobs": [float(-k) for k in range(4)], "points_earned": int(g["points"][i])})
    aug = augment_steps(steps, 0.5, random.Random(3))
    assert len(aug) > 50
    for s in aug:
        before = np.array(s["state_before"], np.int8).reshape(16)
        out, pts, _ = O.move(before[None], s["selected_direction"])
        assert np.array_equal(out[0], np.array(s["result_state"], np.int8).reshape(16))
        assert pts[0] == s["points_earned"]
        legal = O.legal_mask(before[None])[0]
        assert s["action_mask"] == [not (legal >> a & 1) for a in range(4)]
        assert torch.equal(s["game_state"], encode_grid(s["state_before"]))
        assert sorted(s["policy_logprobs"]) == [-3.0, -2.0, -1.0, 0.0]


def test_augmentation_consumes_random_like_the_reference():
    """Same sequence of `random` calls as train.py:779-881 (sample, then random()/choice per step)."""
    from g2048.augment import augment_steps
    steps = [{"state_before": [[0] * 4] * 4, "result_state": [[0] * 4] * 4, "selected_direction": k % 4,
              "action_mask": [False] * 4, "policy_logprobs": [0.0] * 4} for k in range(40)]
    r1 = random.Random(9)
    aug = augment_steps(steps, 0.25, r1)
    r2 = random.Random(9)
    picked = r2.sample(steps, 10)
    expect = 0
    for _ in picked:
        if r2.random() < 0.5:
            r2.choice(["horizontal", "vertical"])
            expect += 1
        if r2.random() < 0.5:
            r2.choice([90, 180, 270])
            expect += 1
    assert len(aug) == expect
    assert r1.random() == r2.random()


def test_grad_bucket_views_and_clip():
    import agent
    from g2048.dist import GradBucket
    torch.manual_seed(0)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=16, num_layers=1, dropout=0.0))
    gb = GradBucket(m.parameters())
    x = torch.randn(32, 48)
    logits, v = m(x)
    (logits.square().sum() + v.sum()).backward()
    assert gb.check_views()
    ref = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone()
    assert torch.equal(gb.flat, ref)
    norm = gb.clip_(1.0)
    assert math.isclose(float(norm), float(ref.norm()), rel_tol=1e-6)
    assert math.isclose(float(gb.flat.norm()), 1.0, rel_tol=1e-4)
    gb.zero()
    assert float(gb.flat.abs().sum()) == 0.0 and gb.check_views()


def test_trim_rows_drops_copies_first_then_random_real_rows():
    """dist.trim_rows (equal_rows' local part): D4 copies go first; real rows are dropped as a
    uniformly random subset kept in order (a tail trim of time-major rows would drop only late moves)."""
    import torch
    from g2048.dist import trim_rows
    m, n_real = 100, 60
    data = {"a": torch.arange(m), "b": torch.arange(m) * 10}
    out = trim_rows(data, 80, n_real)
    assert torch.equal(out["a"], torch.arange(80))
    g = torch.Generator().manual_seed(0)
    out = trim_rows(data, 30, n_real, g)
    a = out["a"]
    assert a.numel() == 30 and torch.equal(out["b"], a * 10)
    assert bool((a < n_real).all()) and bool((a[1:] > a[:-1]).all())  # real rows only, original order
    assert int(a.max()) >= 45  # not a head/tail slice of the time-major rows
    assert a.tolist() != list(range(30))
    assert trim_rows(data, m, n_real) is data


@pytest.mark.parametrize("kind", ["mlp", "urm"])
def test_checkpoint_reload_picks_model_type(kind, tmp_path):
    """evaluate / export-demo rebuild the saved policy from best_model.pt's config (train.py:1893-1901
    layout): a GameURM checkpoint (the trainer's --model-type urm) reloads as GameURM, not GameMLP."""
    import agent
    import train
    torch.manual_seed(0)
    if kind == "urm":
        m = agent.GameURM(agent.GameURMConfig(hidden_dim=32, num_heads=2, num_layers=1, num_loops=2))
    else:
        m = agent.GameMLP(agent.MLPConfig(hidden_dim=32))
    torch.save({"model_state_dict": m.state_dict(), "config": m.config.model_dump(), "eval_avg_score": 1.0,
                "train_step": 3}, tmp_path / "best_model.pt")
    got = train.load_checkpoint_model(torch.load(tmp_path / "best_model.pt", map_location="cpu", weights_only=True))
    assert type(got) is type(m)
    x = torch.rand(5, 48)
    with torch.no_grad():
        a, b = m.eval()(x), got.eval()(x)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_urm_optimizer_groups_skip_gradless_init_hidden():
    """init_hidden feeds only the no-grad truncated loops when num_truncated_loops >= 1 (no gradient:
    torch's AdamW would skip it), so it is in the AdamW group only with num_truncated_loops = 0."""
    import agent
    for trunc, want in ((1, False), (0, True)):
        m = agent.GameURM(agent.GameURMConfig(hidden_dim=32, num_heads=2, num_truncated_loops=trunc))
        ids = {id(p) for g in m.get_param_groups(1e-3, 1e-3) for p in g["params"]}
        assert (id(m.init_hidden) in ids) is want


@pytest.mark.parametrize("ntl", [0, 1])
def test_urm_param_groups_cover_every_parameter_once(ntl):
    """GameURM.get_param_groups: Muon gets exactly the 2-D Linear weights (value head apart), AdamW
    the conv kernels, norms and biases; init_hidden joins the AdamW group only when it can have a
    gradient (num_truncated_loops == 0: the no-grad truncated loops are the only other user).  Every
    trainable parameter is in exactly one group (the group layout an optimizer
    checkpoint is keyed by)."""
    import agent
    m = agent.GameURM(agent.GameURMConfig(num_truncated_loops=ntl))
    o2, o1, v2, v1 = m.get_param_groups(1e-4, 1e-3)
    ids = [id(p) for g in (o2, o1, v2, v1) for p in g["params"]]
    assert len(ids) == len(set(ids))
    every = {id(p) for p in m.parameters()}
    missing = every - set(ids)
    assert missing == ({id(m.init_hidden)} if ntl else set())
    assert all(p.ndim == 2 for p in o2["params"] + v2["params"])
    assert all(p.ndim != 2 or p is m.init_hidden for p in o1["params"] + v1["params"])
    assert (any(p is m.init_hidden for p in o1["params"])) == (ntl == 0)
    assert {id(p) for p in v2["params"] + v1["params"]} == {id(p) for p in m.value_head.parameters()}


def test_muon_normalisation_quotient_is_correctly_rounded():
    """optim.hip's muon_kernel divides the bf16 image by its norm with one reciprocal and two fmas:
    exactly the correctly rounded fp32 quotient for every pair of bf16 significands (rational
    arithmetic, tools/check_bf16_division.py)."""
    import runpy
    import io
    import contextlib
    from pathlib import Path
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        runpy.run_path(str(Path(__file__).resolve().parent.parent / "tools" / "check_bf16_division.py"),
                       run_name="__main__")
    assert "mismatches 0 of 16384" in out.getvalue()
