"""GPU parity of the fused persistent policy rollout (g2048_policy_rollout, csrc/policy_rollout.hip;
SURVEY.md §8(f) f1) against the per-step path it replaces (Rollout._step: obs_encode -> FusedPolicy
-> sample_actions -> env_step, train.py:240-337), which the other GPU tests pin to the reference.

The fused kernel reproduces every operand fragment, MFMA accumulation chain, rounding and reduction
order of the per-step kernels, so the comparison is BITWISE on every record: boards, flags, actions,
log-probabilities, entropies, values, points, max tiles and potentials."""

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

FIELDS = ("boards", "flags", "actions", "logp", "entropy", "value", "points", "max_tile", "pot")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    return torch.device("cuda:0")


def _model(dev, h, seed):
    import agent
    torch.manual_seed(seed)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=h, num_layers=2)).to(dev)
    with torch.no_grad():  # non-trivial heads and LayerNorm affines (the trainer zeroes the heads)
        for p in m.parameters():
            p.add_(torch.randn_like(p) * 0.05)
        m.action_head.weight.mul_(20.0)
    return m.eval()


def _run(dev, m, n, T, fused, episodic=False, seed=9, chunks=None, env_base=0):
    from g2048.rollout import FusedPolicy, Rollout
    pol = FusedPolicy(m)
    ro = Rollout(n, T, dev, seed=seed, env_base=env_base, episodic=episodic)
    ro.use_fused = fused
    assert ro.fused(pol) == fused
    ro.reset()
    for t0, t1 in chunks or [(0, T)]:
        ro.steps(t0, t1, pol)
    torch.cuda.synchronize()
    return {k: getattr(ro.buf, k).clone() for k in FIELDS}


def _assert_same(a, b):
    for k in FIELDS:
        x, y = a[k], b[k]
        if x.dtype.is_floating_point:  # bitwise, -inf included
            x, y = x.view(torch.int32), y.view(torch.int32)
        bad = (x != y).reshape(x.shape[0], x.shape[1], -1).any(-1)
        assert not bool(bad.any()), (k, int(bad.sum()), torch.nonzero(bad)[:5].tolist())


@pytest.mark.parametrize("h,n,T,episodic", [(196, 4099, 24, False), (196, 1000, 40, True), (192, 2048, 16, False),
                                             (64, 777, 32, True), (32, 300, 20, False)])
def test_fused_rollout_bitwise_equals_per_step_path(dev, h, n, T, episodic):
    from g2048 import _lib as L
    assert L.policy_rollout_supported(h, 2)
    m = _model(dev, h, h + n)
    ref = _run(dev, m, n, T, fused=False, episodic=episodic)
    got = _run(dev, m, n, T, fused=True, episodic=episodic)
    _assert_same(ref, got)
    # the records are a real game: every action legal where the game is live
    fl, act = got["flags"][:-1].cpu().numpy(), got["actions"].cpu().numpy()
    live = (fl & 0xF) != 0
    assert ((fl[live] >> act[live]) & 1).all()
    assert bool(torch.isfinite(got["value"]).all())


def test_fused_rollout_chunks_and_env_base(dev):
    """Launches of sub-ranges [t0, t1) continue each other exactly; env_base offsets the Philox env
    ids like the per-step path (a rank's shard)."""
    m = _model(dev, 196, 5)
    ref = _run(dev, m, 2000, 30, fused=False, env_base=777)
    got = _run(dev, m, 2000, 30, fused=True, chunks=[(0, 7), (7, 8), (8, 30)], env_base=777)
    _assert_same(ref, got)


def test_fused_rollout_graph_replay(dev):
    """Rollout.collect(graph=True) with the fused kernel (one launch per rollout, device Philox
    counter) equals the eager per-step collection, replay after replay."""
    from g2048.rollout import FusedPolicy, Rollout
    m = _model(dev, 196, 11)
    pol = FusedPolicy(m)
    outs = []
    for fused, graph in ((False, False), (True, True)):
        ro = Rollout(4096, 16, dev, seed=3)
        ro.use_fused = fused
        ro.reset()
        rec = []
        for _ in range(3):
            ro.collect(pol, graph=graph)
            rec.append({k: getattr(ro.buf, k).clone() for k in FIELDS})
            ro.buf.carry_over()
        outs.append(rec)
    for a, b in zip(*outs):
        _assert_same(a, b)


def test_fused_rollout_full_size_matches_per_step(dev):
    """BASELINE config 3's shape: 65 536 envs, h = 196, fixed horizon."""
    m = _model(dev, 196, 21)
    ref = _run(dev, m, 65536, 12, fused=False)
    got = _run(dev, m, 65536, 12, fused=True)
    _assert_same(ref, got)
    # env transitions are game.step's (C oracle, same Philox spawn stream: counter 1 after the
    # reset, step t's spawn at counter 1 + 2t + 1), bit-exact where no auto-reset happened
    b = got["boards"].cpu().numpy()
    a = got["actions"].cpu().numpy()
    fl = got["flags"].cpu().numpy()
    pts = got["points"].cpu().numpy()
    for t in range(3):
        nxt, f, _, _ = O.step(b[t], a[t], O.RNG_PHILOX, seed=9, step_idx=1 + 2 * t + 1)
        keep = (fl[t + 1] & 0x20) == 0
        np.testing.assert_array_equal(nxt[keep], b[t + 1][keep])
        np.testing.assert_array_equal(f["points"], pts[t])


def test_fused_rollout_rejects_bad_arguments(dev):
    from g2048 import _lib as L
    m = _model(dev, 196, 2)
    from g2048.rollout import FusedPolicy, Rollout
    pol = FusedPolicy(m)
    ro = Rollout(256, 8, dev)
    with pytest.raises(L.G2048Error):
        L.policy_rollout(ro.buf, 0, 9, pol.wbf[0], pol.wbf[1:], [x.weight for x in pol.ln], [x.bias for x in pol.ln],
                         pol.head_bf, pol.heads[1], pol.heads[3], 1, 0, ro.counter, ro.opts)
    assert not L.policy_rollout_supported(196, 3) and not L.policy_rollout_supported(256, 2)
