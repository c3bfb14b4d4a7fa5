"""GPU parity: libg2048 env kernels vs the CPU oracle and the reference's golden vectors.

Integer/byte work must be bit-exact.  Every test here calls through the C ABI (g2048._lib).
"""

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible: GPU tests must run on an MI355X")
    return torch.device("cuda:0")


def L():
    from g2048 import _lib
    return _lib


def to_dev(a, dtype, dev):
    return torch.as_tensor(np.ascontiguousarray(a)).to(dtype).to(dev)


def gpu_step(boards_np, actions_np, dev, mode=None, inject=None, seed=0, counter=0, opts=0, random_actions=False,
             mt_state=None, env_base=0):
    lib = L()
    n = len(boards_np)
    b = to_dev(boards_np, torch.int8, dev)
    a = None if random_actions else to_dev(actions_np, torch.uint8, dev)
    aout = torch.zeros(n, dtype=torch.uint8, device=dev)
    pts = torch.zeros(n, dtype=torch.int32, device=dev)
    mx = torch.zeros(n, dtype=torch.int8, device=dev)
    pot = torch.zeros(n, 4, dtype=torch.int8, device=dev)
    fl = torch.zeros(n, dtype=torch.uint8, device=dev)
    inj = None if inject is None else to_dev(inject, torch.int32, dev)
    rng = lib.make_rng(lib.RNG_PHILOX if mode is None else mode, seed, counter, env_base, mt_state=mt_state,
                       inject=inj)
    lib.env_step(b, b, a, aout, pts, mx, pot, fl, rng, opts)
    torch.cuda.synchronize()
    return (b.cpu().numpy(), aout.cpu().numpy(), pts.cpu().numpy(), mx.cpu().numpy(), pot.cpu().numpy(),
            fl.cpu().numpy())


def random_boards(n, seed, hi=12, p_empty=0.35):
    rng = np.random.default_rng(seed)
    b = rng.integers(1, hi + 1, size=(n, 16)).astype(np.int8)
    b[rng.random(b.shape) < p_empty] = 0
    return b


def test_exhaustive_rows_all_directions(dev):
    """Every row over exponents 0..17 (18^4 rows), placed as row/column k, in all 4 directions."""
    vals = np.arange(18, dtype=np.int8)
    rows = np.stack(np.meshgrid(vals, vals, vals, vals, indexing="ij"), -1).reshape(-1, 4)
    for k, direction, layout in ((0, O.LEFT, "row"), (3, O.RIGHT, "row"), (1, O.UP, "col"), (2, O.DOWN, "col")):
        boards = np.zeros((len(rows), 16), np.int8)
        if layout == "row":
            boards[:, 4 * k:4 * k + 4] = rows
        else:
            boards[:, k::4] = rows
        inj = np.tile(np.array([[0, 1]], np.int32), (len(rows), 1))
        b, _, pts, mx, pot, fl = gpu_step(boards, np.full(len(rows), direction), dev, mode=L().RNG_INJECT, inject=inj)
        ob, f, _, moved = O.step(boards, direction, O.RNG_INJECT, inj_k=inj[:, 0], inj_v=inj[:, 1])
        assert np.array_equal(b, ob)
        assert np.array_equal(pts, f["points"])
        assert np.array_equal(mx, f["max_tile"])
        assert np.array_equal(pot[:, 0], f["mono_b"]) and np.array_equal(pot[:, 1], f["mono_a"])
        assert np.array_equal(pot[:, 2], f["empt_b"]) and np.array_equal(pot[:, 3], f["empt_a"])
        assert np.array_equal((fl >> 4) & 1, f["invalid"])
        assert np.array_equal(fl >> 7, f["done"])
        assert np.array_equal(fl & 0xF, O.legal_mask(ob))


def test_golden_row_table(dev):
    g = golden("rows.npz")
    boards = np.zeros((len(g["rows"]), 16), np.int8)
    boards[:, :4] = g["rows"]
    inj = np.tile(np.array([[0, 1]], np.int32), (len(boards), 1))
    for d, key in ((O.LEFT, "left"), (O.RIGHT, "right")):
        b, _, pts, mx, _, fl = gpu_step(boards, np.full(len(boards), d), dev, mode=L().RNG_INJECT, inject=inj)
        valid = g["legal_lr"][:, 0 if d == O.LEFT else 1].astype(bool)
        assert np.array_equal(((fl >> 4) & 1) == 0, valid)
        # legal moves: the golden row after the move, plus the injected spawn in the first empty cell
        moved = boards.copy()
        moved[:, :4] = g[key]
        exp_pts = np.where(valid, g[f"{key}_points"], 0)
        assert np.array_equal(pts, exp_pts)
        assert np.array_equal(mx, np.where(valid, g[f"{key}_max"], 0))
        first_empty = np.argmax(moved == 0, axis=1)
        moved[np.arange(len(moved)), first_empty] = 1
        assert np.array_equal(b[valid], moved[valid])
        assert np.array_equal(b[~valid], boards[~valid])


def test_seeded_games_mt19937_bit_exact(dev, games):
    """random.seed(s); reset(); step(a_t)... reproduced on the GPU with per-env MT19937 streams."""
    lib = L()
    g = games
    n = int(g["game"].max()) + 1
    seeds = torch.arange(n, dtype=torch.int64, device=dev)
    mt = torch.zeros(625 * n, dtype=torch.int32, device=dev)
    lib.mt_seed(mt, seeds)
    boards = torch.zeros(n, 16, dtype=torch.int8, device=dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    lib.env_reset(boards, flags, lib.make_rng(lib.RNG_MT19937, mt_state=mt))
    torch.cuda.synchronize()
    assert np.array_equal(boards.cpu().numpy(), g["init_boards"])
    by_game = [np.nonzero(g["game"] == s)[0] for s in range(n)]
    T = max(len(x) for x in by_game)
    rng = lib.make_rng(lib.RNG_MT19937, mt_state=mt)
    aout = torch.zeros(n, dtype=torch.uint8, device=dev)
    pts = torch.zeros(n, dtype=torch.int32, device=dev)
    mx = torch.zeros(n, dtype=torch.int8, device=dev)
    pot = torch.zeros(n, 4, dtype=torch.int8, device=dev)
    for t in range(T):
        live = np.array([t < len(x) for x in by_game])
        idx = np.array([x[t] if t < len(x) else 0 for x in by_game])
        acts = np.where(live, g["action"][idx], 0)
        a = to_dev(acts, torch.uint8, dev)
        lib.env_step(boards, boards, a, aout, pts, mx, pot, flags, rng, lib.OPT_SKIP_DONE)
        torch.cuda.synchronize()
        b, p, m, po, fl = (x.cpu().numpy() for x in (boards, pts, mx, pot, flags))
        li = idx[live]
        assert np.array_equal(b[live], g["after"][li]), t
        assert np.array_equal(p[live], g["points"][li])
        assert np.array_equal(m[live], g["max_tile"][li])
        assert np.array_equal(po[live, 0], g["mono_b"][li]) and np.array_equal(po[live, 1], g["mono_a"][li])
        assert np.array_equal(po[live, 2], g["empt_b"][li]) and np.array_equal(po[live, 3], g["empt_a"][li])
        assert np.array_equal((fl[live] >> 4) & 1, g["invalid"][li])
        assert np.array_equal(fl[live] >> 7, g["done"][li])
        assert np.array_equal(fl[live] & 0xF, g["mask_after"][li])
        assert ((fl[~live] & lib.FLAG_INACTIVE) != 0).all()


def test_best_game_replay_injected(dev):
    g = golden("best_game.npz")
    lib = L()
    b = to_dev(g["before"][:1], torch.int8, dev)
    n = len(g["action"])
    one = lambda dt: torch.zeros(1, dtype=dt, device=dev)  # noqa: E731
    aout, pts, mx, pot, fl = one(torch.uint8), one(torch.int32), one(torch.int8), torch.zeros(1, 4, dtype=torch.int8,
                                                                                             device=dev), one(torch.uint8)
    inj_all = torch.as_tensor(np.stack([g["spawn_k"], g["spawn_val"]], 1).astype(np.int32)).to(dev)
    acts = to_dev(g["action"], torch.uint8, dev)
    got_b, got_p = [], []
    for t in range(n):
        lib.env_step(b, b, acts[t:t + 1], aout, pts, mx, pot, fl,
                     lib.make_rng(lib.RNG_INJECT, inject=inj_all[t:t + 1].contiguous()))
        got_b.append(b.clone())
        got_p.append(pts.clone())
    torch.cuda.synchronize()
    assert np.array_equal(torch.cat(got_b).cpu().numpy(), g["after"])
    assert np.array_equal(torch.cat(got_p).cpu().numpy(), g["points"])
    assert int(fl.item()) & lib.FLAG_DONE  # terminal, as in the shipped replay
    assert int(torch.cat(got_p).sum()) == int(g["score"])


@pytest.mark.parametrize("seed", [1, 2])
def test_philox_random_steps_match_oracle(dev, seed):
    """Random legal actions + spawns drawn in-kernel (one Philox stream-1 draw) reproduce on the oracle."""
    n = 1 << 16
    boards = random_boards(n, seed, hi=17)
    ctr = 12345 + seed
    b, aout, pts, mx, pot, fl = gpu_step(boards, None, dev, seed=0x2048 + seed, counter=ctr, random_actions=True,
                                         env_base=777)
    ob, f, oa = O.step_random(boards, 0x2048 + seed, ctr, env_base=777)
    playable = O.legal_mask(boards) != 0
    assert np.array_equal(aout[playable], oa[playable])
    assert np.array_equal(b, ob)
    assert np.array_equal(pts, f["points"])
    assert np.array_equal(pot[:, 0], f["mono_b"]) and np.array_equal(pot[:, 1], f["mono_a"])
    assert np.array_equal(pot[:, 2], f["empt_b"]) and np.array_equal(pot[:, 3], f["empt_a"])
    assert np.array_equal(fl >> 7, f["done"])
    assert np.array_equal(fl & 0xF, O.legal_mask(ob))


@pytest.mark.parametrize("n,steps", [(4096, 200), (1000, 64), (70000, 20)])
def test_rollout_kernel_trajectories_match_oracle(dev, n, steps):
    """env_rollout_kernel (the bench workload): every per-step record bit-exact vs the oracle,
    including boards whose exponents exceed the LDS tables' range (compute-path fallback) and boards
    whose move creates the first exponent 12 (kLine12 -> SWAR statistics fallback)."""
    lib = L()
    init = O.reset(n, O.RNG_PHILOX, seed=31, step_idx=0, env_base=5)
    init[:7] = np.array([1, 2, 1, 2, 2, 1, 2, 1, 1, 2, 1, 2, 2, 1, 2, 1], np.int8)  # finished boards handed in
    hi = random_boards(n // 4, 77, hi=17, p_empty=0.5)
    hi[:, 0] = 14
    hi[:, 1] = 14  # a 14+14 merge produces 15 inside the table path
    init[n // 2:n // 2 + n // 4] = hi
    # boards inside the table range whose move can create a 12 (11 + 11): the next board's legal mask
    # and pair counts then come from the SWAR fallback instead of kLine12
    el = random_boards(n // 8, 78, hi=11, p_empty=0.5)
    el[:, 0] = 11
    el[:, 1] = 11
    init[n // 4:n // 4 + n // 8] = el
    b = to_dev(init, torch.int8, dev)
    tb = torch.zeros(steps, n, 16, dtype=torch.int8, device=dev)
    ta = torch.zeros(steps, n, dtype=torch.uint8, device=dev)
    tp = torch.zeros(steps, n, dtype=torch.int32, device=dev)
    tpot = torch.zeros(steps, n, 4, dtype=torch.int8, device=dev)
    tf = torch.zeros(steps, n, dtype=torch.uint8, device=dev)
    lib.env_rollout_random(b, steps, tb, ta, tp, tpot, tf, lib.make_rng(lib.RNG_PHILOX, 31, 1, 5))
    torch.cuda.synchronize()
    ob, rec = O.random_rollout_record(init, steps, 31, step0=1, env_base=5)
    assert np.array_equal(tb.cpu().numpy(), rec["boards"])
    assert np.array_equal(ta.cpu().numpy(), rec["actions"])
    assert np.array_equal(tp.cpu().numpy(), rec["points"])
    assert np.array_equal(tpot.cpu().numpy(), rec["pot"])
    assert np.array_equal(tf.cpu().numpy(), rec["flags"])
    assert np.array_equal(b.cpu().numpy(), ob)
    assert (rec["flags"] & 0x80).sum() > 0  # episodes ended and were reset inside the launch


@pytest.mark.parametrize("n,chunk,per_graph,k", [(1000, 5, 8, 11), (1000, 64, 8, 8), (65536, 8, 8, 3)])
def test_bench_graph_replay_matches_oracle(dev, n, chunk, per_graph, k):
    """bench.py's timed region: k rollout launches replayed from hipGraphs of `per_graph` launches
    (plus 1-launch graphs for the remainder), each launch advancing the device Philox counter itself
    (g2048_env_rollout_random_adv: its last workgroup adds `chunk`, the ticket word is left zero;
    65 536 boards = the bench's 256-workgroup grid), equal one oracle rollout of k * chunk steps; the
    last launch's records match its tail."""
    from bench import RolloutBench
    rb = RolloutBench(n, chunk, 0, dev)
    rb.capture(per_graph)  # runs one eager warm-up launch, then captures
    torch.cuda.synchronize()
    init, ctr0 = rb.env.boards.cpu().numpy().copy(), int(rb.ctr.item())
    rb.run(k)
    torch.cuda.synchronize()
    assert int(rb.ctr.item()) == ctr0 + k * chunk and int(rb.ticket.item()) == 0
    ob, rec = O.random_rollout_record(init, k * chunk, rb.env.seed, step0=ctr0, env_base=rb.env.env_base)
    assert np.array_equal(rb.env.boards.cpu().numpy(), ob)
    assert np.array_equal(rb.tb.cpu().numpy(), rec["boards"][-chunk:])
    assert np.array_equal(rb.tf.cpu().numpy(), rec["flags"][-chunk:])
    assert np.array_equal(rb.tp.cpu().numpy(), rec["points"][-chunk:])
    # the same k launches as ONE k-launch graph (bench.py's timed region, capture_exact)
    rb.capture_exact(k)
    init, ctr0 = rb.env.boards.cpu().numpy().copy(), int(rb.ctr.item())
    rb.run(k)
    torch.cuda.synchronize()
    assert int(rb.ctr.item()) == ctr0 + k * chunk and int(rb.ticket.item()) == 0
    ob, rec = O.random_rollout_record(init, k * chunk, rb.env.seed, step0=ctr0, env_base=rb.env.env_base)
    assert np.array_equal(rb.env.boards.cpu().numpy(), ob)
    assert np.array_equal(rb.tb.cpu().numpy(), rec["boards"][-chunk:])
    assert np.array_equal(rb.tpot.cpu().numpy(), rec["pot"][-chunk:])


def test_auto_reset_matches_oracle(dev):
    lib = L()
    # boards one move from the end: a full board with a single legal merge
    rng = np.random.default_rng(3)
    n = 4096
    base = np.array([1, 2, 1, 2, 2, 1, 2, 1, 1, 2, 1, 2, 2, 1, 3, 3], np.int8)
    boards = np.tile(base, (n, 1))
    boards[: n // 2] = random_boards(n // 2, 9)
    acts = np.where(np.arange(n) < n // 2, rng.integers(0, 4, n), O.LEFT)
    b, _, pts, _, _, fl = gpu_step(boards, acts, dev, seed=99, counter=5, opts=lib.OPT_AUTO_RESET)
    ob, f, _, _ = O.step(boards, acts, O.RNG_PHILOX, seed=99, step_idx=5)
    done = f["done"].astype(bool)
    assert done.sum() > 0
    fresh = O.reset(n, O.RNG_PHILOX, seed=99, step_idx=5)
    exp = np.where(done[:, None], fresh, ob)
    assert np.array_equal(b, exp)
    assert np.array_equal(((fl >> 5) & 1).astype(bool), done)
    assert np.array_equal(fl & 0xF, O.legal_mask(exp))
    assert np.array_equal(pts, f["points"])


def test_reset_philox_and_mt(dev):
    lib = L()
    n = 10000
    boards = torch.zeros(n, 16, dtype=torch.int8, device=dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    lib.env_reset(boards, flags, lib.make_rng(lib.RNG_PHILOX, 5, 17, env_base=3))
    torch.cuda.synchronize()
    exp = O.reset(n, O.RNG_PHILOX, seed=5, step_idx=17, env_base=3)
    assert np.array_equal(boards.cpu().numpy(), exp)
    assert np.array_equal(flags.cpu().numpy(), O.legal_mask(exp))
    seeds = np.arange(300, 300 + 256, dtype=np.uint64)
    mt = torch.zeros(625 * 256, dtype=torch.int32, device=dev)
    lib.mt_seed(mt, torch.as_tensor(seeds.astype(np.int64)).to(dev))
    b2 = torch.zeros(256, 16, dtype=torch.int8, device=dev)
    lib.env_reset(b2, None, lib.make_rng(lib.RNG_MT19937, mt_state=mt))
    torch.cuda.synchronize()
    assert np.array_equal(b2.cpu().numpy(), O.reset(256, O.RNG_MT, mt=O.MTStates(seeds)))
    # the device MT state after the reset equals the oracle's
    ost = O.MTStates(seeds)
    O.reset(256, O.RNG_MT, mt=ost)
    dev_words = mt.view(625, 256).cpu().numpy().view(np.uint32).T
    assert np.array_equal(dev_words, ost.words())


def test_legal_mask_and_obs(dev):
    lib = L()
    boards = random_boards(50000, 4, hi=17, p_empty=0.2)
    b = to_dev(boards, torch.int8, dev)
    fl = torch.zeros(len(boards), dtype=torch.uint8, device=dev)
    lib.legal_mask(b, fl)
    obs = torch.zeros(len(boards), 48, dtype=torch.float32, device=dev)
    obs16 = torch.zeros(len(boards), 48, dtype=torch.bfloat16, device=dev)
    lib.obs_encode(b, obs)
    lib.obs_encode(b, obs16)
    torch.cuda.synchronize()
    m = O.legal_mask(boards)
    assert np.array_equal(fl.cpu().numpy(), m | np.where(m == 0, 0x80, 0))
    exp = O.obs_encode(boards)
    assert np.array_equal(obs.cpu().numpy().view(np.uint32), exp.view(np.uint32))
    assert torch.equal(obs16.cpu(), torch.from_numpy(exp).to(torch.bfloat16))
    g = golden("mlp.npz")
    b2 = to_dev(g["boards"], torch.int8, dev)
    o2 = torch.zeros(len(g["boards"]), 48, dtype=torch.float32, device=dev)
    lib.obs_encode(b2, o2)
    assert np.array_equal(o2.cpu().numpy().view(np.uint32), g["obs"].view(np.uint32))


def test_large_n_invariants_and_determinism(dev):
    """2^22 boards: value conservation (merges keep sum of 2^e), points = merged values, spawn adds
    exactly one 2 or 4, and two runs with the same seed are identical."""
    lib = L()
    n = 1 << 22
    gen = torch.Generator(device="cpu").manual_seed(0)
    src = torch.randint(0, 12, (n, 16), generator=gen, dtype=torch.int8)
    src[torch.rand(n, 16, generator=gen) < 0.3] = 0
    acts = torch.randint(0, 4, (n,), generator=gen, dtype=torch.uint8)
    outs = []
    for _ in range(2):
        b = src.to(dev)
        n_ = b.shape[0]
        aout, pts = torch.zeros(n_, dtype=torch.uint8, device=dev), torch.zeros(n_, dtype=torch.int32, device=dev)
        mx, pot = torch.zeros(n_, dtype=torch.int8, device=dev), torch.zeros(n_, 4, dtype=torch.int8, device=dev)
        fl = torch.zeros(n_, dtype=torch.uint8, device=dev)
        lib.env_step(b, b, acts.to(dev), aout, pts, mx, pot, fl, lib.make_rng(lib.RNG_PHILOX, 7, 3))
        outs.append((b, pts, fl))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    b, pts, fl = outs[0]
    val = lambda x: torch.where(x > 0, torch.ones_like(x, dtype=torch.int64) << x.to(torch.int64), 0).sum(1)  # noqa
    before, after = val(src.to(dev)), val(b)
    invalid = (fl & lib.FLAG_INVALID) != 0
    spawned = after - before
    assert torch.equal(spawned[invalid], torch.zeros_like(spawned[invalid]))
    assert bool(((spawned[~invalid] == 2) | (spawned[~invalid] == 4)).all())
    assert bool((pts[invalid] == 0).all())
    # subsample vs the oracle
    sub = torch.arange(0, n, 4099)
    ob, f, _, _ = O.step(src[sub].numpy(), acts[sub].numpy(), O.RNG_PHILOX, seed=7, step_idx=3, env_base=0)
    # env ids of the subsample differ from 0..len(sub)-1: only compare the deterministic parts
    assert np.array_equal(pts[sub.to(dev)].cpu().numpy(), f["points"])
    assert np.array_equal((fl[sub.to(dev)].cpu().numpy() >> 4) & 1, f["invalid"])


def test_info_deltas_match_reference_games(dev):
    """g2048_info_deltas (smoothness / corner / adjacency / chain / topological after - before the
    move, game.py:981-1002) on the 8 200 golden transitions of the reference's seeded games:
    bit-identical float64 deltas, zeros on the illegal actions."""
    from g2048 import _lib as L
    g = golden("games.npz")
    b = torch.from_numpy(g["before"]).to(dev)
    a = torch.from_numpy(g["action"].astype(np.uint8)).to(dev)
    out = torch.zeros(len(b), 5, dtype=torch.float64, device=dev)
    anc = torch.zeros(len(b), dtype=torch.int8, device=dev)
    L.info_deltas(b, a, out, anc)
    got = out.cpu().numpy()
    for col, key in enumerate(("smooth_d", "corner_d", "adj_d", "chain_d", "topo_d")):
        np.testing.assert_array_equal(got[:, col], g[key], err_msg=key)
    assert (got[g["invalid"] == 1] == 0).all()
    # anchors vs the C oracle's restatement of _choose_anchor_corner
    _, want = O.info_heuristics(g["before"])
    live = g["invalid"] == 0
    np.testing.assert_array_equal(anc.cpu().numpy()[live], want[live])


def test_info_deltas_high_tiles(dev):
    """Boards with long chains and tiles up to 2^17 (deep DFS) vs the C oracle."""
    from g2048 import _lib as L
    rng = np.random.default_rng(5)
    n = 20000
    boards = rng.integers(0, 18, size=(n, 16)).astype(np.int8)
    boards[rng.random((n, 16)) < 0.3] = 0
    snake = np.array([17, 16, 15, 14, 10, 11, 12, 13, 9, 8, 7, 6, 2, 3, 4, 5], np.int8)
    boards[:500] = snake
    acts = rng.integers(0, 4, size=n).astype(np.uint8)
    out = torch.zeros(n, 5, dtype=torch.float64, device=dev)
    L.info_deltas(torch.from_numpy(boards).to(dev), torch.from_numpy(acts).to(dev), out)
    _, f, info, _ = O.step(boards, acts.astype(np.int64), O.RNG_INJECT, inj_k=np.zeros(n, np.int32),
                           inj_v=np.ones(n, np.int32), full_info=True)
    np.testing.assert_array_equal(out.cpu().numpy(), np.where(f["invalid"][:, None] == 1, 0.0, info))
