"""Python face of the CPU oracle.  TEST INFRASTRUCTURE ONLY -- the checker, never the product.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.

* Engine functions wrap oracle/g2048_oracle.c (built by oracle/Makefile into oracle/_build/) via
  ctypes; see that file's header for the reference lines each function restates.
* `reward_rtg_normalize` restates train.py:699-772 and :898-901 (calculate_advantage without the
  D4 up-sampling) in float64 numpy, in the same operation order as the reference's Python loops.
* `masked_policy` restates the rollout's masked softmax / entropy / log_softmax
  (train.py:266-291, :326) in float64.

Parity pin: tests/test_oracle.py checks everything here against tests/golden/*.npz, produced from
the reference itself by tools/gen_golden.py.
"""

from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "liboracle.so"

UP, DOWN, LEFT, RIGHT = 0, 1, 2, 3
RNG_PHILOX, RNG_MT, RNG_INJECT = 0, 1, 2

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        _lib = ctypes.CDLL(str(LIB_PATH))
        _declare(_lib)
    return _lib


def _p(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _declare(L):
    vp, i64, u64, u32, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.or_mt_state_bytes.restype = ctypes.c_size_t
    L.or_mt_seed_batch.argtypes = [vp, vp, i64]
    L.or_mt_u32_batch.argtypes = [vp, vp, i64]
    L.or_move_batch.argtypes = [vp, vp, vp, vp, vp, i64]
    L.or_legal_batch.argtypes = [vp, vp, i64]
    L.or_potentials_batch.argtypes = [vp, vp, vp, i64]
    L.or_info_batch.argtypes = [vp, vp, vp, i64]
    L.or_obs_batch.argtypes = [vp, vp, i64]
    L.or_step_batch.argtypes = [vp, vp, i64, i32, u64, u64, u32, vp, vp, vp, i32, vp, vp, vp]
    L.or_reset_batch.argtypes = [vp, i64, i32, u64, u64, u32, vp]
    L.or_philox_batch.argtypes = [u64, u64, u32, u32, vp, i64]
    L.or_philox4x32_10.argtypes = [vp, vp, vp]
    L.or_random_rollout.argtypes = [vp, i64, i64, u64, u64, u32, i32]
    L.or_random_rollout.restype = i64
    L.or_random_rollout_rec.argtypes = [vp, i64, i64, u64, u64, u32, i32, vp, vp, vp, vp, vp]
    L.or_random_rollout_rec.restype = i64
    L.or_step_random_batch.argtypes = [vp, i64, u64, u64, u32, vp]


def _boards(b) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(b, dtype=np.int8).reshape(-1, 16))
    return a


# ---------------------------------------------------------------- RNG ---------------------------
class MTStates:
    """A batch of CPython-compatible MT19937 generators, one per env (random.seed(seed_i))."""

    def __init__(self, seeds):
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64).reshape(-1))
        self.n = len(seeds)
        self.nbytes = lib().or_mt_state_bytes()
        self.buf = np.zeros(self.n * self.nbytes, dtype=np.uint8)
        lib().or_mt_seed_batch(_p(self.buf), _p(seeds), self.n)

    def ptr(self):
        return _p(self.buf)

    def words(self) -> np.ndarray:
        """[n, 625] uint32 = mt[624] + index (the layout the device MT state uses too)."""
        return self.buf.view(np.uint32).reshape(self.n, -1)[:, :625].copy()

    def u32(self, count: int, env: int = 0) -> np.ndarray:
        out = np.zeros(count, np.uint32)
        view = self.buf[env * self.nbytes:(env + 1) * self.nbytes]
        lib().or_mt_u32_batch(_p(view), _p(out), count)
        return out


def philox4x32_10(ctr, key) -> np.ndarray:
    c = np.ascontiguousarray(np.asarray(ctr, np.uint32))
    k = np.ascontiguousarray(np.asarray(key, np.uint32))
    out = np.zeros(4, np.uint32)
    lib().or_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def philox_draws(seed: int, step: int, n: int, stream: int, env_base: int = 0) -> np.ndarray:
    out = np.zeros((n, 4), np.uint32)
    lib().or_philox_batch(seed, step, env_base, stream, _p(out), n)
    return out


# ---------------------------------------------------------------- engine ------------------------
def move(boards, dirs):
    b = _boards(boards)
    n = len(b)
    d = np.ascontiguousarray(np.broadcast_to(np.asarray(dirs, np.int64), (n,)))
    out = np.zeros_like(b)
    pts = np.zeros(n, np.int64)
    mx = np.zeros(n, np.int32)
    lib().or_move_batch(_p(b), _p(d), _p(out), _p(pts), _p(mx), n)
    return out, pts, mx


def legal_mask(boards) -> np.ndarray:
    b = _boards(boards)
    m = np.zeros(len(b), np.uint8)
    lib().or_legal_batch(_p(b), _p(m), len(b))
    return m


def potentials(boards):
    b = _boards(boards)
    mono = np.zeros(len(b), np.int32)
    empt = np.zeros(len(b), np.int32)
    lib().or_potentials_batch(_p(b), _p(mono), _p(empt), len(b))
    return mono, empt


def info_heuristics(boards):
    b = _boards(boards)
    out = np.zeros((len(b), 5), np.float64)
    anchor = np.zeros(len(b), np.int32)
    lib().or_info_batch(_p(b), _p(out), _p(anchor), len(b))
    return out, anchor


def obs_encode(boards) -> np.ndarray:
    b = _boards(boards)
    obs = np.zeros((len(b), 48), np.float32)
    lib().or_obs_batch(_p(b), _p(obs), len(b))
    return obs


STEP_FIELDS = ("points", "max_tile", "invalid", "done", "mono_b", "mono_a", "empt_b", "empt_a",
               "maxexp_b", "maxexp_a")


def step(boards, dirs, rng_mode=RNG_PHILOX, seed=0, step_idx=0, env_base=0, mt: MTStates | None = None,
         inj_k=None, inj_v=None, full_info=False):
    """game.step on a batch (in a copy).  Returns (boards_after, dict of fields, info[n,5], moved)."""
    b = _boards(boards).copy()
    n = len(b)
    d = np.ascontiguousarray(np.broadcast_to(np.asarray(dirs, np.int64), (n,)))
    out = np.zeros((n, 10), np.int64)
    info = np.zeros((n, 5), np.float64)
    moved = np.zeros_like(b)
    ik = None if inj_k is None else np.ascontiguousarray(np.asarray(inj_k, np.int32))
    iv = None if inj_v is None else np.ascontiguousarray(np.asarray(inj_v, np.int32))
    lib().or_step_batch(_p(b), _p(d), n, rng_mode, seed, step_idx, env_base, mt.ptr() if mt else None,
                        _p(ik), _p(iv), int(full_info), _p(out), _p(info), _p(moved))
    return b, {k: out[:, i] for i, k in enumerate(STEP_FIELDS)}, info, moved


def reset(n, rng_mode=RNG_PHILOX, seed=0, step_idx=0, env_base=0, mt: MTStates | None = None):
    b = np.zeros((n, 16), np.int8)
    lib().or_reset_batch(_p(b), n, rng_mode, seed, step_idx, env_base, mt.ptr() if mt else None)
    return b


def random_rollout(boards, steps, seed, step0=0, env_base=0, full_info=True):
    """In-place CPU random-legal rollout with auto-reset; returns transitions executed."""
    b = _boards(boards)
    return lib().or_random_rollout(_p(b), len(b), steps, seed, step0, env_base, int(full_info)), b


def random_rollout_record(boards, steps, seed, step0=0, env_base=0):
    """Checker of env_rollout_kernel: returns (final boards, dict of [steps, n] records)."""
    b = _boards(boards).copy()
    n = len(b)
    rec = {"boards": np.zeros((steps, n, 16), np.int8), "actions": np.zeros((steps, n), np.uint8),
           "points": np.zeros((steps, n), np.int32), "pot": np.zeros((steps, n, 4), np.int8),
           "flags": np.zeros((steps, n), np.uint8)}
    lib().or_random_rollout_rec(_p(b), n, steps, seed, step0, env_base, 0, _p(rec["boards"]), _p(rec["actions"]),
                                _p(rec["points"]), _p(rec["pot"]), _p(rec["flags"]))
    return b, rec


def step_random(boards, seed, step_idx=0, env_base=0):
    """The synthetic-policy step (one stream-1 draw for action + spawn). Returns (boards, fields, actions)."""
    b = _boards(boards).copy()
    out = np.zeros((len(b), 11), np.int64)
    lib().or_step_random_batch(_p(b), len(b), seed, step_idx, env_base, _p(out))
    return b, {k: out[:, i] for i, k in enumerate(STEP_FIELDS)}, out[:, 10]


# ---------------------------------------------------------------- policy / returns --------------
def masked_policy(logits, invalid):
    """train.py:266-291,326: probs, entropy over p>0, log_softmax of the -inf-masked logits."""
    lg = np.asarray(logits, np.float64).copy()
    inv = np.asarray(invalid, bool)
    lg[inv] = -np.inf
    m = lg.max(axis=1, keepdims=True)
    e = np.exp(lg - m)
    p = e / e.sum(axis=1, keepdims=True)
    logp = (lg - m) - np.log(e.sum(axis=1, keepdims=True))
    with np.errstate(divide="ignore", invalid="ignore"):
        ent = -np.where(p > 0, p * np.log(np.where(p > 0, p, 1.0)), 0.0).sum(axis=1)
    return p, ent, logp


def reward_rtg_normalize(points, mono_b, mono_a, empt_b, empt_a, done, value, episode_end, gamma,
                         w_points, w_mono, w_empt, rtg_beta, rtg_m2, rtg_mu, rtg_step, rtg_first_moment=None):
    """calculate_advantage (train.py:699-772, 898-901) for flat step arrays in episode order.

    `done` zeroes the "after" potentials like play_game_for_episode does (train.py:318,322);
    `episode_end[i]` marks the last stored step of each episode (G resets after it).
    Returns dict(reward, g_raw, g_norm, adv, moments=(first_moment, m2, mu), batch=(mean, var)).
    """
    points = np.asarray(points, np.float64)
    done = np.asarray(done, bool)
    mono_a = np.where(done, 0.0, np.asarray(mono_a, np.float64))
    empt_a = np.where(done, 0.0, np.asarray(empt_a, np.float64))
    mono_b = np.asarray(mono_b, np.float64)
    empt_b = np.asarray(empt_b, np.float64)
    shaped = 0 + w_mono * (gamma * mono_a - mono_b)  # sum([...]) starts from int 0
    shaped = shaped + w_empt * (gamma * empt_a - empt_b)
    reward = points * w_points + shaped
    n = len(reward)
    g_raw = np.zeros(n, np.float64)
    G = 0.0
    ends = np.asarray(episode_end, bool)
    for t in range(n - 1, -1, -1):
        if ends[t]:
            G = 0.0
        G = reward[t] + gamma * G
        g_raw[t] = G
    if rtg_first_moment is None:
        rtg_first_moment = rtg_mu
    eps = 1e-8
    mean = sum(g_raw.tolist()) / n
    var = 0.0 if n <= 1 else sum((x - mean) ** 2 for x in g_raw.tolist()) / n
    bc = max(1 - rtg_beta ** max(rtg_step, 1), eps)
    mu_c = rtg_mu / bc
    m2_c = rtg_m2 / bc
    std = max(m2_c - mu_c ** 2, eps) ** 0.5
    g_norm = (g_raw - mu_c) / (std + eps)
    adv = g_norm - np.asarray(value, np.float64)
    new_mu = rtg_beta * rtg_mu + (1 - rtg_beta) * mean
    new_m2 = rtg_beta * rtg_m2 + (1 - rtg_beta) * (var + mean ** 2)
    return {"reward": reward, "g_raw": g_raw, "g_norm": g_norm, "adv": adv,
            "moments": (new_mu, new_m2, new_mu), "batch": (mean, var), "mu_c": mu_c, "std": std}


# ---------------------------------------------------------------- D4 up-sampling ----------------
# calculate_advantage's augmentation (train.py:774-881) with the build's device sampling convention
# (include/g2048.h g2048_augment): which rows and transforms are drawn is the build's (Feistel +
# Philox instead of Python's `random`), the transforms themselves restate the reference.

def mirror_grid(g, direction):
    """Game2048.mirror_grid (game.py:509-535), 4x4 nested lists or arrays."""
    out = [[0] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            if direction == "horizontal":
                out[i][3 - j] = g[i][j]
            else:
                out[3 - i][j] = g[i][j]
    return out


def rotate_grid(g, degrees):
    """Game2048.rotate_grid (game.py:537-590), clockwise."""
    out = [[0] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            if degrees == 90:
                out[j][3 - i] = g[i][j]
            elif degrees == 180:
                out[3 - i][3 - j] = g[i][j]
            else:
                out[3 - j][i] = g[i][j]
    return out


_DIRS = [UP, DOWN, LEFT, RIGHT]
_ROT90 = {UP: RIGHT, RIGHT: DOWN, DOWN: LEFT, LEFT: UP}  # train.py:797-803


def remap_direction_mirror(d, axis):  # train.py:784-793
    if axis == "horizontal" and d in (LEFT, RIGHT):
        return LEFT if d == RIGHT else RIGHT
    if axis == "vertical" and d in (UP, DOWN):
        return UP if d == DOWN else DOWN
    return d


def remap_direction_rotate(d, degrees):  # train.py:795-808
    for _ in range(degrees // 90):
        d = _ROT90[d]
    return d


def _lowbias32(h):
    h = np.uint32(h)
    h ^= h >> np.uint32(16)
    h = np.uint32((int(h) * 0x7FEB352D) & 0xFFFFFFFF)
    h ^= h >> np.uint32(15)
    h = np.uint32((int(h) * 0x846CA68B) & 0xFFFFFFFF)
    h ^= h >> np.uint32(16)
    return int(h)


def augment_plan(n, k, seed, counter):
    """[(source row, transforms)] of the build's sampler: sample j -> row perm(j) of a 4-round
    Feistel permutation (keys = Philox (seed, counter, 0xFFFFFFFF, stream 4)) cycle-walked into
    [0, n); Philox (seed, counter, j, stream 3) = x, y, z, w: x < 2^31 -> mirror (y < 2^31
    horizontal), z < 2^31 -> rotation by 90 * (1 + floor(3 w / 2^32)).  Pure Python (small k)."""
    bits = 2
    while (1 << bits) < n:
        bits += 2
    half = bits // 2
    mask = (1 << half) - 1
    key = [int(v) for v in philox4x32_10([counter & 0xFFFFFFFF, counter >> 32, 0xFFFFFFFF, 4],
                                         [seed & 0xFFFFFFFF, seed >> 32])]
    draws = philox_draws(seed, counter, k, 3)
    plan = []
    for j in range(k):
        x = j
        while True:
            lo, hi = x & mask, x >> half
            l, r = hi, lo
            for q in range(4):
                l, r = r, l ^ (_lowbias32(r ^ key[q]) & mask)
            x = (l << half) | r
            if x < n:
                break
        u = [int(v) for v in draws[j]]
        tr = []
        if u[0] < 2 ** 31:
            tr.append(("mirror", "horizontal" if u[1] < 2 ** 31 else "vertical"))
        if u[2] < 2 ** 31:
            tr.append(("rotate", 90 * (1 + ((u[3] * 3) >> 32))))
        plan.append((x, tr))
    return plan


def augment_rows(boards, actions, legal, logp, adv, ret, plan):
    """The copies of train.py:826-881 for `plan`, in order (mirror before rotation per sample):
    returns arrays (boards [c,16] int8, actions, legal (bits 0-3 remapped, others kept), logp [c,4],
    adv, ret)."""
    ob, oa, ol, op, oad, ort = [], [], [], [], [], []
    for src, trs in plan:
        g = np.asarray(boards[src], np.int8).reshape(4, 4).tolist()
        for kind, arg in trs:
            if kind == "mirror":
                ng, fn = mirror_grid(g, arg), (lambda d, a=arg: remap_direction_mirror(d, a))
            else:
                ng, fn = rotate_grid(g, arg), (lambda d, a=arg: remap_direction_rotate(d, a))
            lg = int(legal[src])
            nl = lg & ~0xF
            nlp = [0.0] * 4
            for d in range(4):
                nl |= ((lg >> d) & 1) << fn(d)
                nlp[fn(d)] = float(logp[src][d])
            ob.append(np.asarray(ng, np.int8).reshape(16))
            oa.append(fn(int(actions[src])))
            ol.append(nl)
            op.append(nlp)
            oad.append(float(adv[src]))
            ort.append(float(ret[src]))
    c = len(ob)
    return (np.asarray(ob, np.int8).reshape(c, 16), np.asarray(oa, np.uint8), np.asarray(ol, np.uint8),
            np.asarray(op, np.float32).reshape(c, 4), np.asarray(oad, np.float32), np.asarray(ort, np.float32))
