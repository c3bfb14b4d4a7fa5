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
