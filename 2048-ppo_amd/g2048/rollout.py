"""Policy-driven rollouts into time-major device buffers (replaces play_game_for_episode,
train.py:213-345, and the missing batched_rollout module, train.py:30).

Per step t, for all N envs at once and with no host synchronisation:
  obs_encode(boards[t])                      to_model_format            game.py:92-101
  logits, value = policy(obs)                model(model_input)         train.py:261
  sample(logits, legal[t])                   mask/softmax/multinomial   train.py:266-291, :326
  env_step(boards[t] -> boards[t+1])         game.step                  game.py:952-1030
Buffers are [T(+1), N, ...] so the reward scan and the update read them in place.
"""

from __future__ import annotations

import copy

import torch

from . import _lib as L
from .dist import graph as graph_capture


class InferencePolicy:
    """A low-precision, eval-mode copy of a policy module for rollouts.

    `sync()` copies the master (fp32) weights in place, so tensor addresses stay fixed and a
    captured hipGraph of the rollout keeps working across updates.
    """

    def __init__(self, model: torch.nn.Module, dtype=torch.bfloat16):
        self.master = model
        self.dtype = dtype
        self.module = copy.deepcopy(model).to(dtype).eval()
        for p in self.module.parameters():
            p.requires_grad_(False)

    @torch.no_grad()
    def sync(self):
        for p, q in zip(self.module.parameters(), self.master.parameters()):
            p.copy_(q)

    @torch.no_grad()
    def __call__(self, obs: torch.Tensor):
        logits, value = self.module(obs.to(self.dtype))
        return logits.float(), value.float().view(-1)


class FusedPolicy:
    """The reference's GameMLP in eval mode (game.py:1145-1220) as MFMA kernels for the rollout:
    per layer one g2048_mlp_fwd (Linear + LayerNorm + ReLU [+ residual]), then g2048_head_fwd for
    the action logits and the value.  bf16 weights are refreshed in place by sync() (addresses stay
    fixed for a captured rollout graph); LayerNorm and head parameters are read from the master.
    Drop-in for InferencePolicy: __call__(obs bf16 [n, 48]) -> (logits fp32 [n, 4], value fp32 [n])."""

    def __init__(self, model: torch.nn.Module):
        self.master = model
        self.dtype = torch.bfloat16
        self.lin = [model.stem[0].weight] + [b.mlp[0].weight for b in model.backbone]
        self.ln = [model.stem[1]] + [b.mlp[1] for b in model.backbone]
        self.heads = (model.action_head.weight, model.action_head.bias, model.value_head.weight, model.value_head.bias)
        self.wbf = [torch.empty_like(w, dtype=torch.bfloat16) for w in self.lin]
        h = self.lin[0].shape[0]
        # the fused rollout kernel (g2048_policy_rollout) reads the heads as one zero-padded bf16
        # [5, 32 ceil(h/32)] block: action_head rows 0..3, value_head row 4
        self.fused_rollout = L.policy_rollout_supported(h, len(self.lin) - 1)
        self.head_bf = torch.zeros(5, 32 * ((h + 31) // 32), dtype=torch.bfloat16, device=self.lin[0].device)
        self._n = -1
        self.sync()

    @staticmethod
    def supports(model) -> bool:
        try:
            import agent
        except ImportError:  # pragma: no cover
            return False
        if not isinstance(model, agent.GameMLP):
            return False
        lin = [model.stem[0].weight] + [b.mlp[0].weight for b in model.backbone]
        return all(L.mlp_fwd_supported(w.shape[0], w.shape[1]) for w in lin) and model.config.hidden_dim <= 256

    @torch.no_grad()
    def sync(self):
        for w, b in zip(self.lin, self.wbf):
            b.copy_(w)
        h = self.lin[0].shape[0]
        self.head_bf[:4, :h].copy_(self.heads[0])
        self.head_bf[4, :h].copy_(self.heads[2][0])

    def rollout_steps(self, ro, t0: int, t1: int):
        """Steps t0 .. t1-1 of Rollout `ro` in ONE g2048_policy_rollout launch (bitwise the per-step
        path: obs_encode + this policy + sample_actions + env_step per step)."""
        L.policy_rollout(ro.buf, t0, t1, self.wbf[0], self.wbf[1:], [ln.weight for ln in self.ln],
                         [ln.bias for ln in self.ln], self.head_bf, self.heads[1], self.heads[3], ro.seed,
                         ro.env_base, ro.counter, ro.opts)

    def _buffers(self, n: int, dev):
        if self._n != n:
            h = self.lin[0].shape[0]
            self.h = [torch.empty(n, h, dtype=torch.bfloat16, device=dev) for _ in range(2)]
            self.logits = torch.empty(n, 4, dtype=torch.float32, device=dev)
            self.value = torch.empty(n, dtype=torch.float32, device=dev)
            self._n = n

    @torch.no_grad()
    def __call__(self, obs: torch.Tensor):
        if obs.dtype != torch.bfloat16:
            obs = obs.to(torch.bfloat16)
        self._buffers(obs.shape[0], obs.device)
        x = obs.contiguous()
        for l, (w, ln) in enumerate(zip(self.wbf, self.ln)):
            y = self.h[l % 2]
            L.mlp_fwd(x, w, ln.weight, ln.bias, l > 0, None, y, None, None, None)
            x = y
        L.head_fwd(x, *self.heads, self.logits, self.value)
        return self.logits, self.value


def make_policy(model: torch.nn.Module, dtype=torch.bfloat16):
    """The rollout policy: FusedPolicy for the reference's GameMLP and URMPolicy (g2048/urm.py) for its
    GameURM on a ROCm device (bf16), the generic module copy (InferencePolicy) otherwise."""
    dev = next(model.parameters()).device
    if dtype == torch.bfloat16 and dev.type == "cuda" and FusedPolicy.supports(model):
        return FusedPolicy(model)
    from .urm import URMPolicy
    if dtype == torch.bfloat16 and dev.type == "cuda" and URMPolicy.supports(model):
        return URMPolicy(model)
    return InferencePolicy(model, dtype)


class RolloutBuffers:
    """Time-major trajectory storage for `horizon` steps of `n` envs."""

    def __init__(self, n: int, horizon: int, device):
        d = torch.device(device)
        T = horizon
        self.n, self.T, self.device = n, T, d
        self.boards = torch.zeros(T + 1, n, 16, dtype=torch.int8, device=d)  # boards[t] = state at step t
        self.flags = torch.zeros(T + 1, n, dtype=torch.uint8, device=d)      # flags[t] legal mask of boards[t]
        self.actions = torch.zeros(T, n, dtype=torch.uint8, device=d)
        self.logp = torch.zeros(T, n, 4, dtype=torch.float32, device=d)
        self.entropy = torch.zeros(T, n, dtype=torch.float32, device=d)
        self.value = torch.zeros(T, n, dtype=torch.float32, device=d)
        self.points = torch.zeros(T, n, dtype=torch.int32, device=d)
        self.max_tile = torch.zeros(T, n, dtype=torch.int8, device=d)
        self.pot = torch.zeros(T, n, 4, dtype=torch.int8, device=d)
        self.g_raw = torch.zeros(T, n, dtype=torch.float32, device=d)
        self.g_norm = torch.zeros(T, n, dtype=torch.float32, device=d)
        self.adv = torch.zeros(T, n, dtype=torch.float32, device=d)
        self.obs = torch.zeros(n, 48, dtype=torch.bfloat16, device=d)      # per-step scratch

    @property
    def step_flags(self) -> torch.Tensor:
        """flags written by step t (done / reset / invalid / next legal mask): [T, n]."""
        return self.flags[1:]

    def carry_over(self):
        """Start the next rollout from the last state (fixed-horizon mode)."""
        self.boards[0].copy_(self.boards[self.T])
        self.flags[0].copy_(self.flags[self.T])


class Rollout:
    """Fixed-horizon (auto-reset) or episodic (skip-done) rollouts of a VecEnv-like env state."""

    def __init__(self, n: int, horizon: int, device, seed: int = 0x2048, env_base: int = 0,
                 episodic: bool = False, obs_dtype=torch.bfloat16, mt_seeds=None):
        self.buf = RolloutBuffers(n, horizon, device)
        self.buf.obs = torch.zeros(n, 48, dtype=obs_dtype, device=self.buf.device)
        self.n, self.T = n, horizon
        self.seed, self.env_base = int(seed), int(env_base)
        self.episodic = episodic
        # Philox counter base lives on the device so a captured graph replays with fresh draws
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.buf.device)
        self.opts = L.OPT_SKIP_DONE if episodic else L.OPT_AUTO_RESET
        self._graph = None
        self.use_fused = True  # fused persistent policy rollout when the policy supports it
        # spawns: Philox by default; per-env CPython MT19937 streams when seeds are given, so game i
        # spawns exactly like the reference after random.seed(mt_seeds[i]) (train.py:227-228)
        self.mt_state = None
        if mt_seeds is not None:
            seeds = torch.as_tensor(list(mt_seeds), dtype=torch.int64).to(self.buf.device)
            self.mt_state = torch.zeros(625 * n, dtype=torch.int32, device=self.buf.device)
            L.mt_seed(self.mt_state, seeds)

    def _spawn_rng(self, offset: int) -> L.Rng:
        if self.mt_state is not None:
            return L.make_rng(L.RNG_MT19937, mt_state=self.mt_state)
        return L.make_rng(L.RNG_PHILOX, self.seed, offset, self.env_base, counter_dev=self.counter)

    def reset(self):
        b = self.buf
        L.env_reset(b.boards[0], b.flags[0], self._spawn_rng(0))
        self.counter.add_(1)

    def fused(self, policy) -> bool:
        """Whether steps run in the fused persistent kernel (FusedPolicy of a 2-block GameMLP whose
        weights fit LDS, Philox spawns) rather than one Rollout._step per step."""
        return self.use_fused and self.mt_state is None and getattr(policy, "fused_rollout", False)

    def steps(self, t0: int, t1: int, policy):
        """Steps t0 .. t1-1 (no counter bump): one fused launch, or the per-step path."""
        if self.fused(policy):
            policy.rollout_steps(self, t0, t1)
        else:
            for t in range(t0, t1):
                self._step(t, policy)

    def _step(self, t: int, policy):
        b = self.buf
        L.obs_encode(b.boards[t], b.obs)
        logits, value = policy(b.obs)
        b.value[t].copy_(value)
        # stream 1 draws of step t use counter base + 2t, env steps use base + 2t + 1: never reused
        rng = L.make_rng(L.RNG_PHILOX, self.seed, 2 * t, self.env_base, counter_dev=self.counter)
        L.sample_actions(logits.contiguous(), b.flags[t], b.actions[t], b.logp[t], b.entropy[t], rng)
        L.env_step(b.boards[t], b.boards[t + 1], b.actions[t], None, b.points[t], b.max_tile[t], b.pot[t],
                   b.flags[t + 1], self._spawn_rng(2 * t + 1), self.opts)

    def collect(self, policy, graph: bool = False):
        """Run T steps.  graph=True captures the T-step loop once and replays it afterwards."""
        if graph:
            if self._graph is None:
                self._graph = self._capture(policy)
            self._graph.replay()
        else:
            self.steps(0, self.T, policy)
            self.counter.add_(2 * self.T)
        return self.buf

    def _capture(self, policy):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        snap_b, snap_f, snap_c = self.buf.boards[0].clone(), self.buf.flags[0].clone(), self.counter.clone()
        snap_mt = self.mt_state.clone() if self.mt_state is not None else None
        with torch.cuda.stream(s):  # warm-up (allocator, library handles) outside the capture
            self.steps(0, self.T, policy)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            self.steps(0, self.T, policy)
            self.counter.add_(2 * self.T)
        # capture does not execute: restore the pre-warm-up state so replay #1 is the first rollout
        self.buf.boards[0].copy_(snap_b)
        self.buf.flags[0].copy_(snap_f)
        self.counter.copy_(snap_c)
        if snap_mt is not None:
            self.mt_state.copy_(snap_mt)
        return g
