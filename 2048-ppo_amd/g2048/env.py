"""VecEnv: N independent 2048 boards resident in HBM, stepped by libg2048's HIP kernels.

Replaces the per-game `Game2048` object of the reference (game.py:45-1030) for the rollout: one
[N,16] int8 board tensor instead of N Python list-of-lists, one kernel launch per step for all
envs instead of a Python call per env.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib as L


@dataclass
class StepOut:
    """Per-env outputs of one vectorised step (views into VecEnv-owned or caller buffers)."""
    boards: torch.Tensor    # [N,16] int8 board after the step (after auto-reset if any)
    actions: torch.Tensor   # [N] uint8 action taken
    points: torch.Tensor    # [N] int32 merge points (game.py:237)
    max_tile: torch.Tensor  # [N] int8 max tile exponent created
    pot: torch.Tensor       # [N,4] int8 {mono_b, mono_a, empt_b, empt_a}
    flags: torch.Tensor     # [N] uint8, see include/g2048.h


class VecEnv:
    """`n` boards on `device`.

    rng="philox": stateless Philox4x32-10 keyed by `seed`, counter = the env's step count (the
    fast mode).  rng="mt19937": one CPython random.Random stream per env seeded with seeds[i]
    (bit-exact with game.py's spawns when the reference is seeded the same way).
    """

    def __init__(self, n: int, device="cuda", rng: str = "philox", seed: int = 0x2048, seeds=None,
                 env_base: int = 0):
        if n <= 0:
            raise ValueError("n must be positive")
        self.n = n
        self.device = torch.device(device)
        self.seed = int(seed)
        self.env_base = int(env_base)
        self.counter = 0
        self.mode = {"philox": L.RNG_PHILOX, "mt19937": L.RNG_MT19937, "inject": L.RNG_INJECT}[rng]
        self.boards = torch.zeros(n, 16, dtype=torch.int8, device=self.device)
        self.flags = torch.zeros(n, dtype=torch.uint8, device=self.device)
        self.mt_state = None
        if self.mode == L.RNG_MT19937:
            if seeds is None:
                seeds = torch.arange(n, dtype=torch.int64) + self.seed
            seeds = torch.as_tensor(seeds, dtype=torch.int64).to(self.device)
            self.mt_state = torch.zeros(625 * n, dtype=torch.int32, device=self.device)
            L.mt_seed(self.mt_state, seeds)
        self._alloc_out()

    def _alloc_out(self):
        d, n = self.device, self.n
        self.out = StepOut(self.boards, torch.zeros(n, dtype=torch.uint8, device=d),
                           torch.zeros(n, dtype=torch.int32, device=d), torch.zeros(n, dtype=torch.int8, device=d),
                           torch.zeros(n, 4, dtype=torch.int8, device=d), self.flags)

    def rng(self, inject: torch.Tensor | None = None, counter_dev=None) -> L.Rng:
        return L.make_rng(self.mode, self.seed, self.counter, self.env_base, counter_dev=counter_dev,
                          mt_state=self.mt_state, inject=inject)

    def reset(self, where: torch.Tensor | None = None, inject: torch.Tensor | None = None) -> torch.Tensor:
        L.env_reset(self.boards, self.flags, self.rng(inject), where)
        self.counter += 1
        return self.boards

    def legal(self) -> torch.Tensor:
        L.legal_mask(self.boards, self.flags)
        return self.flags

    def step(self, actions: torch.Tensor | None = None, auto_reset: bool = False, skip_done: bool = False,
             out: StepOut | None = None, boards_out: torch.Tensor | None = None,
             inject: torch.Tensor | None = None) -> StepOut:
        """One step of every env.  actions=None -> uniform random legal actions (Philox stream 1)."""
        o = out or self.out
        dst = boards_out if boards_out is not None else self.boards
        opts = (L.OPT_AUTO_RESET if auto_reset else 0) | (L.OPT_SKIP_DONE if skip_done else 0)
        if actions is not None and actions.dtype != torch.uint8:
            actions = actions.to(torch.uint8)
        L.env_step(self.boards, dst, actions, o.actions, o.points, o.max_tile, o.pot, o.flags, self.rng(inject), opts)
        self.counter += 1
        if dst is not self.boards:
            self.boards.copy_(dst)
        return StepOut(dst, o.actions, o.points, o.max_tile, o.pot, o.flags)

    def obs(self, dtype=torch.float32, out: torch.Tensor | None = None) -> torch.Tensor:
        o = out if out is not None else torch.empty(self.n, 48, dtype=dtype, device=self.device)
        L.obs_encode(self.boards, o)
        return o
