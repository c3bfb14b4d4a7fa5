"""Reward / return-to-go / advantage on the device (calculate_advantage, train.py:651-904).

The reverse discounted scan, the normalisation with the PREVIOUS bias-corrected moments and the
advantage run in one HIP kernel over the time-major [T, N] trajectory (float64 arithmetic); the
batch statistics come back as three float64 sums, which is all a multi-GPU run has to all-reduce
(24 bytes per train step) before the EMA moment update.  No host synchronisation.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib as L


@dataclass
class RewardWeights:
    """The live reward terms of train.py:702-719 (the other shaping flags never reach the reward)."""
    gamma: float = 0.99
    points: float = 0.0
    mono: float = 0.0
    emptiness: float = 0.0
    rtg_beta: float = 0.9

    def cfg(self) -> L.RewardCfg:
        return L.RewardCfg(self.gamma, self.points, self.mono, self.emptiness, self.rtg_beta)


class RTGTracker:
    """Holds the RTG moment state (train.py:1550-1552: mu=0, m2=1) on the device and runs the scan."""

    def __init__(self, n: int, device, weights: RewardWeights, allreduce=None):
        self.device = torch.device(device)
        self.w = weights
        self.state = torch.tensor([0.0, 1.0, 0.0, 1.0, 0.0, 1.0, 0.0, 0.0], dtype=torch.float64, device=self.device)
        self.partials = torch.zeros(3, dtype=torch.float64, device=self.device)
        self.workspace = torch.zeros(L.rtg_workspace_bytes(n), dtype=torch.uint8, device=self.device)
        self.allreduce = allreduce  # callable(tensor) summing in place across ranks, or None

    def set_moments(self, mu: float, m2: float, first_moment: float, step: int):
        self.state[0], self.state[1], self.state[2], self.state[3] = mu, m2, first_moment, float(step)

    def moments(self) -> dict:
        s = self.state.tolist()
        return {"rtg_mu": s[0], "rtg_m2": s[1], "rtg_first_moment": s[2], "rtg_step": int(s[3]),
                "mu_corrected": s[4], "std": s[5], "batch_mean": s[6], "batch_var": s[7]}

    def compute(self, points, pot, step_flags, value, g_raw, g_norm, adv):
        """[T, N] trajectory -> g_raw, g_norm, adv (in place); updates the moments."""
        cfg = self.w.cfg()
        L.rtg_prepare(self.state, cfg)
        L.reward_rtg(points, pot, step_flags, value, self.state, g_raw, g_norm, adv, self.partials,
                     self.workspace, cfg)
        if self.allreduce is not None:
            self.allreduce(self.partials)
        L.rtg_finalize(self.state, self.partials, cfg)
