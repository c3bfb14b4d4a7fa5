"""Optimizers and LR schedule of the trainer (train.py:1232-1281, :1587-1612).

Muon for the 2-D weights (`adjust_lr_fn="match_rms_adamw"`), AdamW for the 1-D LayerNorm / bias
parameters, both with the per-group learning rates of get_param_groups(critic_lr, lr) and the
same cosine-with-warmup schedule, stepped once per train step.  The schedule is the
transformers.get_scheduler("cosine") formula, restated so the trainer does not need transformers.
"""

from __future__ import annotations

import math

import torch


def cosine_with_warmup(num_warmup_steps: int, num_training_steps: int, num_cycles: float = 0.5):
    def f(step: int) -> float:
        if step < num_warmup_steps:
            return float(step) / float(max(1, num_warmup_steps))
        progress = float(step - num_warmup_steps) / float(max(1, num_training_steps - num_warmup_steps))
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))
    return f


class MultiOptimizer:
    """(optimizer, scheduler) pairs behind one step/zero_grad/scheduler_step interface (train.py:1232)."""

    def __init__(self, *pairs):
        self.optimizers, self.schedulers = [], []
        for item in pairs:
            opt, sched = item if isinstance(item, tuple) else (item, None)
            self.optimizers.append(opt)
            self.schedulers.append(sched)

    def step(self):
        for opt in self.optimizers:
            opt.step()

    def zero_grad(self, set_to_none: bool = True):
        for opt in self.optimizers:
            opt.zero_grad(set_to_none=set_to_none)

    def scheduler_step(self, *args, **kwargs):
        for s in self.schedulers:
            if s is not None:
                s.step(*args, **kwargs)

    def get_lr(self):
        return [opt.param_groups[0]["lr"] for opt in self.optimizers]

    def state_dict(self):
        return {"optimizers": [o.state_dict() for o in self.optimizers],
                "schedulers": [s.state_dict() if s else None for s in self.schedulers]}

    def load_state_dict(self, sd):
        for o, s in zip(self.optimizers, sd["optimizers"]):
            o.load_state_dict(s)
        for sc, s in zip(self.schedulers, sd["schedulers"]):
            if sc and s:
                sc.load_state_dict(s)


def build_optimizer(model, lr: float, critic_lr: float, beta1: float = 0.9, beta2: float = 0.999,
                    weight_decay: float = 0.01, warmup_steps: int = 200, total_steps: int = 1000,
                    schedule: bool = True) -> MultiOptimizer:
    """train.py:1587-1612."""
    o2d, o1d, v2d, v1d = model.get_param_groups(critic_lr, lr)
    adamw = torch.optim.AdamW([o1d, v1d], betas=(beta1, beta2), weight_decay=weight_decay)
    muon = torch.optim.Muon([o2d, v2d], adjust_lr_fn="match_rms_adamw", weight_decay=weight_decay)
    if not schedule:
        return MultiOptimizer(muon, adamw)
    lam = cosine_with_warmup(warmup_steps, total_steps)
    return MultiOptimizer((muon, torch.optim.lr_scheduler.LambdaLR(muon, lam)),
                          (adamw, torch.optim.lr_scheduler.LambdaLR(adamw, lam)))
