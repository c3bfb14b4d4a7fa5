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


class MuonAdamW:
    """Graph-capturable Muon (2-D weights) + AdamW (1-D) with the reference's parameter groups.

    Same arithmetic as torch.optim.Muon(adjust_lr_fn="match_rms_adamw", nesterov) and
    torch.optim.AdamW, but learning rates and the Adam step count live in device tensors, so one
    optimizer step contains no host scalars and can sit inside a captured hipGraph; the LR schedule
    is applied with set_lr_scale() between replays.  The 1-D parameters (LayerNorm, biases) are
    re-homed into one flat buffer per group, so AdamW is a handful of kernels on two flat vectors.
    """

    def __init__(self, model, lr: float, critic_lr: float, beta1=0.9, beta2=0.999, weight_decay=0.01,
                 momentum=0.95, nesterov=True, ns_coefficients=(3.4445, -4.775, 2.0315), ns_steps=5,
                 ns_eps=1e-7, adam_eps=1e-8):
        o2d, o1d, v2d, v1d = model.get_param_groups(critic_lr, lr)
        dev = next(model.parameters()).device
        self.dev = dev
        self.base = [o2d["lr"], o1d["lr"], v2d["lr"], v1d["lr"]]
        self.lr = torch.tensor(self.base, dtype=torch.float32, device=dev)
        self.wd, self.b1, self.b2, self.eps = weight_decay, beta1, beta2, adam_eps
        self.momentum, self.nesterov = momentum, nesterov
        self.ns, self.ns_steps, self.ns_eps = ns_coefficients, ns_steps, ns_eps
        self.muon = [(p, 0) for p in o2d["params"]] + [(p, 2) for p in v2d["params"]]
        self.muon_buf = [torch.zeros_like(p) for p, _ in self.muon]
        self.adam_groups = []
        for gi, grp in ((1, o1d), (3, v1d)):
            ps = list(grp["params"])
            if not ps:
                continue
            flat = torch.cat([p.detach().reshape(-1) for p in ps]).contiguous()
            off = 0
            for p in ps:
                n = p.numel()
                p.data = flat[off:off + n].view_as(p)
                off += n
            self.adam_groups.append({"idx": gi, "params": ps, "flat": flat, "m": torch.zeros_like(flat),
                                     "v": torch.zeros_like(flat)})
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.scale = 1.0

    def set_lr_scale(self, s: float):
        self.scale = s
        self.lr.copy_(torch.tensor([b * s for b in self.base], dtype=torch.float32))

    def get_lr(self):
        return [b * self.scale for b in self.base]

    @staticmethod
    def _flat_grad(group):
        ps = group["params"]
        base = ps[0].grad
        # grads of a group are contiguous views when the GradBucket was built in the same order
        if all(p.grad is not None for p in ps):
            start = base.data_ptr()
            total = sum(p.numel() for p in ps)
            if all(p.grad.data_ptr() == start + 4 * sum(q.numel() for q in ps[:k]) for k, p in enumerate(ps)):
                return base.reshape(-1).as_strided((total,), (1,))
        return torch.cat([p.grad.reshape(-1) for p in ps])

    def _newton_schulz(self, g):
        a, b, c = self.ns
        x = g.bfloat16()
        tr = g.size(0) > g.size(1)
        if tr:
            x = x.T
        x = x / x.norm().clamp(min=self.ns_eps)
        for _ in range(self.ns_steps):
            gram = x @ x.T
            upd = torch.addmm(gram, gram, gram, beta=b, alpha=c)
            x = torch.addmm(x, upd, x, beta=a)
        if tr:
            x = x.T
        return x

    @torch.no_grad()
    def step(self):
        # Muon (torch/optim/_muon.py semantics)
        for (p, gi), buf in zip(self.muon, self.muon_buf):
            g = p.grad
            buf.lerp_(g, 1 - self.momentum)
            upd = g.lerp(buf, self.momentum) if self.nesterov else buf
            upd = self._newton_schulz(upd)
            lr = self.lr[gi]
            A, B = p.shape[:2]
            p.mul_(1 - lr * self.wd)
            p.sub_(upd.to(p.dtype) * (lr * (0.2 * math.sqrt(max(A, B)))))
        # AdamW (torch/optim/adamw.py semantics, decoupled weight decay)
        self.step_t.add_(1)
        bc1 = 1 - self.b1 ** self.step_t
        bc2_sqrt = (1 - self.b2 ** self.step_t).sqrt()
        for grp in self.adam_groups:
            lr = self.lr[grp["idx"]]
            flat, m, v = grp["flat"], grp["m"], grp["v"]
            g = self._flat_grad(grp)
            flat.mul_(1 - lr * self.wd)
            m.lerp_(g, 1 - self.b1)
            v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            denom = (v.sqrt() / bc2_sqrt).add_(self.eps)
            flat.sub_((lr / bc1) * m / denom)

    def zero_grad(self, set_to_none: bool = False):
        pass  # gradients live in the trainer's GradBucket, zeroed there

    def state_dict(self):
        return {"lr": self.lr.cpu(), "step": self.step_t.cpu(), "muon_buf": [b.cpu() for b in self.muon_buf],
                "adam": [{"m": g["m"].cpu(), "v": g["v"].cpu()} for g in self.adam_groups], "scale": self.scale}

    def snapshot(self):
        return ([b.clone() for b in self.muon_buf], [(g["m"].clone(), g["v"].clone()) for g in self.adam_groups],
                self.step_t.clone())

    def restore(self, snap):
        bufs, adam, st = snap
        for b, s in zip(self.muon_buf, bufs):
            b.copy_(s)
        for g, (m, v) in zip(self.adam_groups, adam):
            g["m"].copy_(m)
            g["v"].copy_(v)
        self.step_t.copy_(st)


class FusedMuonAdamW(MuonAdamW):
    """MuonAdamW with its step as two kernels (include/g2048_ppo.h, csrc/optim.hip): the partial sums
    of squares of the gradient (the clip coefficient), then every Muon matrix in one launch, one
    block each (momentum, Newton-Schulz on bf16 MFMA in LDS, weight decay, scaled update, bf16
    weight copy) with the AdamW update of the 1-D groups in the same launch's extra blocks.

    Same arithmetic as MuonAdamW up to the accumulation order of the bf16 Newton-Schulz products.
    `supported` is False when a matrix does not fit the one-block Newton-Schulz kernel (h > 196) or
    the model has more than 16 Muon matrices; callers then use MuonAdamW.  Serves GameMLP (5 matrices)
    and GameURM (11, incl. the [64, 3] stem: per-element momentum / update pass).
    """

    def __init__(self, model, *args, **kwargs):
        super().__init__(model, *args, **kwargs)
        from . import _lib as L
        self._L = L
        self.supported = (self.dev.type == "cuda" and 0 < len(self.muon) <= 16 and len(self.adam_groups) <= 4
                          and all(p.ndim == 2 and L.muon_supported(*p.shape) for p, _ in self.muon))
        self.norm_t = torch.zeros((), dtype=torch.float32, device=self.dev)
        self.coef_t = torch.ones((), dtype=torch.float32, device=self.dev)
        self.norm_part = torch.zeros(64, dtype=torch.float32, device=self.dev)
        self._bf16 = {}
        self._mats = self._groups = None
        self._cfg = L.MuonCfg(self.momentum, self.wd, self.ns[0], self.ns[1], self.ns[2], self.ns_eps, self.ns_steps,
                              int(self.nesterov))
        # the h 196 / 192 square matrices' Newton-Schulz on MUON_PARTS CUs each (row blocks, one
        # exchange of X per iteration through this workspace); G2048_MUON_PARTS=1: one CU per matrix
        if self.supported:
            import os
            parts = int(os.environ.get("G2048_MUON_PARTS", self.MUON_PARTS))
            if parts > 1:
                self._ws = torch.zeros(int(L.load().g2048_muon_workspace_bytes()), dtype=torch.uint8, device=self.dev)
                self._cfg.parts = parts
                self._cfg.workspace = self._ws.data_ptr()

    MUON_PARTS = 13

    def error_count(self):
        """Device int32 [1] view of the Muon workspace's sticky count of timed-out hand-off waits (a
        multi-CU Newton-Schulz part that never became resident: that step's weights are garbage), or
        None without a multi-CU workspace.  Read with the train step's one host sync."""
        ws = getattr(self, "_ws", None)
        if ws is None:
            return None
        off = int(self._L.load().g2048_muon_error_offset())
        return ws[off:off + 4].view(torch.int32)

    def check_errors(self, count: float | int | None = None):
        """Raise when a multi-CU Muon step timed out (count: the value already read by the caller)."""
        if count is None:
            t = self.error_count()
            count = 0 if t is None else int(t.item())
        if count:
            raise RuntimeError(f"fused Muon: {int(count)} multi-CU Newton-Schulz hand-off wait(s) timed out (a part "
                               f"was not resident); the optimizer state is invalid")

    def set_bf16_copies(self, mapping: dict):
        """{parameter: bf16 tensor} refreshed by the Muon kernel after each step."""
        self._bf16 = {id(p): t for p, t in mapping.items()}
        self._mats = None

    def set_head_frag(self, frag, rows: dict) -> bool:
        """frag: g2048_head_split's fragment image; rows {head weight parameter: its first head row}
        (action head 0, value head 4).  The Muon kernel then writes those matrices' three-term bf16
        split with each step (no g2048_head_split launch after it).  False when a head is not a
        Muon matrix of this optimizer (the caller keeps splitting)."""
        ids = {id(p) for p, _ in self.muon}
        if not all(id(p) in ids for p in rows):
            return False
        self._frag = (frag, {id(p): r for p, r in rows.items()})
        self._mats = None
        return True

    def _build(self):
        L = self._L
        mats = (L.MuonMatrix * len(self.muon))()
        for k, ((p, gi), buf) in enumerate(zip(self.muon, self.muon_buf)):
            if p.grad is None or not p.grad.is_contiguous():
                raise RuntimeError("FusedMuonAdamW needs contiguous gradients (a GradBucket)")
            bf = self._bf16.get(id(p))
            frag, frow = getattr(self, "_frag", (None, {}))
            fr = frow.get(id(p))
            mats[k] = L.MuonMatrix(p.data_ptr(), p.grad.data_ptr(), buf.data_ptr(), bf.data_ptr() if bf is not None else None,
                                   frag.data_ptr() if fr is not None else None, p.shape[0], p.shape[1], gi,
                                   fr if fr is not None else 0)
        groups = (L.AdamWGroup * len(self.adam_groups))()
        for k, grp in enumerate(self.adam_groups):
            g = self._flat_grad(grp)
            if g.data_ptr() != grp["params"][0].grad.data_ptr():
                raise RuntimeError("FusedMuonAdamW needs each AdamW group's gradients contiguous in the bucket")
            groups[k] = L.AdamWGroup(grp["flat"].data_ptr(), g.data_ptr(), grp["m"].data_ptr(), grp["v"].data_ptr(),
                                     grp["flat"].numel(), grp["idx"], 0)
        self._mats, self._groups = mats, groups

    def _run(self, clip, max_norm=None):
        if self._mats is None:
            self._build()
        L = self._L
        if max_norm is None:
            L.muon_step(self._mats, self.lr, clip, self._cfg, self.lr)
        else:  # the clip coefficient is computed inside the Muon launch from the grad_sumsq partials
            L.muon_step_clip(self._mats, self.lr, self.norm_part, max_norm, self.norm_t, self.coef_t, self._cfg)
        self.step_t.add_(1)
        if len(self._groups):
            L.adamw_step(self._groups, self.lr, self.step_t, clip, self.b1, self.b2, self.eps, self.wd)

    @torch.no_grad()
    def step(self):
        if not self.supported:
            return super().step()
        self._run(None)

    @torch.no_grad()
    def step_clipped(self, flat_grad: torch.Tensor, max_norm: float, sq: torch.Tensor | None = None) -> torch.Tensor:
        """clip_grad_norm_(max_norm) folded into the step (the bucket itself is left unclipped);
        returns the pre-clip norm as a device scalar.  sq: the gradient's sum-of-squares partials
        already written (g2048_colsum_batch_sq, which also counted the step) -- then one launch."""
        if self._mats is None:
            self._build()
        # two launches: partial sums of squares (+ the step count), then Muon with the clip folded in
        # and the AdamW blocks of the 1-D groups
        if sq is None:
            self._L.grad_sumsq_tick(flat_grad, self.norm_part, self.step_t)
            part, self._cfg.npartials = self.norm_part, 0
        else:
            part, self._cfg.npartials = sq, sq.numel()
        self._L.muon_adamw_step_clip(self._mats, self._groups if len(self._groups) else None, self.lr, self.step_t,
                                     part, max_norm, self.norm_t, self.coef_t, self._cfg, self.b1, self.b2,
                                     self.eps, self.wd)
        return self.norm_t


class ScheduledMuonAdamW:
    """MuonAdamW + the cosine-with-warmup schedule stepped once per train step (train.py:1598-1612, :625)."""

    def __init__(self, opt: MuonAdamW, warmup: int, total: int):
        self.opt = opt
        self.fn = cosine_with_warmup(warmup, total)
        self.t = 0
        self.opt.set_lr_scale(self.fn(0))
        self.optimizers = [self]

    @property
    def param_groups(self):
        return [{"lr": lr} for lr in self.opt.get_lr()]

    def step(self):
        self.opt.step()

    @property
    def fused(self) -> bool:
        return getattr(self.opt, "supported", False)

    def step_clipped(self, flat_grad, max_norm, sq=None):
        return self.opt.step_clipped(flat_grad, max_norm, sq=sq)

    def set_bf16_copies(self, mapping):
        self.opt.set_bf16_copies(mapping)

    def set_head_frag(self, frag, rows):
        return self.opt.set_head_frag(frag, rows)

    def zero_grad(self, set_to_none: bool = False):
        pass

    def scheduler_step(self):
        self.t += 1
        self.opt.set_lr_scale(self.fn(self.t))

    def snapshot(self):
        return self.opt.snapshot()

    def restore(self, snap):
        self.opt.restore(snap)

    def state_dict(self):
        return {"opt": self.opt.state_dict(), "t": self.t}
