"""The PPO minibatch step of GameURM with its loss on device kernels (model_optimize_step,
train.py:414-642, for the reference's GameURM, game.py:1355-1458).

PPOUpdater runs the loss as a torch expression (ppo.ppo_losses: ~25 kernels forward, as many in its
autograd backward, plus the heads' cast / pad / copy kernels and ~20 for the KL diagnostic and the
statistics).  URMPPOUpdater keeps the model's own device Functions for the transformer (agent.GameURM
.features: stem, loops, token mean) and replaces everything after the pooled features:

    obs        g2048_obs_gather (boards[idx] -> bf16 features; autocast's stem operand)
    loss       URMHeadLossFn: heads + PPO-clip / entropy / smooth-L1 + dz + masked logits + sums in
               ONE launch (g2048_urm_head_loss); its backward dpooled and the head gradients in one
               more (g2048_urm_head_loss_bwd)
    backward   the model's Functions, every shared weight's gradient added straight into its .grad
               (urm.direct_weight_grads: no autograd accumulation kernels)
    step       [RCCL all-reduce] the fused clip + Muon/AdamW launch (step_clipped) when available
    KL         the one-launch training-mode re-forward (urm.train_nograd_forward), then KL(old || new)
               and the statistics update in one launch (g2048_urm_kl_stats)

Same math as PPOUpdater (tests/test_gpu_urm.py compares the two); the rounding points of the heads
are autocast's (bf16 operands, one bf16 rounding of the biased fp32 sum), the summation orders are
the kernels' fixed ones.
"""

from __future__ import annotations

import torch

from . import _lib as L
from . import urm as U
from .ppo import PPOUpdater


class URMHeadLossFn(torch.autograd.Function):
    """loss = -mean(ppo - critic v + beta H) of one minibatch from GameURM's pooled features
    [m, h] through its action / value heads (game.py:1452-1456) -- g2048_urm_head_loss forward,
    g2048_urm_head_loss_bwd backward.  `run` carries the batch columns and the outputs the update
    reads afterwards (masked logits, loss sums).  Head gradients go straight into the parameters'
    .grad under urm.direct_weight_grads, else they are returned."""

    @staticmethod
    def forward(ctx, pooled: torch.Tensor, wa, ba, wv, bv, run: dict):
        pooled = pooled.contiguous()
        m, h = pooled.shape
        dev = pooled.device
        dz = torch.empty(m, 8, dtype=torch.float32, device=dev)
        masked = torch.empty(m, 4, dtype=torch.float32, device=dev)
        sums = torch.empty(3, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        part = torch.empty(L.urm_head_loss_partials(m, h), dtype=torch.float32, device=dev)
        L.urm_head_loss(pooled, wa.detach(), ba.detach(), wv.detach(), bv.detach(), run["batch"], run["beta"],
                        run["critic"], run["clip"], dz, masked, part, run["sync"], sums, loss)
        run["masked"], run["sums"] = masked, sums
        ctx.save_for_backward(pooled, dz)
        ctx.params = (wa, ba, wv, bv)
        ctx.direct = U._DIRECT[0]
        ctx.sync = run["sync"]
        return loss

    @staticmethod
    def backward(ctx, gout: torch.Tensor):
        pooled, dz = ctx.saved_tensors
        wa, ba, wv, bv = ctx.params
        m, h = pooled.shape
        dp = torch.empty_like(pooled)
        part = torch.empty(L.urm_head_loss_partials(m, h), dtype=torch.float32, device=pooled.device)
        sinks = [U._grad_sink(p if ctx.direct else None, p.shape) for p in (wa, ba, wv, bv)]
        acc = all(s is not None for s in sinks)
        outs = sinks if acc else [torch.empty(p.shape, dtype=torch.float32, device=pooled.device) for p in (wa, ba, wv, bv)]
        go = gout.detach().float().reshape(1).contiguous()
        L.urm_head_loss_bwd(pooled, wa.detach(), wv.detach(), dz, go, dp, part, ctx.sync, outs[0], outs[1], outs[2],
                            outs[3], accumulate=acc)
        if acc:
            return dp, None, None, None, None, None
        return (dp,) + tuple(o.to(p.dtype) for o, p in zip(outs, (wa, ba, wv, bv))) + (None,)


def supports(model, amp_dtype) -> bool:
    """URMPPOUpdater applies: a GameURM under bf16 autocast whose heads and pooled width the loss
    kernels cover (h 64 or 32, biased heads, coupled critic)."""
    try:
        import agent
    except ImportError:  # pragma: no cover
        return False
    if not isinstance(model, agent.GameURM) or amp_dtype != torch.bfloat16:
        return False
    h = model.config.hidden_dim
    return (h in (32, 64) and model.action_head.bias is not None and model.value_head.bias is not None
            and L.urm_head_loss_partials(1, h) > 0)


class URMPPOUpdater(PPOUpdater):
    """PPOUpdater for GameURM on the device loss kernels (module docstring); graph capture, the RCCL
    all-reduce split and the ragged last minibatch behave as in PPOUpdater."""

    def __init__(self, model, optimizer, cfg, grads, generator=None, graph: bool = False):
        super().__init__(model, optimizer, cfg, grads, generator, graph)
        self.sync = torch.zeros(1, dtype=torch.int32, device=self.dev)  # the loss kernels' ticket word

    def _gather(self, boards: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        """bf16 features of boards[idx] (g2048_obs_gather: autocast's operand of the stem)."""
        n = idx.shape[0]
        obs = torch.empty(n, 48, dtype=torch.bfloat16, device=self.dev)
        L.obs_gather(boards, idx, obs)
        return obs

    def _pre(self, idx, data, beta, encode):
        cfg = self.cfg
        obs = self._gather(data["boards"], idx)
        run = {"batch": L.make_ppo_batch(idx, data["actions"], data["legal"], data["logp"], data["adv"], data["ret"]),
               "beta": beta if torch.is_tensor(beta) else torch.tensor(float(beta), device=self.dev),
               "critic": cfg.critic, "clip": cfg.clip_eps, "sync": self.sync, "idx": idx}
        m = self.model
        with torch.autocast("cuda", dtype=cfg.amp_dtype, cache_enabled=not self.graph), U.direct_weight_grads():
            pooled = m.features(obs)
            loss = URMHeadLossFn.apply(pooled, m.action_head.weight, m.action_head.bias, m.value_head.weight,
                                       m.value_head.bias, run)
        self.grads.zero()
        if getattr(self, "_one", None) is None or self._one.device != loss.device:
            self._one = torch.ones((), dtype=torch.float32, device=self.dev)  # (no ones_like + fill per minibatch)
        with U.direct_weight_grads():
            loss.backward(self._one)
        return {"obs": obs, "masked": run["masked"], "sums": run["sums"], "beta": run["beta"]}

    def _post(self, st, beta):
        cfg = self.cfg
        if getattr(self.opt, "fused", False):
            gn = self.opt.step_clipped(self.grads.flat, cfg.max_grad_norm)
        else:
            gn = self.grads.clip_(cfg.max_grad_norm)
            self.opt.step()
        with torch.no_grad():
            new_logits, _ = self._forward(st["obs"])
            m = new_logits.shape[0]
            part = torch.empty(2 * ((m + 255) // 256), dtype=torch.float32, device=self.dev)
            L.urm_kl_stats(st["masked"], new_logits.contiguous(), st["sums"], gn.reshape(()).float(), st["beta"],
                           cfg.critic, self.stats, part, self.sync)
