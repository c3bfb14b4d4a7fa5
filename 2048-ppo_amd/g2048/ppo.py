"""PPO-clip policy-gradient update (model_optimize_step, train.py:414-642), tensor-native.

Per minibatch (same math as the reference):
  masked = logits.masked_fill(invalid, -inf);  logpi = log_softmax(masked)            :497-515
  rho = exp(clamp(logpi(a) - logpi_old(a), -20, 20));  ppo = min(A rho, A clip(rho, 0.8, 1.2)) :517-523
  H = -sum_valid softmax(clamp(masked, -20, 20)) * log_softmax(...)                  :531-535
  v = smooth_l1(V, G_norm)                                                           :544-546
  loss = -mean(ppo - c v + beta H);  backward;  [all-reduce];  clip 1.0;  Muon+AdamW  :553-568
  KL(old || new) diagnostic on a no-grad re-forward (train mode, as in the reference) :578-601
Differences by design: minibatches are gathered on the device from the flat [T*N] trajectory with
a device permutation (no DataLoader, no per-sample Python), statistics stay on the device (one
host sync per train step), and the forward runs under bf16 autocast on MI355X.  For the
reference's GameMLP the trainer uses fastmlp.FusedPPOUpdater instead: the same step written out
as MFMA / fused kernels.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .dist import graph as graph_capture

STAT_KEYS = ("loss", "policy_loss", "entropy_loss", "value_loss", "grad_norm", "entropy", "kl_total", "kl_average",
             "kl_max")


@dataclass
class PPOConfig:
    batch_size: int = 65536
    epochs: int = 1
    clip_eps: float = 0.2
    critic: float = 1.0          # --critic (critic_strength)
    max_grad_norm: float = 1.0
    amp_dtype: torch.dtype | None = torch.bfloat16


def invalid_from_legal(legal: torch.Tensor) -> torch.Tensor:
    """uint8 legal mask (bit a = action a legal) -> bool [B,4] invalid mask (train.py:268)."""
    bits = torch.arange(4, device=legal.device, dtype=torch.int32)
    return ((legal.to(torch.int32).unsqueeze(-1) >> bits) & 1) == 0


def ppo_losses(logits, value, actions, invalid, old_logp, adv, ret, beta, critic, clip_eps=0.2):
    """Returns (loss, parts) for one minibatch; logits/value float32."""
    masked = logits.masked_fill(invalid, float("-inf"))
    new_lp_all = masked.log_softmax(dim=-1)
    a = actions.long().unsqueeze(1)
    new_lp = new_lp_all.gather(1, a).squeeze(1)
    old_lp = old_logp.gather(1, a).squeeze(1)
    ratio = (new_lp - old_lp).clamp(-20, 20).exp()
    ppo = torch.minimum(adv * ratio, adv * ratio.clamp(1 - clip_eps, 1 + clip_eps))
    lp2 = masked.clamp(-20, 20).log_softmax(dim=-1)
    ent = -(lp2 * lp2.exp()).masked_fill(invalid, 0.0).sum(dim=-1)
    v = value.reshape(-1)
    vloss = F.smooth_l1_loss(v, ret, reduction="none")
    loss = -(ppo - critic * vloss + beta * ent).mean()
    return loss, {"ppo": ppo, "entropy": ent, "vloss": vloss, "masked": masked}


def kl_old_new(old_masked_logits, new_logits, invalid):
    """torch.masked KL(old || new) over valid actions (train.py:594-601)."""
    new_masked = new_logits.masked_fill(invalid, float("-inf"))
    lo = old_masked_logits.log_softmax(dim=-1)
    ln = new_masked.log_softmax(dim=-1)
    term = lo.exp() * (lo - ln)
    return term.masked_fill(invalid, 0.0).sum(dim=-1)


class PPOUpdater:
    """Minibatch PPO over a flat trajectory.  `grads` is a dist.GradBucket (flat .grad views).

    graph=True (device tensors, graph-safe optimizer such as optim.MuonAdamW): the whole minibatch
    step -- gather, encode, forward, loss, backward, clip, optimizer, KL diagnostic, statistics --
    is captured once into a hipGraph and replayed per minibatch with a new index vector; the RCCL
    gradient all-reduce is captured with it (gloo: the step is split into two graphs around an eager
    host-staged all-reduce).
    """

    def __init__(self, model, optimizer, cfg: PPOConfig, grads, generator: torch.Generator | None = None,
                 graph: bool = False):
        self.model, self.opt, self.cfg, self.grads = model, optimizer, cfg, grads
        self.gen = generator
        self.dev = next(model.parameters()).device
        self.stats = torch.zeros(len(STAT_KEYS), dtype=torch.float32, device=self.dev)
        self.graph = graph and self.dev.type == "cuda"
        self.beta_t = torch.zeros((), dtype=torch.float32, device=self.dev)
        self._g = None
        self.weight_cache = None  # urm.Bf16Weights (refreshed at every update and after a capture)

    ragged_pad = False  # True: the updater runs a ragged minibatch padded to full size (_set_rows)

    def _set_rows(self, n: int):
        raise NotImplementedError

    def _forward(self, obs):
        if self.cfg.amp_dtype is not None and obs.is_cuda:
            with torch.autocast("cuda", dtype=self.cfg.amp_dtype, cache_enabled=not self.graph):
                logits, value = self.model(obs)
        else:
            logits, value = self.model(obs)
        return logits.float(), value.float()

    def update(self, data: dict, beta: float, encode) -> dict:
        """data: flat tensors boards [M,16] int8, actions [M], legal [M] uint8, logp [M,4], adv [M], ret [M].
        `encode(boards) -> obs [B,48]` builds the model input of a gathered minibatch."""
        cfg = self.cfg
        m_total = data["actions"].shape[0]
        bs = min(cfg.batch_size, m_total)
        self.stats.zero_()
        self.beta_t.fill_(beta)
        nb = 0
        self.model.train()
        if self.weight_cache is not None:
            self.weight_cache.refresh()
        use_graph = self.graph and (m_total % bs == 0 or self.ragged_pad)
        if use_graph:
            self._ensure_graph(data, bs, encode)
        for _ in range(cfg.epochs):
            perm = self._epoch_perm(m_total)
            for s in range(0, m_total, bs):
                idx = perm[s:s + bs]
                n = idx.shape[0]
                if n < bs and self.ragged_pad:  # DataLoader's ragged last batch (drop_last=False), padded
                    idx = torch.cat([idx, idx.new_zeros(bs - n)])
                    self._set_rows(n)
                if use_graph:
                    self._replay(idx)
                else:
                    self._minibatch(idx, data, self.beta_t, encode)
                if n < bs and self.ragged_pad:
                    self._set_rows(bs)
                nb += 1
        st = self.stats / max(nb, 1)
        st[STAT_KEYS.index("kl_max")] = self.stats[STAT_KEYS.index("kl_max")]
        return {k: st[i] for i, k in enumerate(STAT_KEYS)}

    def _epoch_perm(self, m_total: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """The epoch's minibatch order (DataLoader(shuffle=True), train.py:470).  On the device:
        g2048_permutation keyed by one int64 drawn from the update's generator (no host read; one
        launch instead of torch.randperm's radix sort of m_total keys); `out` (optional) receives it."""
        if self.dev.type != "cuda":  # the CPU (gloo) updater of the host tests
            perm = torch.randperm(m_total, device=self.dev, generator=self.gen)
            return perm if out is None else out[:m_total].copy_(perm)
        from . import _lib as L
        key = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=self.dev, generator=self.gen)
        if out is None:
            out = torch.empty(m_total, dtype=torch.int64, device=self.dev)
        L.permutation(out, m_total, key)
        return out[:m_total]

    # ---------------------------------------------------------------- eager minibatch ------
    def _pre(self, idx, data, beta, encode):
        cfg = self.cfg
        obs = encode(data["boards"].index_select(0, idx))
        actions = data["actions"].index_select(0, idx)
        invalid = invalid_from_legal(data["legal"].index_select(0, idx))
        old_logp = data["logp"].index_select(0, idx)
        adv = data["adv"].index_select(0, idx)
        ret = data["ret"].index_select(0, idx)
        logits, value = self._forward(obs)
        loss, parts = ppo_losses(logits, value, actions, invalid, old_logp, adv, ret, beta, cfg.critic, cfg.clip_eps)
        self.grads.zero()
        loss.backward()
        return {"obs": obs, "invalid": invalid, "loss": loss.detach(), "ppo": parts["ppo"].detach(),
                "entropy": parts["entropy"].detach(), "vloss": parts["vloss"].detach(),
                "masked": parts["masked"].detach()}

    def _post(self, st, beta):
        cfg = self.cfg
        gn = self.grads.clip_(cfg.max_grad_norm)
        self.opt.step()
        with torch.no_grad():
            new_logits, _ = self._forward(st["obs"])
            kl = kl_old_new(st["masked"], new_logits, st["invalid"])
            vals = torch.stack([
                st["loss"], -st["ppo"].mean(), -beta * st["entropy"].mean(), cfg.critic * st["vloss"].mean(), gn,
                st["entropy"].mean(), kl.sum(), kl.mean(), torch.zeros((), device=self.dev)])
            self.stats.add_(vals)
            k = STAT_KEYS.index("kl_max")
            self.stats[k] = torch.maximum(self.stats[k], kl.max())

    def _minibatch(self, idx, data, beta, encode):
        st = self._pre(idx, data, beta, encode)
        self.grads.allreduce_mean()
        self._post(st, beta)

    # ---------------------------------------------------------------- graphed minibatch ----
    def _ensure_graph(self, data, bs, encode):
        key = (bs,) + tuple(t.data_ptr() for t in data.values())
        if self._g is not None and self._g["key"] == key:
            return
        self._g = None
        torch.cuda.synchronize()
        # the gradient all-reduce: captured inside the one graph under RCCL (and a no-op on a single
        # process without torch.distributed); gloo's host-staged all-reduce cannot be captured, so
        # there it runs eagerly between two graphs (g1: forward, loss, backward; g2: clip, optimizer,
        # KL); force_split exercises that path on one GPU
        split = not self.grads.capturable() or self.force_split
        idx = torch.zeros(bs, dtype=torch.int64, device=self.dev)
        params = [p for p in self.model.parameters()]
        snap_p = [p.detach().clone() for p in params]
        snap_o = self.opt.snapshot()
        snap_s = self.stats.clone()
        snap_x = self._extra_snapshot()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):  # warm-up outside the capture (library handles, autograd plans)
                self._minibatch(idx, data, self.beta_t, encode)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        g1, g2 = torch.cuda.CUDAGraph(), None
        with graph_capture(g1, pool=pool):
            st = self._pre(idx, data, self.beta_t, encode)
            if not split:
                self.grads.allreduce_mean()
                self._post(st, self.beta_t)
        if split:
            g2 = torch.cuda.CUDAGraph()
            with graph_capture(g2, pool=pool):
                self._post(st, self.beta_t)
        with torch.no_grad():
            for p, q in zip(params, snap_p):
                p.copy_(q)
        self.opt.restore(snap_o)
        self.stats.copy_(snap_s)
        self._extra_restore(snap_x)
        if self.weight_cache is not None:  # the warm-up's optimizer steps wrote the stepped weights' copies
            self.weight_cache.refresh()
        self._g = {"key": key, "idx": idx, "g1": g1, "g2": g2, "st": st}

    force_split = False

    def _extra_snapshot(self):
        return None

    def _extra_restore(self, snap):
        pass

    def _replay(self, idx):
        g = self._g
        g["idx"].copy_(idx)
        g["g1"].replay()
        if g["g2"] is not None:
            self.grads.allreduce_mean()
            g["g2"].replay()

    def close(self):
        """Drop the captured minibatch graphs (and, under RCCL, the all-reduce nodes captured in them)
        once the device is idle.  Call before torch.distributed.destroy_process_group(): a graph
        holding a captured collective must not outlive its communicator (RCCL frees the graph's
        persistent plan through the communicator when the graph is destroyed)."""
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)
        self._g = None
        if self.dev.type == "cuda":
            torch.cuda.synchronize(self.dev)
