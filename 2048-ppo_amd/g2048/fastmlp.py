"""The PPO minibatch step of GameMLP as explicit kernels (model_optimize_step, train.py:414-642).

PPOUpdater runs the reference's step through torch autograd.  For the reference's own policy,
GameMLP (game.py:1049-1220: stem Linear-LayerNorm-ReLU, L x [x + Dropout(ReLU(LN(W x)))],
action/value heads), FusedPPOUpdater writes the forward and backward out by hand:

    forward   X0 = obs(boards[idx])                          g2048_obs_gather
              G_l = H_{l-1} W_l^T                             g2048_mlp_fwd: one MFMA kernel per layer
              H_l = H_{l-1} + Drop(ReLU(LN(G_l)))             (hipBLASLt + g2048_ln_act_fwd beyond h=256)
    loss      heads + PPO-clip + entropy + smooth-L1 and      g2048_ppo_head_loss
              d/dH_L, d/d(head params), loss sums
    backward  dG_l, dgamma_l, dbeta_l from dy_l =            g2048_ln_act_bwd (after the fused train pass:
              heads(dz) + sum_{j>l} P_j                        all layers and P_l in ONE launch,
              P_l = dG_l W_l                                  g2048_ppo_backward; else per layer, P_l on
                                                              g2048_linear_dgrad)
              dW_l = dG_l^T H_{l-1}                           g2048_wgrad (bf16 MFMA, fp32 straight
                                                              into the flat gradient bucket)
    step      [RCCL all-reduce] clip, Muon + AdamW            dist.GradBucket / optim.MuonAdamW
    KL        re-forward with the new weights (train mode)    g2048_mlp_fwd per layer, the last block fused
                                                              with the head + KL (g2048_mlp_fwd_kl; else
                                                              g2048_ppo_head_kl)

Activations are bf16, LayerNorm statistics / gradients / reductions fp32, master weights fp32.
Dropout keep masks are Philox draws regenerated in the backward pass (nothing stored); they are
statistically, not bitwise, the reference's torch.nn.Dropout.  The whole step is one hipGraph
(two around the all-reduce with several ranks), replayed per minibatch; the ragged last minibatch of
an epoch replays the same graph, padded, with a device row count that masks the padding out of
the loss, the gradient and the statistics.
"""

from __future__ import annotations

import torch

from . import _lib as L
from .dist import graph as graph_capture
from .dist import world
from .ppo import STAT_KEYS, PPOConfig, PPOUpdater


def supports(model) -> bool:
    """FusedPPOUpdater handles the reference's GameMLP (hidden % 4 == 0, <= 1024)."""
    try:
        import agent
    except ImportError:  # pragma: no cover
        return False
    if not isinstance(model, agent.GameMLP):
        return False
    h = model.config.hidden_dim
    return h % 4 == 0 and h <= 1024


def head_grad_job(job, h: int, dwa, dwv, spill):
    """Re-describes the deferred column sum of g2048_wgrad(dz_bf16 [m, 16], H2 [m, h]) (partial rows
    [nb][16 h]: hi^T H2 in rows 0-7, lo^T H2 in rows 8-15) as 2 nb rows of 8 h, so the one column-sum
    adds the hi and lo halves: rows 0-3 -> dwa (action_head.weight.grad), row 4 -> dwv, 5-7 -> spill."""
    job.nb *= 2
    job.cols = 8 * h
    job.nseg = 3
    for k, (dst, n) in enumerate(((dwa, 4 * h), (dwv, h), (spill, 3 * h))):
        job.dst[k] = dst.data_ptr()
        job.len[k] = n
    return job


def _mm(a, b, out):
    """out = a @ b with fp32 accumulation (bf16 operands); fp32 `out` gets an fp32 result."""
    if out.dtype == a.dtype:
        torch.mm(a, b, out=out)
    else:
        out.copy_(torch.mm(a, b, out_dtype=out.dtype))


class FusedPPOUpdater(PPOUpdater):
    def __init__(self, model, optimizer, cfg: PPOConfig, grads, generator: torch.Generator | None = None,
                 graph: bool = False, seed: int = 0x5EED):
        if not supports(model):
            raise ValueError("FusedPPOUpdater needs an agent.GameMLP with hidden_dim % 4 == 0 and <= 1024")
        super().__init__(model, optimizer, cfg, grads, generator, graph)
        self.h = model.config.hidden_dim
        self.p_drop = float(model.config.dropout)
        self.decouple = bool(model.decouple_critic)
        self.lin = [model.stem[0].weight] + [b.mlp[0].weight for b in model.backbone]
        self.ln = [model.stem[1]] + [b.mlp[1] for b in model.backbone]
        self.wa, self.ba = model.action_head.weight, model.action_head.bias
        self.wv, self.bv = model.value_head.weight, model.value_head.bias
        self.wbf = [torch.empty_like(w, dtype=torch.bfloat16) for w in self.lin]
        self.mf_ok = [L.mlp_fwd_supported(w.shape[0], w.shape[1]) for w in self.lin]
        self.counter = torch.zeros(1, dtype=torch.int64, device=self.dev)  # dropout counter base
        # a fused optimizer (optim.FusedMuonAdamW) clips, steps and refreshes the bf16 weights itself
        self.fused_opt = bool(getattr(optimizer, "fused", False) or getattr(optimizer, "supported", False))
        if self.fused_opt:
            optimizer.set_bf16_copies(dict(zip(self.lin, self.wbf)))
        self.seed = seed
        self.bs = 0
        self.fused_pass = False
        self.opt_splits_heads = False

    # ---------------------------------------------------------------- buffers -------------
    def _alloc(self, bs: int):
        if self.bs == bs:
            return
        d, h, nl = self.dev, self.h, len(self.lin)
        bf = torch.bfloat16
        self.x0 = torch.empty(bs, 48, dtype=bf, device=d)
        self.G = [torch.empty(bs, h, dtype=bf, device=d) for _ in range(nl)]
        self.H = [torch.empty(bs, h, dtype=bf, device=d) for _ in range(nl)]
        self.mean = [torch.empty(bs, dtype=torch.float32, device=d) for _ in range(nl)]
        self.rstd = [torch.empty(bs, dtype=torch.float32, device=d) for _ in range(nl)]
        self.masked = torch.empty(bs, 4, dtype=torch.float32, device=d)
        self.dz = torch.empty(bs, 8, dtype=torch.float32, device=d)
        self.dg = torch.empty(bs, h, dtype=bf, device=d)
        # matmul gradients P_l = dG_l W_l of the blocks (l >= 1); with few blocks every one is kept and
        # each LayerNorm backward sums the ones above it (no fp32 residual-gradient round trips)
        self.keep_p = nl - 1 <= L.DY_MAX_P
        self.P = [torch.empty(bs, h, dtype=bf, device=d) for _ in range(nl if self.keep_p else 1)]
        self.dres = None if self.keep_p else torch.empty(bs, h, dtype=torch.float32, device=d)
        self.wg_ok = [L.wgrad_partials(bs, w.shape[0], w.shape[1]) > 0 for w in self.lin]
        self.dgrad_ok = [L.linear_dgrad_supported(w.shape[0], w.shape[1]) for w in self.lin]
        # per-reduction partial rows: every column sum of the backward is deferred into ONE
        # g2048_colsum_batch launch (and the KL's into the statistics kernel)
        f32 = torch.float32
        self.part_head = torch.empty(L.ppo_head_partials(bs, h), dtype=f32, device=d)
        self.part_kl = torch.empty(L.ppo_head_partials(bs, h), dtype=f32, device=d)
        self.part_ln = [torch.empty(L.ln_act_bwd_partials(bs, h), dtype=f32, device=d) for _ in range(nl)]
        self.part_wg = [torch.empty(max(1, L.wgrad_partials(bs, w.shape[0], w.shape[1])), dtype=f32, device=d)
                        for w in self.lin]
        self.sums = torch.zeros(3, dtype=torch.float32, device=d)
        self.kl = torch.zeros(2, dtype=torch.float32, device=d)
        self.rows = torch.full((1,), bs, dtype=torch.int64, device=d)  # valid rows (ragged last minibatch)
        # the fused train / KL passes (g2048_ppo_forward_loss / _kl): dz as bf16 for the head weight
        # gradient dz^T H2 on g2048_wgrad, the head weights split for the passes' MFMA operand
        self.fused_pass = (L.mlp_pass_supported(h, nl - 1) and bs * 2 * h < 2 ** 32
                           and L.wgrad_partials(bs, 16, h) > 0 and not self.force_layer_kernels)
        if self.fused_pass:
            self.dzb = torch.empty(bs, 16, dtype=bf, device=d)
            self.head_frag = torch.zeros(L.head_split_bytes(h), dtype=torch.uint8, device=d)
            # the fused Muon step writes the heads' split itself (no g2048_head_split per minibatch)
            self.opt_splits_heads = bool(self.fused_opt and hasattr(self.opt, "set_head_frag") and self.opt.set_head_frag(
                self.head_frag, {self.wa: 0, self.wv: 4}))
            self.part_fwd = torch.empty(L.mlp_pass_partials(bs, True), dtype=f32, device=d)
            self.part_klp = torch.empty(L.mlp_pass_partials(bs, False), dtype=f32, device=d)
            self.part_wh = torch.empty(L.wgrad_partials(bs, 16, h), dtype=f32, device=d)
            self.wh_spill = torch.empty(3 * h, dtype=f32, device=d)  # rows 5..7 of dz^T H2 (zero columns)
            self.wh_out = torch.empty(16, h, dtype=f32, device=d)   # (unused: the job's segments route it)
            # the fused backward (g2048_ppo_backward): every layer's dG kept for its weight gradient
            self.DG = [torch.empty(bs, h, dtype=bf, device=d) for _ in range(nl)]
            self.part_back = torch.empty(L.mlp_back_partials(bs, h), dtype=f32, device=d)
            # the blocks' dropout keep bits of the train pass (64 B per row), read by the backward
            # instead of re-drawing its Philox masks
            self.keep = torch.empty(2, bs, 4, dtype=torch.int64, device=d)
            npair = L.wgrad_pair_partials(bs, h, h)
            self.part_pair = [torch.empty(npair, dtype=f32, device=d) for _ in range(2)] if npair else None
            # the four weight gradients (head, stem, both blocks) in one streaming launch
            nmw = L.mlp_wgrad_partials(bs, h) if nl == 3 and bs * 4 * h < 2 ** 31 else 0
            self.part_mw = torch.empty(nmw, dtype=f32, device=d) if nmw else None
        self.bs = bs

    def _drop(self, layer: int, pass_: int):
        return L.make_dropout(self.p_drop if self.model.training else 0.0, layer, pass_, self.seed, 0, self.counter)

    force_layer_kernels = False  # tests: the per-layer kernel chain instead of the fused passes
    force_layer_backward = False  # tests: the fused train pass with the per-layer backward chain

    force_split_wgrad = False  # tests: g2048_wgrad / g2048_wgrad_pair instead of the one-launch g2048_mlp_wgrad

    @property
    def fused_back(self) -> bool:
        return self.fused_pass and all(self.wg_ok) and not self.force_layer_backward

    @property
    def wgrad_one_launch(self) -> bool:
        """The fused backward's weight gradients (and the head's) in one g2048_mlp_wgrad launch."""
        return self.fused_back and getattr(self, "part_mw", None) is not None and not self.force_split_wgrad

    @torch.no_grad()
    def refresh_weights(self):
        for w, b in zip(self.lin, self.wbf):
            b.copy_(w)
        self._split_heads()

    def _split_heads(self):
        if self.bs and self.fused_pass:
            L.head_split(self.wa, self.wv, self.head_frag)

    def _pass_args(self, data, idx, pass_: int, train: bool):
        """g2048_mlp_pass_args of this minibatch (pass 0: the train pass, 1: the KL re-forward)."""
        batch = L.make_ppo_batch(idx, data["actions"], data["legal"], data["logp"], data["adv"], data["ret"],
                                 rows=self.rows)
        common = dict(w_stem=self.wbf[0], w_blocks=self.wbf[1:], gammas=[ln.weight for ln in self.ln],
                      betas=[ln.bias for ln in self.ln], head_frag=self.head_frag, ba=self.ba,
                      drops=(self._drop(1, pass_), self._drop(2, pass_)), masked=self.masked)
        if self._offset:
            common["idx_offset"] = self.idx_off
        if not train:
            return L.make_mlp_pass(data["boards"], batch, idx.shape[0], partials=self.part_klp, **common)
        return L.make_mlp_pass(data["boards"], batch, idx.shape[0], bv=self.bv, beta_dev=self._beta_dev,
                               critic=self.cfg.critic, clip_eps=self.cfg.clip_eps, decouple=self.decouple, x0=self.x0,
                               g=self.G, h=self.H, mean=self.mean, rstd=self.rstd, dz=self.dz, dz_bf16=self.dzb,
                               partials=self.part_fwd, keep=self.keep, **common)

    def fused_forward_loss(self, data, idx, beta):
        """The train pass in one launch (obs -> GameMLP -> heads -> PPO loss, dz), then the head weight
        gradient dz^T H2 on g2048_wgrad (dz as two bf16 terms: fp32-accurate, like
        g2048_ppo_head_loss); returns the deferred column-sum jobs (bias gradients / loss sums, head
        weight gradients)."""
        self._beta_dev = beta if torch.is_tensor(beta) else torch.tensor(float(beta), device=self.dev)
        args = self._pass_args(data, idx, 0, True)
        self._kl_args = self._pass_args(data, idx, 1, False)
        j_loss, j_head = L.ColsumJob(), L.ColsumJob()
        L.ppo_forward_loss(args, self.ba.grad, self.bv.grad, self.sums, defer=j_loss)
        if self.wgrad_one_launch:  # the head weight gradient joins the backward's weight-gradient launch
            return [j_loss]
        L.wgrad(self.dzb, self.H[-1], self.part_wh, self.wh_out, defer=j_head)
        head_grad_job(j_head, self.h, self.wa.grad, self.wv.grad, self.wh_spill)
        return [j_loss, j_head]

    # ---------------------------------------------------------------- passes --------------
    def forward_features(self, boards, idx, pass_: int):
        """H_L of the minibatch boards[idx] (train mode: dropout of pass `pass_`)."""
        L.obs_gather(boards, idx, self.x0)
        return self._layers(pass_)

    def _layers(self, pass_: int, upto: int | None = None):
        x = self.x0
        for l, (w, ln) in enumerate(zip(self.wbf[:upto], self.ln[:upto])):
            drop = self._drop(l, pass_) if l > 0 else None
            if self.mf_ok[l]:  # Linear + LayerNorm + ReLU + dropout + residual in one MFMA kernel
                keep = pass_ == 0  # the KL re-forward (pass 1) needs no G / LayerNorm statistics
                L.mlp_fwd(x, w, ln.weight, ln.bias, l > 0, self.G[l] if keep else None, self.H[l],
                          self.mean[l] if keep else None, self.rstd[l] if keep else None, drop)
            else:
                _mm(x, w.t(), self.G[l])
                L.ln_act_fwd(self.G[l], ln.weight, ln.bias, x if l > 0 else None, self.H[l], self.mean[l],
                             self.rstd[l], drop)
            x = self.H[l]
        return x

    def fused_backward(self, jobs):
        """The backward after the fused train pass: g2048_ppo_backward (three LayerNorm backwards and
        the two block input gradients in one launch), then the weight gradients dW_l = dG_l^T X_l and
        the head's dz^T H2 in one g2048_mlp_wgrad launch (else g2048_wgrad / g2048_wgrad_pair); every
        column sum deferred into `jobs` and run as one g2048_colsum_batch."""
        ln = self.ln
        args = L.make_mlp_back(self.bs, self.wbf[1:], [x.weight for x in ln], [x.bias for x in ln], self.wa,
                               None if self.decouple else self.wv, self.dz, self.G, self.mean, self.rstd,
                               drops=(self._drop(1, 0), self._drop(2, 0)), dg=self.DG, partials=self.part_back,
                               keep=self.keep)
        jb = [L.ColsumJob() for _ in range(3)]
        L.ppo_backward(args, [x.weight.grad for x in ln], [x.bias.grad for x in ln], defer=jb)
        jobs.extend(jb)
        if self.wgrad_one_launch:  # head, stem and both blocks: one streaming launch, four column sums
            jw = [L.ColsumJob() for _ in range(4)]
            L.mlp_wgrad(self.bs, self.dzb, self.H[-1], self.DG, [self.x0, self.H[0], self.H[1]], self.part_mw,
                        self.wh_out, [w.grad for w in self.lin], defer=jw)
            head_grad_job(jw[0], self.h, self.wa.grad, self.wv.grad, self.wh_spill)
            jobs.extend(jw)
            self._colsum(jobs)
            return
        jobs.append(L.ColsumJob())
        L.wgrad(self.DG[0], self.x0, self.part_wg[0], self.lin[0].grad, defer=jobs[-1])
        if self.part_pair is not None:  # the two block layers' weight gradients in one launch
            jp = [L.ColsumJob(), L.ColsumJob()]
            L.wgrad_pair(self.DG[1], self.H[0], self.DG[2], self.H[1], self.part_pair[0], self.part_pair[1],
                         self.lin[1].grad, self.lin[2].grad, defer=jp)
            jobs.extend(jp)
        else:
            for l in (1, 2):
                jobs.append(L.ColsumJob())
                L.wgrad(self.DG[l], self.H[l - 1], self.part_wg[l], self.lin[l].grad, defer=jobs[-1])
        self._colsum(jobs)

    def _colsum(self, jobs):
        """The minibatch's deferred column sums in one launch; single process with the fused optimizer:
        g2048_colsum_batch_sq, which also writes the gradient norm's partials and counts the step, so
        the optimizer step needs no pass over the bucket (self._sq_done)."""
        inner = getattr(self.opt, "opt", self.opt)
        self._sq_done = False
        if (self.fused_opt and len(jobs) <= L.COLSUM_MAX_JOBS and hasattr(inner, "step_t") and world()[1] == 1
                and L.colsum_batch_blocks(jobs) <= L.COLSUM_SQ_MAX):
            skip = {self.sums.data_ptr(), getattr(self, "wh_spill", self.sums).data_ptr()}
            for j in jobs:  # pad_ bit k: segment k is a gradient (not the loss sums, not the head spill)
                j.pad_ = sum(1 << k for k in range(j.nseg) if j.dst[k] not in skip)
            if self.sq_part is None:
                self.sq_part = torch.zeros(L.COLSUM_SQ_MAX, dtype=torch.float32, device=self.dev)
            L.colsum_batch_sq(jobs, self.sq_part, inner.step_t)
            self._sq_done = True
            return
        for i in range(0, len(jobs), L.COLSUM_MAX_JOBS):
            L.colsum_batch(jobs[i:i + L.COLSUM_MAX_JOBS])

    sq_part = None
    _sq_done = False
    kl_sync = None  # the fused KL pass's ticket word (g2048_ppo_forward_kl_stats)

    def loss_backward(self, data, idx, beta, jobs=None):
        """Heads + PPO loss (unless the fused train pass did them: its `jobs`) + backward of the
        minibatch; gradients land in the GradBucket views."""
        nl = len(self.lin)
        if jobs is not None and self.fused_back:
            return self.fused_backward(jobs)
        if jobs is None:
            batch = L.make_ppo_batch(idx, data["actions"], data["legal"], data["logp"], data["adv"], data["ret"],
                                     rows=self.rows)
            # the heads write only their output gradient dz [m, 8]; the last block's backward
            # recomputes their share dz W of its output gradient (no [m, h] head gradient in HBM)
            jobs = [L.ColsumJob()]
            L.ppo_head_loss(self.H[-1], self.wa, self.ba, self.wv, self.bv, batch, beta, self.cfg.critic,
                            self.cfg.clip_eps, self.decouple, self.masked, None, self.part_head,
                            self.wa.grad, self.ba.grad, self.wv.grad, self.bv.grad, self.sums, dz=self.dz,
                            defer=jobs[-1])
        head = (self.dz, self.wa, None if self.decouple else self.wv)
        for l in range(nl - 1, -1, -1):
            ln = self.ln[l]
            if self.keep_p:  # dy_l = heads + sum_{j > l} P_j
                dy = L.make_dy(None, self.P[l + 1:], head)
                dres_out = None
            else:  # deep nets: the fp32 residual gradient dres accumulates P_{l+1} layer by layer
                dy = L.make_dy(self.dres if l < nl - 1 else None, [self.P[0]] if l < nl - 1 else [],
                               head if l == nl - 1 else None)
                dres_out = self.dres if l > 0 else None
            jobs.append(L.ColsumJob())
            L.ln_act_bwd(None, None, self.G[l], self.mean[l], self.rstd[l], ln.weight, ln.bias, self.dg, dres_out,
                         self.part_ln[l], ln.weight.grad, ln.bias.grad, self._drop(l, 0) if l > 0 else None, dy=dy,
                         defer=jobs[-1])
            x_in = self.H[l - 1] if l > 0 else self.x0
            if self.wg_ok[l]:  # dW = dG^T X on the MFMA weight-gradient kernel
                jobs.append(L.ColsumJob())
                L.wgrad(self.dg, x_in, self.part_wg[l], self.lin[l].grad, defer=jobs[-1])
            else:
                _mm(self.dg.t(), x_in, self.lin[l].grad)
            if l > 0:  # P_l = dG_l W_l, the input gradient, on the MFMA dgrad kernel (library GEMM otherwise)
                if self.dgrad_ok[l]:
                    L.linear_dgrad(self.dg, self.wbf[l], self.P[l if self.keep_p else 0])
                else:
                    _mm(self.dg, self.wbf[l], self.P[l if self.keep_p else 0])
        for i in range(0, len(jobs), L.COLSUM_MAX_JOBS):  # every deferred column sum, in one launch
            L.colsum_batch(jobs[i:i + L.COLSUM_MAX_JOBS])

    # ---------------------------------------------------------------- PPOUpdater hooks ----
    ragged_pad = True  # the ragged last minibatch runs padded to full size (g2048_ppo_batch.rows)
    MULTI = 8          # minibatch steps per captured graph in the offset path
    _og = None         # the offset path's graphs (see _update_offset)
    _offset = False    # the fused passes read rows perm[*idx_off + r] (set while capturing that path)

    @property
    def captured(self) -> bool:
        return self._g is not None or self._og is not None

    @property
    def graph_split(self) -> bool:
        return self._og is None and self._g is not None and self._g["g2"] is not None

    def _set_rows(self, n: int):
        self.rows.fill_(n)

    def update(self, data: dict, beta: float, encode=None) -> dict:
        bs = min(self.cfg.batch_size, data["actions"].shape[0])
        self._alloc(bs)
        self.refresh_weights()
        if self.graph and self.fused_pass and self.grads.capturable() and not self.force_split:
            return self._update_offset(data, beta, bs)
        return super().update(data, beta, encode)

    # ---------------------------------------------------------------- offset path ---------
    # The epoch's permutation lives in one device buffer and the fused passes read the minibatch's
    # rows at a device offset that the KL pass's last block advances, so consecutive minibatch steps
    # need no index copy and no host work between them: MULTI steps are captured in one hipGraph
    # (plus a one-step graph for the rest and the padded ragged minibatch).
    def _update_offset(self, data: dict, beta: float, bs: int) -> dict:
        cfg = self.cfg
        m_total = data["actions"].shape[0]
        self.stats.zero_()
        self.beta_t.fill_(beta)
        self.model.train()
        g = self._ensure_offset_graphs(data, bs)
        nb = 0
        for _ in range(cfg.epochs):
            self._epoch_perm(m_total, out=g["perm"])
            g["perm"][m_total:m_total + bs].zero_()  # the padded ragged minibatch reads row 0
            self.idx_off.zero_()
            nfull, rag = divmod(m_total, bs)
            k = 0
            while k + self.MULTI <= nfull:
                g["multi"].replay()
                k += self.MULTI
            while k < nfull:
                g["single"].replay()
                k += 1
            if rag:
                self._set_rows(rag)
                g["single"].replay()
                self._set_rows(bs)
                k += 1
            nb += k
        st = self.stats / max(nb, 1)
        st[STAT_KEYS.index("kl_max")] = self.stats[STAT_KEYS.index("kl_max")]
        return {k: st[i] for i, k in enumerate(STAT_KEYS)}

    def _ensure_offset_graphs(self, data, bs):
        cap = data["actions"].untyped_storage().nbytes() // data["actions"].element_size()
        key = (bs, cap) + tuple(t.data_ptr() for t in data.values())
        if self._og is not None and self._og["key"] == key:
            return self._og
        self._og = None
        torch.cuda.synchronize()
        perm = torch.zeros(cap + bs, dtype=torch.int64, device=self.dev)
        if getattr(self, "idx_off", None) is None:
            self.idx_off = torch.zeros(1, dtype=torch.int64, device=self.dev)
        idx = perm[:bs]
        params = list(self.model.parameters())
        snap_p = [p.detach().clone() for p in params]
        snap_o = self.opt.snapshot()
        snap_s = self.stats.clone()
        snap_x = self._extra_snapshot()
        self._offset = True
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm-up outside the capture
                    self._minibatch(idx, data, self.beta_t, None)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            pool = torch.cuda.graph_pool_handle()
            graphs = {}
            for name, n in (("single", 1), ("multi", self.MULTI)):
                gr = torch.cuda.CUDAGraph()
                with graph_capture(gr, pool=pool):
                    for _ in range(n):
                        st = self._pre(idx, data, self.beta_t, None)
                        self.grads.allreduce_mean()
                        self._post(st, self.beta_t)
                graphs[name] = gr
        finally:
            self._offset = False
        with torch.no_grad():
            for p, q in zip(params, snap_p):
                p.copy_(q)
        self.opt.restore(snap_o)
        self.stats.copy_(snap_s)
        self._extra_restore(snap_x)
        self._og = {"key": key, "perm": perm, **graphs}
        return self._og

    def _pre(self, idx, data, beta, encode):
        if idx.shape[0] != self.bs:  # ragged last minibatch of an eager pass
            self._alloc(idx.shape[0])
            self._split_heads()
        if self.fused_pass:
            self.loss_backward(data, idx, beta, jobs=self.fused_forward_loss(data, idx, beta))
        else:
            self.forward_features(data["boards"], idx, 0)
            self.loss_backward(data, idx, beta)
        return {}

    def _post(self, st, beta):
        cfg, m = self.cfg, self.bs
        if self.fused_opt:
            gn = self.opt.step_clipped(self.grads.flat, cfg.max_grad_norm,
                                       sq=self.sq_part if self._sq_done else None)
        else:
            gn = self.grads.clip_(cfg.max_grad_norm)
            self.opt.step()
            self.refresh_weights()
        with torch.no_grad():
            # KL re-forward of the same minibatch (x0 still holds its encoding); the KL partial rows
            # are reduced by the statistics kernel
            kl_job = L.ColsumJob()
            nl = len(self.lin)
            w_last = self.wbf[-1]
            b = beta if torch.is_tensor(beta) else torch.tensor(float(beta), device=self.dev)
            if gn.dim() != 0:
                gn = gn.reshape(())
            if self.fused_pass:  # the whole re-forward + KL + the statistics in one launch
                if not self.opt_splits_heads:
                    self._split_heads()
                if self.kl_sync is None:
                    self.kl_sync = torch.zeros(1, dtype=torch.int32, device=self.dev)
                L.ppo_forward_kl_stats(self._kl_args, self.sums, gn.float().contiguous(), b, cfg.critic, m,
                                       self.stats, self.kl_sync, counter=self.counter, rows=self.rows,
                                       idx_offset=self.idx_off if self._offset else None, idx_step=m)
                return
            elif nl > 1 and self.mf_ok[-1] and L.mlp_fwd_kl_supported(w_last.shape[0], w_last.shape[1]):
                # the last block fused with the action head and the KL reduction (no H write / re-read)
                x = self._layers(1, upto=nl - 1)
                ln = self.ln[-1]
                L.mlp_fwd_kl(x, w_last, ln.weight, ln.bias, self._drop(nl - 1, 1), self.wa, self.ba, self.masked,
                             self.part_kl, self.kl, defer=kl_job, rows=self.rows)
            else:
                x = self._layers(1)
                L.ppo_head_kl(x, self.wa, self.ba, self.masked, self.part_kl, self.kl, defer=kl_job, rows=self.rows)
            b = beta if torch.is_tensor(beta) else torch.tensor(float(beta), device=self.dev)
            if gn.dim() != 0:
                gn = gn.reshape(())
            # one launch: the statistics of this minibatch, and the next minibatch's dropout counter
            kl_part = self.part_klp if self.fused_pass else self.part_kl  # the KL kernel's partial rows
            L.ppo_stats(self.sums, kl_part, gn.float().contiguous(), b, cfg.critic, m, self.stats, self.counter,
                        kl_rows=kl_job.nb, rows=self.rows)

    idx_off = None  # the offset path's device row offset (advanced by the KL pass's last block)

    def close(self):
        """PPOUpdater.close(), and the offset path's graphs (MULTI captured all-reduces each)."""
        torch.cuda.synchronize(self.dev)
        self._og = None
        super().close()

    def _extra_snapshot(self):
        return (self.counter.clone(), None if self.idx_off is None else self.idx_off.clone())

    def _extra_restore(self, snap):
        self.counter.copy_(snap[0])
        if snap[1] is not None:
            self.idx_off.copy_(snap[1])
        self.refresh_weights()  # the capture warm-up stepped (and then restored) the master weights
