"""GameURM policy forward on the device (game.py:1355-1458) for rollouts: the URM transformer's
kernels of include/g2048_urm.h (fused-epilogue MFMA projections for h <= 64; hipBLASLt through
torch.mm around the elementwise kernels otherwise; bf16 operands, fp32 accumulate).

The default config (h 64, 4 heads, inter 120, 1-2 layers) runs as ONE persistent kernel
(g2048_urm_forward: activations in registers / LDS, each layer's weights streamed through LDS).
Otherwise, per forward of n boards (16 n token rows):
  urm_stem                         emb = SiLU(LN(Linear(3->h))),  x = init_hidden + emb
  num_loops x num_layers blocks, h <= 64 (fused projections, no projection output in HBM):
                                   urm_linear (qkv) -> urm_attention -> urm_linear_rms (o_proj + residual
                                   + RMSNorm) -> urm_linear_swiglu (gate_up + SwiGLU + conv) ->
                                   urm_linear_rms (down_proj + residual + RMSNorm [+ emb])
  larger h:                        the same with torch.mm projections and urm_residual_rms /
                                   urm_swiglu_conv between them
                                   (the last block of a loop adds emb: the next loop's input)
  urm_pool_heads                   mean over the 16 tokens, action / value heads
Every buffer is allocated once per batch size and the weights are refreshed in place by sync(), so
a captured rollout graph keeps working across updates (same contract as rollout.FusedPolicy).
The truncated loops (no-grad in training, game.py:1437-1443) are ordinary loops in inference.
"""

from __future__ import annotations

import torch

from . import _lib as L


class URMPolicy:
    """Drop-in for rollout.InferencePolicy with a GameURM master: __call__(obs [n, 48] fp32/bf16) ->
    (logits fp32 [n, 4], value fp32 [n])."""

    def __init__(self, model: torch.nn.Module):
        self.master = model
        self.dtype = torch.bfloat16
        cfg = model.config
        self.h, self.heads = cfg.hidden_dim, cfg.num_heads
        self.loops, self.eps = cfg.num_loops, float(cfg.rms_norm_eps)
        self.inter = model.layers[0].mlp.inter
        self.mats = []  # per layer (Wqkv, Wo, Wgu, Wd) as bf16 copies
        # the trainer's Bf16Weights copies when attached (kept current by the optimizer; sync()
        # refreshes them like its own), else this policy's own copies
        self.shared = all(getattr(w, "_g2048_bf16", None) is not None for blk in model.layers
                          for w in (blk.attn.qkv_proj.weight, blk.attn.o_proj.weight, blk.mlp.gate_up_proj.weight,
                                    blk.mlp.down_proj.weight))
        for blk in model.layers:
            ws = (blk.attn.qkv_proj.weight, blk.attn.o_proj.weight, blk.mlp.gate_up_proj.weight, blk.mlp.down_proj.weight)
            self.mats.append([w._g2048_bf16 if self.shared else torch.empty_like(w, dtype=torch.bfloat16) for w in ws])
        dev = model.stem[0].weight.device
        # the conv taps / biases and init_hidden: the master tensors themselves where the one-launch
        # forward can stage them (fp32, contiguous, 16-byte aligned: it reads 16-byte chunks), else own
        # copies -- an optimizer may re-home the 1-D parameters into a flat buffer at any 4-byte offset
        # (round 5: read in place, the KL re-forward's ~5 copy kernels per minibatch are gone)
        def direct(t, shape):
            ok = t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 16 == 0 and t.device.type == "cuda"
            return t.detach().view(shape) if ok else None
        self._direct = {}
        self.conv_w, self.conv_b = [], []
        for blk in model.layers:
            cw = direct(blk.mlp.dwconv.weight, (self.inter, 2))
            cb = direct(blk.mlp.dwconv.bias, (self.inter,))
            self.conv_w.append(cw if cw is not None else torch.empty(self.inter, 2, dtype=torch.float32, device=dev))
            self.conv_b.append(cb if cb is not None else torch.empty(self.inter, dtype=torch.float32, device=dev))
            self._direct[id(self.conv_w[-1])] = cw is not None
            self._direct[id(self.conv_b[-1])] = cb is not None
        ih = direct(model.init_hidden, (16, self.h))
        self.init_hidden = ih if ih is not None else torch.empty(16, self.h, dtype=torch.float32, device=dev)
        self._direct[id(self.init_hidden)] = ih is not None
        h, i = self.h, self.inter
        # projections with fused epilogues when the kernels cover these shapes (h <= 64)
        self.fused = (L.urm_linear_supported(0, h, 3 * h) and L.urm_linear_supported(1, h, h)
                      and L.urm_linear_supported(2, h, 2 * i, i) and L.urm_linear_supported(1, i, h))
        # the whole forward in one persistent launch for the default config (g2048_urm_forward)
        self.mega = L.urm_forward_supported(h, self.heads, i, len(model.layers), cfg.conv_kernel)
        self._w = None
        if self.mega:
            w = L.UrmWeights()
            w.hidden, w.heads, w.inter, w.num_layers, w.num_loops = h, self.heads, i, len(model.layers), self.loops
            w.eps = self.eps
            ptr = lambda t: t.data_ptr()  # noqa: E731
            w.stem_w, w.ln_w, w.ln_b = ptr(model.stem[0].weight), ptr(model.stem[1].weight), ptr(model.stem[1].bias)
            w.init_hidden = ptr(self.init_hidden)
            w.wa, w.ba = ptr(model.action_head.weight), ptr(model.action_head.bias)
            w.wv, w.bv = ptr(model.value_head.weight), ptr(model.value_head.bias)
            for l, (blk, mats, cw) in enumerate(zip(model.layers, self.mats, self.conv_w)):
                w.qkv[l], w.o[l], w.gate_up[l], w.down[l] = (ptr(m) for m in mats)
                w.conv_w[l], w.conv_b[l] = ptr(cw), ptr(self.conv_b[l])
            self._w = w
        self._n = -1
        self.sync()

    def param_ptrs(self) -> tuple:
        """The master parameters the one-launch forward reads in place (an optimizer that re-homes
        parameters into flat buffers changes these: the caller rebuilds the policy then)."""
        m = self.master
        ts = [m.stem[0].weight, m.stem[1].weight, m.stem[1].bias, m.action_head.weight, m.action_head.bias,
              m.value_head.weight, m.value_head.bias, m.init_hidden]
        ts += [t for blk in m.layers for t in (blk.mlp.dwconv.weight, blk.mlp.dwconv.bias)]
        return tuple(t.data_ptr() for t in ts)

    def forward_train(self, obs: torch.Tensor, p: float):
        """The one-launch forward with the model's attention dropout (training mode, no gradient):
        the PPO update's KL re-forward (train.py:577-582).  Masks from the same Philox key and device
        call counter as URMAttentionFn (application app at counter + app; the counter is bumped by the
        number of applications).  Fresh output tensors."""
        n = obs.shape[0]
        logits = torch.empty(n, 4, dtype=torch.float32, device=obs.device)
        value = torch.empty(n, dtype=torch.float32, device=obs.device)
        seed, ctr = _attn_drop_state(obs.device)
        L.urm_forward_drop(self._w, obs.contiguous(), logits, value, p, seed, ctr)
        ctr.add_(self.loops * len(self.master.layers))
        return logits, value

    @staticmethod
    def supports(model) -> bool:
        try:
            import agent
        except ImportError:  # pragma: no cover
            return False
        if not isinstance(model, agent.GameURM):
            return False
        c = model.config
        return (c.conv_kernel == 2 and c.hidden_dim % 4 == 0 and c.hidden_dim <= 512 and c.hidden_dim % c.num_heads == 0
                and c.hidden_dim // c.num_heads <= 64)

    @torch.no_grad()
    def sync(self, mats: bool = True):
        """Refresh the copies from the master weights (mats=False: only the conv / init_hidden copies --
        the KL re-forward inside the update, whose shared bf16 projection copies the optimizer step
        itself has just written)."""
        for blk, mt, cw in zip(self.master.layers, self.mats, self.conv_w):
            if mats or not self.shared:
                for dst, src in zip(mt, (blk.attn.qkv_proj.weight, blk.attn.o_proj.weight, blk.mlp.gate_up_proj.weight,
                                         blk.mlp.down_proj.weight)):
                    dst.copy_(src)
            if not self._direct[id(cw)]:
                cw.copy_(blk.mlp.dwconv.weight.view(self.inter, 2))
        for blk, cb in zip(self.master.layers, self.conv_b):
            if not self._direct[id(cb)]:
                cb.copy_(blk.mlp.dwconv.bias)
        if not self._direct[id(self.init_hidden)]:
            self.init_hidden.copy_(self.master.init_hidden.view(16, self.h))

    def _buffers(self, n: int, dev):
        if self._n == n:
            return
        r, h, i = 16 * n, self.h, self.inter
        bf = torch.bfloat16
        self.emb = torch.empty(r, h, dtype=torch.float32, device=dev)
        self.x = torch.empty(r, h, dtype=torch.float32, device=dev)
        self.xb = torch.empty(r, h, dtype=bf, device=dev)
        self.qkv = torch.empty(r, 3 * h, dtype=bf, device=dev)
        self.att = torch.empty(r, h, dtype=bf, device=dev)
        self.y = torch.empty(r, h, dtype=bf, device=dev)
        self.gu = torch.empty(r, 2 * i, dtype=bf, device=dev)
        self.act = torch.empty(r, i, dtype=bf, device=dev)
        self.logits = torch.empty(n, 4, dtype=torch.float32, device=dev)
        self.value = torch.empty(n, dtype=torch.float32, device=dev)
        self._n = n

    @torch.no_grad()
    def __call__(self, obs: torch.Tensor):
        m = self.master
        n = obs.shape[0]
        if self.mega:
            if getattr(self, "_nm", -1) != n:
                self.mlogits = torch.empty(n, 4, dtype=torch.float32, device=obs.device)
                self.mvalue = torch.empty(n, dtype=torch.float32, device=obs.device)
                self._nm = n
            L.urm_forward(self._w, obs.contiguous(), self.mlogits, self.mvalue)
            return self.mlogits, self.mvalue
        self._buffers(n, obs.device)
        L.urm_stem(obs.contiguous(), m.stem[0].weight, m.stem[1].weight, m.stem[1].bias, self.init_hidden, self.emb,
                   self.x, self.xb)
        nl = len(self.mats)
        for loop in range(self.loops):
            for li, (blk, (wqkv, wo, wgu, wd), cw) in enumerate(zip(m.layers, self.mats, self.conv_w)):
                nxt = self.emb if (li == nl - 1 and loop < self.loops - 1) else None
                if self.fused:
                    L.urm_linear(self.xb, wqkv, self.qkv)
                    L.urm_attention(self.qkv, self.att, self.heads)
                    L.urm_linear_rms(self.att, wo, self.x, None, self.xb, self.eps)
                    L.urm_linear_swiglu(self.xb, wgu, cw, blk.mlp.dwconv.bias, self.act)
                    L.urm_linear_rms(self.act, wd, self.x, nxt, self.xb, self.eps)
                    continue
                torch.mm(self.xb, wqkv.t(), out=self.qkv)
                L.urm_attention(self.qkv, self.att, self.heads)
                torch.mm(self.att, wo.t(), out=self.y)
                L.urm_residual_rms(self.x, self.y, None, self.xb, self.eps)
                torch.mm(self.xb, wgu.t(), out=self.gu)
                L.urm_swiglu_conv(self.gu, cw, blk.mlp.dwconv.bias, self.act)
                torch.mm(self.act, wd.t(), out=self.y)
                L.urm_residual_rms(self.x, self.y, nxt, self.xb, self.eps)
        L.urm_pool_heads(self.x, m.action_head.weight, m.action_head.bias, m.value_head.weight, m.value_head.bias,
                         self.logits, self.value)
        return self.logits, self.value


_ATTN_DROP: dict = {}  # device -> (seed, device int64 [1] call counter) of the attention dropout masks


def _attn_drop_state(dev):
    """The dropout masks' Philox key (drawn once per device from torch's CPU generator, so
    torch.manual_seed makes runs repeatable) and the device call counter, bumped by every training
    forward (a captured graph bumps it per replay: a fresh mask per minibatch)."""
    st = _ATTN_DROP.get(dev)
    if st is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        st = (seed, torch.zeros(1, dtype=torch.int64, device=dev))
        _ATTN_DROP[dev] = st
    return st


_ATTN_FWD: dict = {}  # device -> [counter snapshot, next application, counter] of the forward in progress


class attn_forward:
    """The scope of one GameURM forward (agent.GameURM.forward): its attention applications k = 0, 1, ...
    draw their dropout masks at (the counter when the first one ran) + k, and the device counter is bumped
    ONCE at the end by the number of applications -- the masks of round 4's per-application
    snapshot-and-bump, with two kernels per forward instead of two per application.  A nested scope
    joins the outer one."""

    def __init__(self, dev: torch.device):
        self.dev, self.st = dev, None

    def __enter__(self):
        if self.dev.type == "cuda" and self.dev not in _ATTN_FWD:
            self.st = [None, 0, None]
            _ATTN_FWD[self.dev] = self.st
        return self

    def __exit__(self, *exc):
        if self.st is None:
            return False
        del _ATTN_FWD[self.dev]
        if self.st[1] and exc[0] is None:
            self.st[2].add_(self.st[1])
        return False


class URMAttentionFn(torch.autograd.Function):
    """The attention core of GameURMAttention (game.py:1296-1317: scaled_dot_product_attention,
    no mask, dropout_p = config.dropout in training) for autograd training on the device: forward
    g2048_urm_attention(_drop), backward g2048_urm_attention_bwd(_drop) (P and the dropout mask
    regenerated; head_dim 16).  qkv bf16 [16 n, 3 h] -> out bf16 [16 n, h].  Inside attn_forward the
    mask counter is the forward's snapshot + this application's index; alone, a snapshot of its own
    and a bump of the device counter by one."""

    @staticmethod
    def forward(ctx, qkv: torch.Tensor, heads: int, p: float = 0.0):
        qkv = qkv.contiguous()
        out = torch.empty(qkv.shape[0], qkv.shape[1] // 3, dtype=qkv.dtype, device=qkv.device)
        ctx.heads, ctx.p, ctx.seed, ctx.off = heads, float(p), 0, 0
        if p > 0.0:
            seed, ctr = _attn_drop_state(qkv.device)
            st = _ATTN_FWD.get(qkv.device)
            if st is not None:
                if st[0] is None:
                    st[0], st[2] = ctr.clone(), ctr
                c, ctx.off = st[0], st[1]
                st[1] += 1
            else:
                c = ctr.clone()  # this call's counter value: the backward regenerates the mask from it
            L.urm_attention(qkv, out, heads, p, seed, c, offset=ctx.off)
            if st is None:
                ctr.add_(1)
            ctx.seed = seed
            ctx.save_for_backward(qkv, c)
        else:
            L.urm_attention(qkv, out, heads)
            ctx.save_for_backward(qkv)
        return out

    @staticmethod
    def backward(ctx, dout: torch.Tensor):
        qkv = ctx.saved_tensors[0]
        dqkv = torch.empty_like(qkv)
        if ctx.p > 0.0:
            L.urm_attention_bwd(qkv, dout.to(qkv.dtype).contiguous(), dqkv, ctx.heads, ctx.p, ctx.seed,
                                ctx.saved_tensors[1], offset=ctx.off)
        else:
            L.urm_attention_bwd(qkv, dout.to(qkv.dtype).contiguous(), dqkv, ctx.heads)
        return dqkv, None, None


def attention_supported(qkv: torch.Tensor, seq: int, hidden: int, heads: int, dropout: float) -> bool:
    """The device attention path applies: bf16 qkv on the GPU (autocast), 16 tokens, head_dim 16,
    attention dropout 0 <= p < 1 (the device mask)."""
    return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and seq == 16 and hidden == 16 * heads
            and 0.0 <= dropout < 1.0)


class StemFn(torch.autograd.Function):
    """GameURM's stem (game.py:1376-1380: Linear(3 -> 64, no bias) + LayerNorm + SiLU) under bf16
    autocast, for autograd training on the device: one kernel forward (g2048_urm_stem_fwd), one
    backward (g2048_urm_stem_bwd: dW, d ln_w, d ln_b with deterministic column sums, everything
    recomputed from the 12-byte token input) instead of the bf16 GEMM, LayerNorm and SiLU kernels
    and a K = 16 n weight-gradient GEMM.  obs [n, 48] -> emb fp32 [16 n, 64]; obs gets no gradient."""

    @staticmethod
    def forward(ctx, obs: torch.Tensor, w: torch.Tensor, ln_w: torch.Tensor, ln_b: torch.Tensor, eps: float):
        obs = obs.contiguous()
        wf, gf, bf = (t.detach().float().contiguous() for t in (w, ln_w, ln_b))
        emb = torch.empty(obs.shape[0] * 16, 64, dtype=torch.float32, device=obs.device)
        L.urm_stem_fwd(obs, wf, gf, bf, emb, eps)
        ctx.save_for_backward(obs, wf, gf, bf)
        ctx.eps = eps
        ctx.dtypes = (w.dtype, ln_w.dtype, ln_b.dtype)
        ctx.targets = tuple(_direct_target(t) for t in (w, ln_w, ln_b))
        return emb

    @staticmethod
    def backward(ctx, demb: torch.Tensor):
        obs, wf, gf, bf = ctx.saved_tensors
        part = torch.empty(L.urm_stem_partials(obs.shape[0]), dtype=torch.float32, device=obs.device)
        sinks = [_grad_sink(t, s) for t, s in zip(ctx.targets, ((64, 3), (64,), (64,)))]
        if all(k is not None for k in sinks):  # direct_weight_grads: straight into the three .grad
            L.urm_stem_bwd3(obs, wf, gf, bf, demb.float().contiguous(), *sinks, part, ctx.eps, accumulate=True)
            return None, None, None, None, None
        grads = torch.empty(320, dtype=torch.float32, device=obs.device)
        L.urm_stem_bwd(obs, wf, gf, bf, demb.float().contiguous(), grads, part, ctx.eps)
        dw, dg, db = grads[:192].view(64, 3), grads[192:256], grads[256:]
        return (None, dw.to(ctx.dtypes[0]), dg.to(ctx.dtypes[1]), db.to(ctx.dtypes[2]), None)


def train_nograd_forward(model, obs: torch.Tensor):
    """GameURM.forward in training mode without autograd on the device (the PPO update's KL
    diagnostic re-forward, train.py:577-582): the one-launch forward g2048_urm_forward_drop with the
    model's attention dropout instead of ~50 per-op kernels.  Rounding points are the inference
    kernel's (fp32 stem, fused epilogues), not autocast's; the KL is a logged diagnostic only.
    Returns None when the one-launch forward does not cover the model (caller falls back)."""
    if not (obs.is_cuda and obs.dtype in (torch.float32, torch.bfloat16) and obs.ndim == 2 and obs.shape[1] == 48):
        return None
    c = model.config
    # the kernel rounds like bf16 autocast: an fp32 (--fp32) update keeps the module's own forward
    if not (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return None
    if not (URMPolicy.supports(model) and 0.0 <= c.dropout < 1.0
            and L.urm_forward_supported(c.hidden_dim, c.num_heads, model.layers[0].mlp.inter, len(model.layers),
                                        c.conv_kernel)):
        return None
    pol = model.__dict__.get("_g2048_train_fwd")
    shared = all(getattr(w, "_g2048_bf16", None) is not None for blk in model.layers
                 for w in (blk.attn.qkv_proj.weight, blk.attn.o_proj.weight, blk.mlp.gate_up_proj.weight,
                           blk.mlp.down_proj.weight))
    if pol is None or pol.param_ptrs() != pol._ptrs or pol.shared != shared:
        pol = URMPolicy(model)
        pol._ptrs = pol.param_ptrs()
        model.__dict__["_g2048_train_fwd"] = pol
    else:
        # the bf16 weight copies of the current parameters (captured with a graph); shared Bf16Weights
        # copies were written by the optimizer step itself: only the conv / init_hidden copies
        pol.sync(mats=False)
    logits, value = pol.forward_train(obs, float(c.dropout))
    return logits, value.view(-1, 1)


def training_graph_ok(model) -> bool:
    """The PPO minibatch step of this GameURM can be captured into one hipGraph (like GameMLP's):
    every op of its training forward / backward is a device Function or a plain torch op (h 64,
    16-wide heads, conv kernel 2: the one-launch forward's config, so the KL re-forward is that
    kernel too) -- no library path that would sync the host inside the capture."""
    c = model.config
    st = model.stem
    return (URMPolicy.supports(model) and c.hidden_dim == 64 and c.hidden_dim == 16 * c.num_heads
            and 0.0 <= c.dropout < 1.0 and len(st) == 3 and isinstance(st[0], torch.nn.Linear) and st[0].bias is None
            and L.urm_forward_supported(c.hidden_dim, c.num_heads, model.layers[0].mlp.inter, len(model.layers),
                                        c.conv_kernel))


def stem_supported(model, obs: torch.Tensor) -> bool:
    """The device training stem applies: bf16 autocast on the GPU, h = 64, the default stem
    (Linear(3, 64, bias=False), affine LayerNorm, SiLU), an observation without gradient."""
    st = model.stem
    return (obs.is_cuda and obs.dtype in (torch.float32, torch.bfloat16) and not obs.requires_grad
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and len(st) == 3 and isinstance(st[0], torch.nn.Linear) and st[0].bias is None
            and tuple(st[0].weight.shape) == (64, 3) and isinstance(st[1], torch.nn.LayerNorm)
            and st[1].weight is not None and st[1].bias is not None and isinstance(st[2], torch.nn.SiLU))


class ResidualRMSFn(torch.autograd.Function):
    """rms_norm(h + a) of GameURMBlock (game.py:1346-1350, h = 64) for autograd training on the
    device: one kernel forward (g2048_urm_rms_res_fwd2), one backward (g2048_urm_rms_res_bwd2)
    instead of torch's ~10 elementwise / reduction launches each way.  h fp32, a fp32 or bf16.
    with_bf16=True also returns the output's bf16 copy (the next projection's autocast operand),
    written by the same kernel; its gradient is added in the backward kernel (no cast kernels)."""

    @staticmethod
    def forward(ctx, h: torch.Tensor, a: torch.Tensor, eps: float, with_bf16: bool = False):
        ctx.set_materialize_grads(False)
        shape = h.shape
        h2 = h.reshape(-1, shape[-1]).contiguous()
        a2 = a.reshape(-1, shape[-1]).contiguous()
        out = torch.empty_like(h2)
        outb = torch.empty(h2.shape, dtype=torch.bfloat16, device=h.device) if with_bf16 else None
        rstd = torch.empty(h2.shape[0], dtype=torch.float32, device=h.device)
        L.urm_rms_res_fwd(h2, a2, out, rstd, eps, outb)
        ctx.save_for_backward(out, rstd)
        ctx.a_dtype = a.dtype
        ctx.shape = shape
        if with_bf16:
            return out.view(shape), outb.view(shape)
        return out.view(shape)

    @staticmethod
    def backward(ctx, dout: torch.Tensor, doutb: torch.Tensor | None = None):
        out, rstd = ctx.saved_tensors
        if dout is None and doutb is None:
            return None, None, None, None
        dh = torch.empty_like(out)
        da = torch.empty(out.shape, dtype=ctx.a_dtype, device=out.device)
        d32 = None if dout is None else dout.reshape(out.shape).float().contiguous()
        db16 = None if doutb is None else doutb.reshape(out.shape).to(torch.bfloat16).contiguous()
        L.urm_rms_res_bwd(d32, out, rstd, dh, da, db16)
        return dh.view(ctx.shape), da.view(ctx.shape), None, None


class EmbGradAcc:
    """The emb gradient of GameURM's grad-enabled loops, summed inside their AddCastFn backward kernels
    (g2048_urm_add_cast_bwd_acc) instead of by autograd's accumulation adds over [rows, h] fp32: the
    loops' backwards run last loop first, each adds its gradient to the running sum, and the earliest
    loop returns the total -- the sum autograd would form, in its order ((g_K + g_K-1) + ...)."""

    def __init__(self):
        self.pending = 0  # AddCastFn applications recorded with this accumulator (agent.GameURM._loop)
        self.acc = None


class AddCastFn(torch.autograd.Function):
    """A loop start of GameURM (game.py:1441: hidden_states + emb) under bf16 autocast, for autograd
    training on the device: the fp32 sum and its bf16 copy -- the first block's qkv operand, which
    autocast would cast in a kernel of its own -- in one kernel (g2048_urm_add_cast); the backward
    sums the fp32 gradient (residual RMSNorm) and the bf16 one (the projection) in one kernel
    instead of autocast's cast backward plus autograd's accumulation.  Values bitwise those of
    `h + emb` and its `.to(bfloat16)`.  h [b, 16, 64] (contiguous, or init_hidden [1, 16, 64]
    expanded over the boards), emb [b, 16, 64] fp32 -> (out fp32, outb bf16).  acc (EmbGradAcc,
    optional): the emb gradient is summed over the loops in the backward kernels (round 5)."""

    @staticmethod
    def forward(ctx, h: torch.Tensor, emb: torch.Tensor, acc: EmbGradAcc | None = None):
        ctx.set_materialize_grads(False)
        b, s, hid = emb.shape
        e2 = emb.reshape(-1, hid).contiguous()
        bcast = h.shape[0] == 1 or h.stride(0) == 0
        a = (h[:1] if bcast else h).reshape(-1, hid).contiguous()
        out = torch.empty_like(e2)
        outb = torch.empty(e2.shape, dtype=torch.bfloat16, device=emb.device)
        L.urm_add_cast(a, s if bcast else 0, e2, out, outb)
        ctx.bcast, ctx.shape, ctx.acc = bcast, (b, s, hid), acc
        return out.view(b, s, hid), outb.view(b, s, hid)

    @staticmethod
    def backward(ctx, dout: torch.Tensor | None, doutb: torch.Tensor | None):
        acc = ctx.acc
        if dout is None and doutb is None:
            if acc is not None:
                acc.pending -= 1
                if acc.pending == 0 and acc.acc is not None:
                    total, acc.acc = acc.acc, None
                    return None, (total.view(ctx.shape) if ctx.needs_input_grad[1] else None), None
            return None, None, None
        b, s, hid = ctx.shape
        dev = (dout if dout is not None else doutb).device
        d32 = None if dout is None else dout.reshape(-1, hid).float().contiguous()
        d16 = None if doutb is None else doutb.reshape(-1, hid).to(torch.bfloat16).contiguous()
        need_h, need_e = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if acc is None or not need_e:
            dx = torch.empty(b * s, hid, dtype=torch.float32, device=dev)
            L.urm_add_cast_bwd(d32, d16, dx)
            dx = dx.view(b, s, hid)
            # the gradient of h in the shape it came in (an expanded init_hidden: expand's backward sums it)
            return (dx if need_h else None), (dx if need_e else None), None
        acc.pending -= 1
        if acc.pending < 0:
            raise RuntimeError("EmbGradAcc: more AddCastFn backwards than grad-enabled loops (retain_graph?)")
        if acc.acc is None and acc.pending > 0:  # the last loop (first backward): the running sum is its dx
            dx = torch.empty(b * s, hid, dtype=torch.float32, device=dev)
            L.urm_add_cast_bwd(d32, d16, dx)
            acc.acc = dx
            return (dx.view(b, s, hid) if need_h else None), None, None
        out = torch.empty(b * s, hid, dtype=torch.float32, device=dev)
        dx = torch.empty(b * s, hid, dtype=torch.float32, device=dev) if need_h and acc.acc is not None else None
        L.urm_add_cast_bwd(d32, d16, dx, acc_in=acc.acc, acc_out=out)
        if acc.acc is None:  # a single loop: the sum is dx itself
            dx = out
        if acc.pending == 0:  # the earliest loop: the total is emb's gradient
            acc.acc = None
            return (dx.view(b, s, hid) if need_h else None), out.view(b, s, hid), None
        acc.acc = out
        return (dx.view(b, s, hid) if need_h else None), None, None


class MeanPoolFn(torch.autograd.Function):
    """GameURM's token mean-pool (game.py:1450, h.mean(dim=1)) whose backward hands on dpooled / 16
    EXPANDED over the 16 tokens (a stride-0 view) instead of torch's materialised [b, 16, h] division:
    the last residual RMSNorm backward reads the [b, h] gradient itself (g2048_urm_rms_res_bwd3),
    anything else materialises the view on use.  Values bitwise torch's mean backward."""

    @staticmethod
    def forward(ctx, h: torch.Tensor):
        ctx.shape = h.shape
        return h.mean(dim=1)

    @staticmethod
    def backward(ctx, dp: torch.Tensor):
        b, s, hid = ctx.shape
        return (dp / s).unsqueeze(1).expand(b, s, hid)


def _pooled_grad(dout: torch.Tensor | None, shape) -> torch.Tensor | None:
    """The [b, h] base of a mean-pool gradient (MeanPoolFn's expanded view over the 16 tokens), or None."""
    if dout is None or dout.dim() != 3 or dout.shape[1] != 16 or dout.stride(1) != 0 or dout.dtype != torch.float32:
        return None
    base = dout[:, 0, :]
    return base if base.is_contiguous() and tuple(dout.shape) == tuple(shape) else None


def add_cast_supported(h: torch.Tensor, emb: torch.Tensor) -> bool:
    """AddCastFn applies: bf16 autocast on the GPU, fp32 [b, 16, 64] operands (h possibly the
    expanded init_hidden)."""
    if not (emb.is_cuda and h.is_cuda and emb.dtype == torch.float32 and h.dtype == torch.float32):
        return False
    if emb.ndim != 3 or h.ndim != 3 or tuple(emb.shape[1:]) != (16, 64) or tuple(h.shape[1:]) != (16, 64):
        return False
    if not emb.is_contiguous() or h.shape[0] not in (1, emb.shape[0]):
        return False
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


def rms_res_supported(h: torch.Tensor, a: torch.Tensor) -> bool:
    """The device residual RMSNorm applies: fp32 residual stream of hidden size 64 on the GPU."""
    return (h.is_cuda and h.dtype == torch.float32 and a.dtype in (torch.float32, torch.bfloat16)
            and h.shape == a.shape and h.shape[-1] == 64)


class SwiGLUConvFn(torch.autograd.Function):
    """silu(conv2(silu(gate) * up)) of GameConvSwiGLU (game.py:1264-1276, kernel-2 depthwise conv
    over the 16 tokens of a board) for autograd training on the device: gu bf16 [16 n, 2 inter] ->
    act bf16 [16 n, inter] (the down_proj operand); backward dgu, dw [inter, 2], db [inter]."""

    @staticmethod
    def forward(ctx, gu: torch.Tensor, w: torch.Tensor, b: torch.Tensor):
        gu = gu.contiguous()
        wf, bf = w.detach().float().contiguous(), b.detach().float().contiguous()
        act = torch.empty(gu.shape[0], gu.shape[1] // 2, dtype=torch.bfloat16, device=gu.device)
        L.urm_swiglu_conv_fwd(gu, wf, bf, act)
        ctx.save_for_backward(gu, wf, bf)
        ctx.w_dtype, ctx.b_dtype = w.dtype, b.dtype
        return act

    @staticmethod
    def backward(ctx, dact: torch.Tensor):
        gu, wf, bf = ctx.saved_tensors
        rows, inter = gu.shape[0], gu.shape[1] // 2
        dgu = torch.empty_like(gu)
        dw = torch.empty(inter, 2, dtype=torch.float32, device=gu.device)
        db = torch.empty(inter, dtype=torch.float32, device=gu.device)
        part = torch.empty(L.urm_swiglu_conv_partials(rows // 16, inter), dtype=torch.float32, device=gu.device)
        L.urm_swiglu_conv_bwd(gu, wf, bf, dact.to(torch.bfloat16).contiguous(), dgu, dw, db, part)
        return dgu, dw.to(ctx.w_dtype), db.to(ctx.b_dtype)


def _wgrad(dy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW fp32 [n, k] = dy^T x over the token rows (g2048_urm_wgrad, deterministic)."""
    m, n = dy.shape
    k = x.shape[1]
    dw = torch.empty(n, k, dtype=torch.float32, device=dy.device)
    part = torch.empty(L.urm_wgrad_partials(m, n, k), dtype=torch.float32, device=dy.device)
    L.urm_wgrad(dy.contiguous(), x.contiguous(), dw, part)
    return dw


_DIRECT = [False]  # direct_weight_grads() in force


class direct_weight_grads:
    """Within this scope the training Functions add the gradients of GameURM's shared weights (the
    projections and the conv, applied once per loop) straight into the parameters' fp32 .grad, inside
    the kernels that produce them (g2048_urm_wgrad_acc / g2048_urm_gate_up_swiglu_bwd_acc), and return
    None for them: autograd's accumulation of the returned gradients -- an add_ kernel per extra
    application and parameter, ~40 per minibatch -- is gone, and the bits are the same (each
    application's sum is rounded once and added in the order autograd would add it; the first lands
    on the zeroed .grad).  For callers that zero .grad before the backward (the PPO update's
    GradBucket); torch.autograd.grad-style callers stay outside the scope."""

    def __enter__(self):
        self.prev = _DIRECT[0]
        _DIRECT[0] = True
        return self

    def __exit__(self, *exc):
        _DIRECT[0] = self.prev
        return False


def _direct_target(w: torch.Tensor):
    """w (a leaf parameter) when its gradient may be accumulated in place (direct_weight_grads), else
    None; decided at forward time, checked again at backward (_grad_sink)."""
    return w if (_DIRECT[0] and w.is_leaf and w.requires_grad and w.dtype == torch.float32) else None


def _grad_sink(w: torch.Tensor | None, shape) -> torch.Tensor | None:
    """w.grad as an fp32 contiguous [shape] view to accumulate into, or None (then return the gradient)."""
    if w is None:
        return None
    g = w.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or not g.is_cuda:
        return None
    return g.view(shape)


def _wgrad_into(dy: torch.Tensor, x: torch.Tensor, target, dtype):
    """The weight gradient dy^T x: added into target.grad (returns None) when it is a direct target,
    else returned (fp32, cast to `dtype`)."""
    m, n = dy.shape
    k = x.shape[1]
    sink = _grad_sink(target, (n, k))
    if sink is None:
        return _wgrad(dy, x).to(dtype)
    part = torch.empty(L.urm_wgrad_partials(m, n, k), dtype=torch.float32, device=dy.device)
    L.urm_wgrad(dy.contiguous(), x.contiguous(), sink, part, accumulate=True)
    return None


def _gemm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y bf16 [rows, n] = x w^T for bf16 x [rows, k], w [n, k]: the MFMA projection kernel
    (g2048_urm_linear) when it covers the shape, else autocast's library GEMM (torch.mm)."""
    rows, k = x.shape
    n = w.shape[0]
    if rows % 16 == 0 and n % 8 == 0 and L.urm_linear_supported(0, k, n):
        y = torch.empty(rows, n, dtype=torch.bfloat16, device=x.device)
        L.urm_linear(x, w.contiguous(), y)
        return y
    return torch.mm(x, w.t())


def _gemm_t(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx bf16 [rows, k] = dy [rows, n] w for w [n, k] (a projection's input gradient): the MFMA
    projection kernel stages W^T itself (g2048_urm_linear_t; bitwise _gemm(dy, w.t().contiguous())),
    else the library GEMM."""
    rows, n = dy.shape
    k = w.shape[1]
    if rows % 16 == 0 and k % 8 == 0 and n % 4 == 0 and L.urm_linear_supported(0, n, k):
        y = torch.empty(rows, k, dtype=torch.bfloat16, device=dy.device)
        L.urm_linear_t(dy, w.contiguous(), y)
        return y
    return torch.mm(dy, w)


def bf16_weight(w: torch.Tensor) -> torch.Tensor:
    """The autocast bf16 operand of a projection weight: its Bf16Weights copy (written by the fused
    Muon step with the weight itself, so no cast kernel per use) when one is attached and current,
    else a cast.  Current = no torch op wrote the weight since the copy's last refresh (the fused
    step writes both through raw pointers and bumps no version counter; load_state_dict, a torch
    optimizer or any in-place op on the weight does): a stale copy is never used silently."""
    c = getattr(w, "_g2048_bf16", None)
    if c is not None and getattr(w, "_g2048_bf16_ver", None) == w._version:
        return c
    return w.detach().to(torch.bfloat16)


class Bf16Weights:
    """bf16 copies of GameURM's projection weights (qkv, o, gate_up, down of every layer) kept current
    by the optimizer: FusedMuonAdamW writes them in the same launch that updates the fp32 weights
    (set_bf16_copies), refresh() copies them eagerly (the trainer calls it at the start of every
    update and after a capture's warm-up restored the weights).  The training Functions read them
    through bf16_weight() instead of casting every weight at every use (~40 cast / transpose kernels
    per minibatch); the KL re-forward's one-launch kernel reads them too."""

    def __init__(self, model, opt):
        self.pairs = []
        for blk in model.layers:
            for w in (blk.attn.qkv_proj.weight, blk.attn.o_proj.weight, blk.mlp.gate_up_proj.weight,
                      blk.mlp.down_proj.weight):
                t = torch.empty_like(w, dtype=torch.bfloat16)
                w._g2048_bf16 = t
                self.pairs.append((w, t))
        inner = getattr(opt, "opt", opt)
        inner.set_bf16_copies({w: t for w, t in self.pairs})
        self.refresh()

    @torch.no_grad()
    def refresh(self):
        for w, t in self.pairs:
            t.copy_(w)
            w._g2048_bf16_ver = w._version

    def detach(self):
        for w, _ in self.pairs:
            w._g2048_bf16 = None
            w._g2048_bf16_ver = None


def attach_bf16_weights(model, opt):
    """Bf16Weights for a GameURM whose optimizer writes bf16 copies (the fused Muon/AdamW kernel covers
    every projection), else None."""
    inner = getattr(opt, "opt", opt)
    if not getattr(inner, "supported", False) or not hasattr(inner, "set_bf16_copies"):
        return None
    muon_ids = {id(p) for p, _ in inner.muon}
    ws = [w for blk in model.layers for w in (blk.attn.qkv_proj.weight, blk.attn.o_proj.weight,
                                              blk.mlp.gate_up_proj.weight, blk.mlp.down_proj.weight)]
    if not all(id(w) in muon_ids for w in ws):
        return None
    return Bf16Weights(model, opt)


def gemm_supported(n: int, k: int) -> bool:
    """Both GEMMs of a projection w [n, k] (forward x w^T and input gradient dy w) run on the MFMA
    projection kernel (no library GEMM)."""
    return n % 8 == 0 and k % 8 == 0 and L.urm_linear_supported(0, k, n) and L.urm_linear_supported(0, n, k)


class URMLinearFn(torch.autograd.Function):
    """A bias-free projection y = x W^T of the GameURM blocks (qkv_proj, o_proj, down_proj) under bf16
    autocast: forward and input gradient are autocast's bf16 GEMMs (bf16 operands, fp32
    accumulation, bf16 result) on the MFMA projection kernel g2048_urm_linear -- the input gradient
    dY W as dY (W^T)^T with a 16-KB transposed weight copy -- and the weight gradient (a reduction
    over 16 n token rows) is g2048_urm_wgrad instead of a library GEMM with K = 16 n.
    x [rows, k] (bf16 or fp32: cast like autocast), w [n, k] -> y bf16 [rows, n]."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor):
        xb = x.to(torch.bfloat16).contiguous()
        wb = bf16_weight(w)
        ctx.save_for_backward(xb, wb)
        ctx.dtypes = (x.dtype, w.dtype)
        ctx.wt = _direct_target(w)
        return _gemm(xb, wb)

    @staticmethod
    def backward(ctx, dy: torch.Tensor):
        xb, wb = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        dx = _gemm_t(dy, wb) if ctx.needs_input_grad[0] else None
        dW = _wgrad_into(dy, xb, ctx.wt, ctx.dtypes[1])
        return (None if dx is None else dx.to(ctx.dtypes[0])), dW


class URMHeadsFn(torch.autograd.Function):
    """GameURM's action_head and value_head on the pooled features under bf16 autocast
    (game.py:1452-1456) without the library's K = n GEMMs (hipBLASLt ran the heads' weight gradient
    at ~0.2 ms and its input gradient at ~0.16 ms per 65 536 boards): the two heads as one [8, h]
    projection (action rows 0-3, value row 4, zero rows) on g2048_urm_linear_bias, the bf16 bias added
    to the fp32 accumulator before the one rounding (autocast's biased GEMM); backward: dW on
    g2048_urm_wgrad (dy zero-padded to 16 columns), dpooled = dy W on g2048_urm_linear, db a column
    sum.  pooled fp32 or bf16 [n, h] -> logits bf16 [n, 4], value bf16 [n, 1]."""

    @staticmethod
    def forward(ctx, pooled: torch.Tensor, wa: torch.Tensor, ba: torch.Tensor, wv: torch.Tensor, bv: torch.Tensor):
        h = pooled.shape[1]
        pb = pooled.to(torch.bfloat16).contiguous()
        w8 = torch.zeros(8, h, dtype=torch.bfloat16, device=pooled.device)
        w8[:4] = wa.detach()
        w8[4:5] = wv.detach()
        b8 = torch.zeros(8, dtype=torch.float32, device=pooled.device)  # autocast casts the bias to bf16
        b8[:4] = ba.detach().to(torch.bfloat16).float()
        b8[4:5] = bv.detach().to(torch.bfloat16).float()
        y = torch.empty(pb.shape[0], 8, dtype=torch.bfloat16, device=pooled.device)
        L.urm_linear_bias(pb, w8, b8, y)  # x W^T + b accumulated in fp32, ONE bf16 rounding (round 4)
        logits, value = y[:, :4].contiguous(), y[:, 4:5].contiguous()
        ctx.save_for_backward(pb, w8)
        ctx.dtypes = (pooled.dtype, wa.dtype, ba.dtype, wv.dtype, bv.dtype)
        return logits, value

    @staticmethod
    def backward(ctx, dlogits: torch.Tensor, dvalue: torch.Tensor):
        pb, w8 = ctx.saved_tensors
        n = pb.shape[0]
        dy = torch.zeros(n, 16, dtype=torch.bfloat16, device=pb.device)
        if dlogits is not None:
            dy[:, :4] = dlogits
        if dvalue is not None:
            dy[:, 4:5] = dvalue
        dw = _wgrad(dy, pb)                                        # [16, h] fp32
        db = dy[:, :5].float().sum(0)
        dp = _gemm_t(dy[:, :8].contiguous(), w8)                   # [n, h] bf16 = dy W
        t = ctx.dtypes
        return (dp.to(t[0]), dw[:4].to(t[1]), db[:4].to(t[2]), dw[4:5].to(t[3]), db[4:5].to(t[4]))


def heads_supported(model, pooled: torch.Tensor) -> bool:
    """URMHeadsFn applies: bf16 autocast on the GPU, whole boards of 16 (the projection kernel's row
    granularity), hidden 64 or 32 (the instantiated shapes)."""
    n, h = pooled.shape
    return (pooled.is_cuda and n % 16 == 0 and h in (32, 64) and model.action_head.bias is not None
            and model.value_head.bias is not None and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16 and L.urm_wgrad_supported(16, h)
            and L.urm_linear_supported(0, h, 8) and L.urm_linear_supported(0, 8, h))


def linear_supported(lin, x: torch.Tensor) -> bool:
    """URMLinearFn applies: bf16 autocast on the GPU, no bias, g2048_urm_wgrad's shapes."""
    n, k = lin.weight.shape
    return (x.is_cuda and lin.bias is None and x.shape[-1] == k and L.urm_wgrad_supported(n, k)
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)


def project(lin, x: torch.Tensor) -> torch.Tensor:
    """lin(x) through URMLinearFn when it applies (any leading shape), else the module."""
    if linear_supported(lin, x):
        return URMLinearFn.apply(x.reshape(-1, x.shape[-1]), lin.weight).view(*x.shape[:-1], lin.weight.shape[0])
    return lin(x)


class LinResRMSFn(torch.autograd.Function):
    """o_proj / down_proj + residual + post-norm of GameURMBlock (game.py:1346-1350: h = rms_norm(h +
    proj(x))) under bf16 autocast in ONE forward kernel (g2048_urm_linear_res_rms: the projection on
    MFMA, its autocast bf16 output added to h in the epilogue, RMSNorm, fp32 out + bf16 copy + rstd):
    the projection output's HBM round trip of URMLinearFn + ResidualRMSFn is gone.  Backward (round 5,
    h 64, k 64 / 120): ONE pass, g2048_urm_linres_bwd (dh fp32, and from the bf16 da held on chip dX
    on MFMA and dW accumulated per block); otherwise ResidualRMSFn's kernel (dh fp32, da bf16) then
    URMLinearFn's (dX on the projection kernel, dW on g2048_urm_wgrad).  h fp32 [..., n], x [..., k] (bf16, or cast like autocast), w [n, k] -> out fp32
    (and its bf16 copy with with_bf16)."""

    fused_bwd = True  # False: the round-4 three-launch backward (tests compare the two)

    @staticmethod
    def forward(ctx, h: torch.Tensor, x: torch.Tensor, w: torch.Tensor, eps: float, with_bf16: bool = False):
        ctx.set_materialize_grads(False)
        shape = h.shape
        h2 = h.reshape(-1, shape[-1]).contiguous()
        xb = x.reshape(-1, x.shape[-1]).to(torch.bfloat16).contiguous()
        wb = bf16_weight(w)
        out = torch.empty_like(h2)
        outb = torch.empty(h2.shape, dtype=torch.bfloat16, device=h.device) if with_bf16 else None
        rstd = torch.empty(h2.shape[0], dtype=torch.float32, device=h.device)
        L.urm_linear_res_rms(xb, wb, h2, out, outb, rstd, eps)
        ctx.save_for_backward(out, rstd, xb, wb)
        ctx.shape, ctx.xshape, ctx.dtypes = shape, x.shape, (x.dtype, w.dtype)
        ctx.wt = _direct_target(w)
        if with_bf16:
            return out.view(shape), outb.view(shape)
        return out.view(shape)

    @staticmethod
    def backward(ctx, dout: torch.Tensor | None, doutb: torch.Tensor | None = None):
        out, rstd, xb, wb = ctx.saved_tensors
        if dout is None and doutb is None:
            return None, None, None, None, None
        dh = torch.empty_like(out)
        dpool = _pooled_grad(dout, ctx.shape)  # the mean-pool's broadcast gradient, read as [b, h]
        d32 = None if dout is None or dpool is not None else dout.reshape(out.shape).float().contiguous()
        db16 = None if doutb is None else doutb.reshape(out.shape).to(torch.bfloat16).contiguous()
        n, k = wb.shape
        rows = out.shape[0]
        if LinResRMSFn.fused_bwd and ctx.needs_input_grad[2] and rows % 16 == 0 and L.urm_linres_bwd_supported(n, k):
            # round 5: one pass (g2048_urm_linres_bwd) -- the bf16 da never round-trips through HBM
            dx = torch.empty(rows, k, dtype=torch.bfloat16, device=out.device) if ctx.needs_input_grad[1] else None
            sink = _grad_sink(ctx.wt, (n, k))
            dwt = sink if sink is not None else torch.empty(n, k, dtype=torch.float32, device=out.device)
            part = torch.empty(L.urm_linres_bwd_partials(rows, k), dtype=torch.float32, device=out.device)
            L.urm_linres_bwd(out, rstd, wb, xb, dh, dwt, part, dout=d32, dpool=dpool, doutb=db16, dx=dx,
                             accumulate=sink is not None)
            dw = None if sink is not None else dwt.to(ctx.dtypes[1])
            return (dh.view(ctx.shape), None if dx is None else dx.to(ctx.dtypes[0]).view(ctx.xshape), dw, None, None)
        da = torch.empty(out.shape, dtype=torch.bfloat16, device=out.device)
        L.urm_rms_res_bwd(d32, out, rstd, dh, da, db16, dpool=dpool)
        dx = _gemm_t(da, wb) if ctx.needs_input_grad[1] else None
        dw = _wgrad_into(da, xb, ctx.wt, ctx.dtypes[1]) if ctx.needs_input_grad[2] else None
        return (dh.view(ctx.shape), None if dx is None else dx.to(ctx.dtypes[0]).view(ctx.xshape), dw, None, None)


def linres_supported(lin, h: torch.Tensor) -> bool:
    """LinResRMSFn applies: URMLinearFn's conditions, an fp32 residual stream of hidden size 64 (the
    residual RMSNorm kernels), the instantiated projection shapes."""
    n, k = lin.weight.shape
    return (h.is_cuda and h.dtype == torch.float32 and lin.bias is None and h.shape[-1] == n == 64
            and L.urm_wgrad_supported(n, k) and L.urm_linear_supported(4, k, n) and L.urm_linear_supported(0, n, k)
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16)


class GateUpSwiGLUFn(torch.autograd.Function):
    """gate_up_proj + SwiGLU + kernel-2 depthwise conv + SiLU of GameConvSwiGLU (game.py:1264-1276)
    under bf16 autocast, for autograd training on the device: ONE forward kernel
    (g2048_urm_linear_swiglu_train: the projection on MFMA with the SwiGLU-conv epilogue) instead of a
    library GEMM writing gu and a SwiGLU kernel reading it back.  Round 5: gu is not stored at all --
    the backward (g2048_urm_gate_up_swiglu_bwd) recomputes it from x on MFMA, bit for bit, instead of
    reading 2 inter bf16 per token back (x is h) -- then the input gradient dgu W on g2048_urm_linear_t
    and the weight gradient on g2048_urm_wgrad.  recompute=False (tests) stores gu and runs
    g2048_urm_swiglu_conv_bwd on it, the round-4 path.
    x [rows, h] (bf16 or fp32: cast like autocast), w [2 inter, h], cw [inter, 2], cb [inter]."""

    recompute = True

    @staticmethod
    def forward(ctx, x: torch.Tensor, w: torch.Tensor, cw: torch.Tensor, cb: torch.Tensor):
        xb = x.to(torch.bfloat16).contiguous()
        wb = bf16_weight(w)
        # the conv parameters as they are (fp32, contiguous views: the kernels stage them through LDS)
        cwf = cw.detach().float().contiguous()
        cbf = cb.detach().float().contiguous()
        inter = w.shape[0] // 2
        rec = GateUpSwiGLUFn.recompute and L.urm_gate_up_swiglu_bwd_supported(xb.shape[1], inter)
        gu = None if rec else torch.empty(xb.shape[0], 2 * inter, dtype=torch.bfloat16, device=x.device)
        act = torch.empty(xb.shape[0], inter, dtype=torch.bfloat16, device=x.device)
        L.urm_linear_swiglu_train(xb, wb, cwf, cbf, gu, act)
        if rec:
            ctx.save_for_backward(xb, wb, cwf, cbf)
        else:
            ctx.save_for_backward(xb, wb, cwf, cbf, gu)
        ctx.rec, ctx.inter = rec, inter
        ctx.dtypes = (x.dtype, w.dtype, cw.dtype, cb.dtype)
        ctx.wt = _direct_target(w)
        # the conv parameters: cw arrives as a view ([inter, 1, 2] -> [inter, 2]) of the leaf
        ctx.cwt = _direct_target(cw._base if cw._base is not None else cw)
        ctx.cbt = _direct_target(cb)
        return act

    @staticmethod
    def backward(ctx, dact: torch.Tensor):
        xb, wb, cwf, cbf = ctx.saved_tensors[:4]
        rows, inter = xb.shape[0], ctx.inter
        dgu = torch.empty(rows, 2 * inter, dtype=torch.bfloat16, device=xb.device)
        part = torch.empty(L.urm_swiglu_conv_partials(rows // 16, inter), dtype=torch.float32, device=xb.device)
        da = dact.to(torch.bfloat16).contiguous()
        # the conv gradients straight into both parameters' .grad (direct_weight_grads), else returned
        sw, sb = _grad_sink(ctx.cwt, (inter, 2)), _grad_sink(ctx.cbt, (inter,))
        acc = ctx.rec and sw is not None and sb is not None
        if acc:
            dw, db = sw, sb
        else:
            dw = torch.empty(inter, 2, dtype=torch.float32, device=xb.device)
            db = torch.empty(inter, dtype=torch.float32, device=xb.device)
        if ctx.rec:
            L.urm_gate_up_swiglu_bwd(xb, wb, cwf, cbf, da, dgu, dw, db, part, accumulate=acc)
        else:
            L.urm_swiglu_conv_bwd(ctx.saved_tensors[4], cwf, cbf, da, dgu, dw, db, part)
        dx = _gemm_t(dgu, wb)  # autocast's bf16 input-gradient GEMM, on MFMA
        dW = _wgrad_into(dgu, xb, ctx.wt, ctx.dtypes[1])  # the weight gradient on g2048_urm_wgrad (fp32)
        if acc:
            return dx.to(ctx.dtypes[0]), dW, None, None
        return dx.to(ctx.dtypes[0]), dW, dw.to(ctx.dtypes[2]), db.to(ctx.dtypes[3])


def gate_up_swiglu_nograd(x: torch.Tensor, w: torch.Tensor, cw: torch.Tensor, cb: torch.Tensor) -> torch.Tensor:
    """The same block outside autograd (GameURM's no-grad truncated loops, game.py:1437-1443): the
    training kernel's epilogue with no gu stored (g2048_urm_linear_swiglu_train, gu = NULL: act only,
    368 instead of 848 MB per call at 65 536 boards), so the hidden state handed to the gradient loops
    follows autocast's rounding points (gu rounded to bf16 before SwiGLU) and equals the training
    kernel's bit for bit (round 4; round 3 kept the projection in fp32 into the epilogue)."""
    xb = x.to(torch.bfloat16).contiguous()
    wb = bf16_weight(w)
    cwf = cw.detach().float().contiguous()
    cbf = cb.detach().float().contiguous()
    act = torch.empty(xb.shape[0], w.shape[0] // 2, dtype=torch.bfloat16, device=x.device)
    L.urm_linear_swiglu_train(xb, wb, cwf, cbf, None, act)
    return act


def gate_up_swiglu_supported(mlp, x: torch.Tensor) -> bool:
    """The fused training gate_up + SwiGLU-conv applies: bf16 autocast on the GPU, 16 tokens, conv
    kernel 2, a bias-free gate_up projection whose shape the fused kernel covers."""
    h = x.shape[-1]
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.ndim == 3 and x.shape[1] == 16
            and torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and mlp.dwconv.kernel_size[0] == 2 and mlp.gate_up_proj.bias is None
            and L.urm_linear_supported(3, h, 2 * mlp.inter, mlp.inter) and L.urm_linear_supported(2, h, 2 * mlp.inter, mlp.inter)
            and L.urm_wgrad_supported(2 * mlp.inter, h))


def swiglu_conv_supported(gu: torch.Tensor, seq: int, inter: int, kernel: int) -> bool:
    """The device SwiGLU + conv applies: bf16 gate_up output on the GPU (autocast), 16 tokens,
    conv kernel 2, inter <= 128."""
    return gu.is_cuda and gu.dtype == torch.bfloat16 and seq == 16 and kernel == 2 and inter <= 128
