"""agent.py -- the policy/value nn.Module interface of the 2048 trainer.

The reference's `agent.py` is empty; its modules live in game.py (GameMLP game.py:1049-1220,
GameURM game.py:1355-1458, configs game.py:24-42).  This module provides the same call contract
and the same state_dict keys, so a reference checkpoint (docs/data/best_model.pt, written by
train.py:1893-1901) loads unchanged:

  forward(x[B,48]) -> (logits[B,4], value[B,1]), logits ordered UP, DOWN, LEFT, RIGHT
  .directions, .get_param_groups(value_lr, other_lr), .action_head, .value_head

Sub-modules are created in the reference's order and re-initialised with the same Kaiming-uniform
scheme, so under the same torch seed the initial weights are identical to the reference's.
On MI355X these modules are the parameter containers and the eager reference: the rollout runs the
fused HIP policy (g2048.policy), the PPO update the kernel-written forward / backward / optimizer
of g2048.fastmlp and g2048.optim (GameMLP) and g2048.urm (GameURM) on the same parameters.
"""

from __future__ import annotations

from enum import Enum

import torch
import torch.nn as nn
import torch.nn.functional as F
from pydantic import BaseModel

N_CELLS = 16
N_FEATURES = 3 * N_CELLS
N_ACTIONS = 4


class Direction(Enum):
    """game.py:14-18; also the model head order (game.py:1087-1092)."""
    UP = "up"
    DOWN = "down"
    LEFT = "left"
    RIGHT = "right"


ACTION_ORDER = [Direction.UP, Direction.DOWN, Direction.LEFT, Direction.RIGHT]


class MLPConfig(BaseModel):
    hidden_dim: int = 64
    num_layers: int = 2
    dropout: float = 0.1
    decouple_critic: bool = False


class GameURMConfig(BaseModel):
    hidden_dim: int = 64
    num_layers: int = 2
    num_heads: int = 4
    expansion: float = 2.67
    dropout: float = 0.1
    num_loops: int = 4
    num_truncated_loops: int = 1
    conv_kernel: int = 2
    rms_norm_eps: float = 1e-5


def _kaiming_linear(m: nn.Module) -> None:
    if isinstance(m, nn.Linear):
        nn.init.kaiming_uniform_(m.weight, nonlinearity="relu")
        if m.bias is not None:
            nn.init.zeros_(m.bias)


def _split_param_groups(model: nn.Module, value_lr: float, other_lr: float) -> list[dict]:
    """[other 2-D, other 1-D, value-head 2-D, value-head 1-D] (game.py:1093-1127): 2-D go to Muon,
    1-D (LayerNorm, biases) to AdamW in the trainer."""
    groups = {("o", 2): [], ("o", 1): [], ("v", 2): [], ("v", 1): []}
    for name, child in model.named_children():
        side = "v" if name == "value_head" else "o"
        for p in child.parameters():
            groups[(side, 2 if p.ndim >= 2 else 1)].append(p)
    return [{"params": groups[("o", 2)], "lr": other_lr}, {"params": groups[("o", 1)], "lr": other_lr},
            {"params": groups[("v", 2)], "lr": value_lr}, {"params": groups[("v", 1)], "lr": value_lr}]


class ResidualBlock(nn.Module):
    """x + Dropout(ReLU(LayerNorm(W x)))  (game.py:1033-1046)."""

    def __init__(self, hidden_dim: int, dropout: float = 0.1):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(hidden_dim, hidden_dim, bias=False), nn.LayerNorm(hidden_dim), nn.ReLU(),
                                 nn.Dropout(dropout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x + self.mlp(x)


class GameMLP(nn.Module):
    """Residual MLP policy + value heads (game.py:1049-1220)."""

    N = N_CELLS
    NUM_ACTIONS = N_ACTIONS

    def __init__(self, config: MLPConfig) -> None:
        super().__init__()
        h = config.hidden_dim
        self.config = config
        self.decouple_critic = config.decouple_critic
        self.stem = nn.Sequential(nn.Linear(N_FEATURES, h, bias=False), nn.LayerNorm(h), nn.ReLU())
        self.backbone = nn.ModuleList(ResidualBlock(h, config.dropout) for _ in range(config.num_layers))
        self.action_head = nn.Linear(h, N_ACTIONS)
        self.value_head = nn.Linear(h, 1)
        self.apply(_kaiming_linear)

    @property
    def directions(self) -> list[Direction]:
        return list(ACTION_ORDER)

    def get_param_groups(self, value_lr: float, other_lr: float) -> list[dict]:
        return _split_param_groups(self, value_lr, other_lr)

    def get_1d_and_2d_params(self) -> tuple[list, list]:
        one = [p for p in self.parameters() if p.ndim == 1]
        two = [p for p in self.parameters() if p.ndim >= 2]
        return one, two

    def features(self, x: torch.Tensor) -> torch.Tensor:
        x = self.stem(x)
        for block in self.backbone:
            x = block(x)
        return x

    def forward(self, inputs: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        if inputs.ndim <= 1:
            raise ValueError(f"input must consist of shape (batch, channel), got: {inputs.shape}")
        if inputs.shape[-1] != N_FEATURES:
            raise AssertionError(f"{inputs.shape[-1]} does not equal {N_FEATURES}")
        # float32 like the reference (game.py:1191); a low-precision inference copy keeps its own dtype
        x = self.features(inputs.to(self.stem[0].weight.dtype))
        logits = self.action_head(x)
        value = self.value_head(x.detach() if self.decouple_critic else x)
        return logits, value


# ------------------------------------------------------------------------------------ URM ------
def rms_norm(x: torch.Tensor, eps: float) -> torch.Tensor:
    """Parameter-free RMSNorm computed in float32 (game.py:1223-1229)."""
    dt = x.dtype
    x32 = x.to(torch.float32)
    return (x32 * torch.rsqrt(x32.pow(2).mean(-1, keepdim=True) + eps)).to(dt)


class GameConvSwiGLU(nn.Module):
    """SwiGLU + depthwise causal-trimmed Conv1d over the 16 cells (game.py:1232-1276)."""

    def __init__(self, hidden_size: int, expansion: float, conv_kernel: int = 2):
        super().__init__()
        inter = round(expansion * hidden_size * 2 / 3)
        inter = -(-inter // 8) * 8
        self.inter = inter
        self.gate_up_proj = nn.Linear(hidden_size, 2 * inter, bias=False)
        self.dwconv = nn.Conv1d(inter, inter, kernel_size=conv_kernel, padding=conv_kernel // 2, groups=inter,
                                bias=True)
        self.down_proj = nn.Linear(inter, hidden_size, bias=False)

    def act(self, x: torch.Tensor) -> torch.Tensor | None:
        """The down_proj operand act [B, S, I] on the fused device path (gate_up + SwiGLU + conv in one
        kernel), or None where that path does not apply (the caller then runs forward)."""
        if x.is_cuda:
            from g2048 import urm as _urm  # fused gate_up + SwiGLU + conv (training, g2048_urm.h)
            if _urm.gate_up_swiglu_supported(self, x):
                b, s, h = x.shape
                args = (x.reshape(b * s, h), self.gate_up_proj.weight, self.dwconv.weight.view(-1, 2), self.dwconv.bias)
                act = (_urm.GateUpSwiGLUFn.apply(*args) if torch.is_grad_enabled()
                       else _urm.gate_up_swiglu_nograd(*args))
                return act.view(b, s, self.inter)
        return None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        act = self.act(x)
        if act is not None:
            from g2048 import urm as _urm
            return _urm.project(self.down_proj, act)
        gu = self.gate_up_proj(x)
        if gu.is_cuda:
            from g2048 import urm as _urm  # the device SwiGLU + conv and its backward (g2048_urm.h)
            if _urm.swiglu_conv_supported(gu, x.shape[1], self.inter, self.dwconv.kernel_size[0]):
                b, s, _ = gu.shape
                act = _urm.SwiGLUConvFn.apply(gu.reshape(b * s, 2 * self.inter), self.dwconv.weight.view(-1, 2),
                                              self.dwconv.bias)
                return self.down_proj(act.view(b, s, self.inter))
        gate, up = gu.chunk(2, dim=-1)
        y = F.silu(gate) * up                                        # [B, S, I]
        if self.dwconv.kernel_size[0] == 2:
            # the kernel-2, padding-1 depthwise conv trimmed to S is y_t w0 shifted by one token plus
            # y_t w1 + b: written elementwise (same parameters and math; the library's depthwise
            # Conv1d path for bf16 on this platform is a naive kernel, ~100x slower)
            w = self.dwconv.weight.view(-1, 2)
            prev = F.pad(y, (0, 0, 1, 0))[:, :-1]
            y = prev * w[:, 0] + y * w[:, 1] + self.dwconv.bias
            return self.down_proj(F.silu(y))
        y = self.dwconv(y.transpose(1, 2))[..., : x.shape[1]]       # [B, I, S] trimmed to S
        return self.down_proj(F.silu(y).transpose(1, 2).contiguous())


class GameURMAttention(nn.Module):
    """Bidirectional multi-head self-attention over the 16 cells (game.py:1279-1317)."""

    def __init__(self, hidden_size: int, num_heads: int, dropout: float = 0.0):
        super().__init__()
        self.hidden_size = hidden_size
        self.num_heads = num_heads
        self.head_dim = hidden_size // num_heads
        self.dropout = dropout
        self.qkv_proj = nn.Linear(hidden_size, 3 * hidden_size, bias=False)
        self.o_proj = nn.Linear(hidden_size, hidden_size, bias=False)

    def forward(self, h: torch.Tensor, hb: torch.Tensor | None = None, pre_proj: bool = False):
        """hb: h's bf16 copy when the caller already has it (bf16 autocast: the same operand).
        pre_proj: return (o, True) -- the attention output BEFORE o_proj -- where the device attention
        ran (the caller fuses o_proj into its residual RMSNorm), else (attn(h), False)."""
        b, s, _ = h.shape
        p = self.dropout if self.training else 0.0
        if h.is_cuda:
            from g2048 import urm as _urm  # the HIP attention core and its backward (g2048_urm.h)
            qkv = _urm.project(self.qkv_proj, h if hb is None else hb)
            if _urm.attention_supported(qkv, s, self.hidden_size, self.num_heads, p):
                o = _urm.URMAttentionFn.apply(qkv.reshape(b * s, 3 * self.hidden_size), self.num_heads, p)
                if pre_proj:
                    return o.view(b, s, self.hidden_size), True
                return _urm.project(self.o_proj, o.view(b, s, self.hidden_size))
        else:
            qkv = self.qkv_proj(h)
        q, k, v = qkv.view(b, s, 3, self.num_heads, self.head_dim).permute(2, 0, 3, 1, 4).unbind(0)
        o = F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=False)
        a = self.o_proj(o.transpose(1, 2).reshape(b, s, self.hidden_size))
        return (a, False) if pre_proj else a


class GameURMBlock(nn.Module):
    """post-norm: h = rms(h + attn(h)); h = rms(h + mlp(h))  (game.py:1320-1352)."""

    def __init__(self, config: GameURMConfig):
        super().__init__()
        self.attn = GameURMAttention(config.hidden_dim, config.num_heads, config.dropout)
        self.mlp = GameConvSwiGLU(config.hidden_dim, config.expansion, config.conv_kernel)
        self.norm_eps = config.rms_norm_eps

    def forward(self, h: torch.Tensor, hb: torch.Tensor | None = None, want_hb: bool = False):
        """want_hb: also return the output's bf16 copy (None when not produced) for the next block's
        qkv projection; on the device under bf16 autocast the residual RMSNorm kernel writes it, so
        autocast's cast kernels (and their backward) disappear."""
        if h.is_cuda:
            from g2048 import urm as _urm
            if _urm.linres_supported(self.attn.o_proj, h) and _urm.linres_supported(self.mlp.down_proj, h):
                # o_proj / down_proj fused with their residual RMSNorm (LinResRMSFn, one kernel each)
                o, pre = self.attn(h, hb, pre_proj=True)
                h, hb1 = (_urm.LinResRMSFn.apply(h, o, self.attn.o_proj.weight, self.norm_eps, True) if pre
                          else _urm.ResidualRMSFn.apply(h, o, self.norm_eps, True))
                act = self.mlp.act(hb1)
                if act is not None:
                    res = _urm.LinResRMSFn.apply(h, act, self.mlp.down_proj.weight, self.norm_eps, want_hb)
                else:
                    res = _urm.ResidualRMSFn.apply(h, self.mlp(hb1), self.norm_eps, want_hb)
                return res
        a = self.attn(h, hb)
        if h.is_cuda:
            from g2048 import urm as _urm  # the device residual RMSNorm and its backward (g2048_urm.h)
            if _urm.rms_res_supported(h, a):
                fuse = torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
                if fuse:
                    h, hb1 = _urm.ResidualRMSFn.apply(h, a, self.norm_eps, True)
                    m = self.mlp(hb1)
                else:
                    h = _urm.ResidualRMSFn.apply(h, a, self.norm_eps)
                    m = self.mlp(h)
                if _urm.rms_res_supported(h, m):
                    if want_hb and fuse:
                        return _urm.ResidualRMSFn.apply(h, m, self.norm_eps, True)
                    out = _urm.ResidualRMSFn.apply(h, m, self.norm_eps)
                else:
                    out = rms_norm(h + m, self.norm_eps)
                return (out, None) if want_hb else out
        h = rms_norm(h + a, self.norm_eps)
        out = rms_norm(h + self.mlp(h), self.norm_eps)
        return (out, None) if want_hb else out


class GameURM(nn.Module):
    """Universal-reasoning transformer policy (game.py:1355-1458): shared blocks looped num_loops
    times over the 16 cell tokens, the first num_truncated_loops without gradient, mean-pooled heads."""

    N = N_CELLS
    NUM_ACTIONS = N_ACTIONS

    def __init__(self, config: GameURMConfig):
        super().__init__()
        self.config = config
        h = config.hidden_dim
        self.stem = nn.Sequential(nn.Linear(3, h, bias=False), nn.LayerNorm(h), nn.SiLU())
        self.layers = nn.ModuleList(GameURMBlock(config) for _ in range(config.num_layers))
        self.init_hidden = nn.Parameter(torch.zeros(1, N_CELLS, h))
        nn.init.trunc_normal_(self.init_hidden, std=0.02)
        self.action_head = nn.Linear(h, N_ACTIONS)
        self.value_head = nn.Linear(h, 1)
        for m in self.modules():
            _kaiming_linear(m)

    @property
    def directions(self) -> list[Direction]:
        return list(ACTION_ORDER)

    def get_param_groups(self, value_lr: float, other_lr: float) -> list[dict]:
        """The reference's GameURM has no parameter groups (its trainer refuses URM, train.py:1523-1532);
        these follow GameMLP's split with Muon taking only the 2-D Linear weights: the depthwise conv
        kernels [inter, 1, 2] and init_hidden [1, 16, h] (a direct parameter, not a child module) go
        to the AdamW group with the norms and biases.  init_hidden only feeds the no-grad truncated
        loops when num_truncated_loops >= 1 (game.py:1437-1443), so it never has a gradient and torch's
        AdamW would skip it every step: it joins the group only when it can get one."""
        o2, o1, v2, v1 = _split_param_groups(self, value_lr, other_lr)
        trained = [self.init_hidden] if self.config.num_truncated_loops == 0 else []
        o1["params"] = [p for p in o2["params"] if p.ndim != 2] + o1["params"] + trained
        o2["params"] = [p for p in o2["params"] if p.ndim == 2]
        return [o2, o1, v2, v1]

    def _loop(self, h: torch.Tensor, emb: torch.Tensor, acc=None) -> torch.Tensor:
        hb = None  # bf16 copy of h handed from block to block (device path, bf16 autocast)
        if emb.is_cuda:
            from g2048 import urm as _urm  # h + emb with its bf16 copy in one kernel (g2048_urm.h)
            if _urm.add_cast_supported(h, emb):
                if acc is not None:
                    acc.pending += 1
                h, hb = _urm.AddCastFn.apply(h, emb, acc)
        if hb is None:
            h = h + emb
        last = len(self.layers) - 1
        for i, layer in enumerate(self.layers):
            if i < last:
                h, hb = layer(h, hb, want_hb=True)
            else:
                h = layer(h, hb)
        return h

    def forward(self, inputs: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        if inputs.ndim == 1:
            inputs = inputs.unsqueeze(0)
        if inputs.is_cuda and self.training and not torch.is_grad_enabled():
            from g2048 import urm as _urm  # training-mode no-grad forward (the KL re-forward) in one launch
            out = _urm.train_nograd_forward(self, inputs)
            if out is not None:
                return out
        pooled = self.features(inputs)
        if pooled.is_cuda:
            from g2048 import urm as _urm  # both heads as one device projection (training, g2048_urm.h)
            if _urm.heads_supported(self, pooled):
                return _urm.URMHeadsFn.apply(pooled, self.action_head.weight, self.action_head.bias,
                                             self.value_head.weight, self.value_head.bias)
        return self.action_head(pooled), self.value_head(pooled)

    def features(self, inputs: torch.Tensor) -> torch.Tensor:
        """The pooled features [b, h] the two heads read (game.py:1409-1451): stem, loops, token mean.
        On the device its attention applications share one dropout-counter scope (urm.attn_forward)."""
        if inputs.ndim == 1:
            inputs = inputs.unsqueeze(0)
        if not inputs.is_cuda:
            return self._features(inputs)
        from g2048 import urm as _urm
        with _urm.attn_forward(inputs.device):
            return self._features(inputs)

    def _features(self, inputs: torch.Tensor) -> torch.Tensor:
        b = inputs.shape[0]
        emb = None
        if inputs.is_cuda:
            from g2048 import urm as _urm  # the device training stem and its backward (g2048_urm.h)
            if _urm.stem_supported(self, inputs):
                ln = self.stem[1]
                emb = _urm.StemFn.apply(inputs.reshape(b, 3 * N_CELLS), self.stem[0].weight, ln.weight, ln.bias,
                                        ln.eps).view(b, N_CELLS, -1)
        if emb is None:
            emb = self.stem(inputs.view(b, N_CELLS, 3))
        h = self.init_hidden.expand(b, -1, -1)  # (the reference clones it; every use here is out of place)
        n_trunc = self.config.num_truncated_loops
        if n_trunc > 0:
            with torch.no_grad():
                for _ in range(n_trunc):
                    h = self._loop(h, emb)
            if torch.is_autocast_enabled(h.device.type):
                # autocast caches its bf16 weight casts; the ones made under no_grad carry no
                # autograd history, and reusing them in the loops below would leave every projection
                # weight without a gradient -- drop them so those loops cast again with history
                torch.clear_autocast_cache()
        acc = None
        if emb.is_cuda and torch.is_grad_enabled() and emb.requires_grad:
            from g2048 import urm as _urm  # the loops' emb gradient summed in their backward kernels
            acc = _urm.EmbGradAcc()
        for _ in range(self.config.num_loops - n_trunc):
            h = self._loop(h, emb, acc)
        if h.is_cuda and torch.is_grad_enabled() and h.requires_grad and h.dim() == 3 and h.shape[1] == N_CELLS:
            from g2048 import urm as _urm  # its backward hands the last RMSNorm a [b, h] gradient
            return _urm.MeanPoolFn.apply(h)
        return h.mean(dim=1)


def mlp_flops_per_sample(hidden: int, layers: int) -> int:
    """Forward FLOPs of GameMLP per board (2 x MACs of the linears)."""
    macs = N_FEATURES * hidden + layers * hidden * hidden + hidden * (N_ACTIONS + 1)
    return 2 * macs


def param_count(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


__all__ = ["Direction", "MLPConfig", "GameURMConfig", "ResidualBlock", "GameMLP", "rms_norm", "GameConvSwiGLU",
           "GameURMAttention", "GameURMBlock", "GameURM", "mlp_flops_per_sample", "param_count"]
