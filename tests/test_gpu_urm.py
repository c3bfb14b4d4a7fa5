"""GameURM policy forward on the device (g2048/urm.py over include/g2048_urm.h) vs the reference's
own fp32 forward (tests/golden/urm.npz, game.py:1355-1458) and vs the fp32 module at the default
and README-like sizes; and rollouts driven by it.

Two stated bounds on the fp32 logits / value:
  * vs the fp32 forward (the reference's numbers): |got - ref| <= 0.05 + 0.03 |ref| on the golden
    case; on the random-init module cases max |got - ref| <= 0.08 max|ref| (measured 0.016-0.067 of
    the logit scale; torch's own bf16 autocast of the module errs 0.015-0.098 on the same cases).  The
    projections take bf16 operands (rel. rounding 2^-9) through num_loops x num_layers = 8 post-norm
    blocks; a torch restatement with bf16 rounding at exactly the kernels' points (_emulate below)
    shows the same error (0.042 max on urm.npz), so this is the bf16 operand effect, not the kernels.
  * vs that bf16-rounding restatement: mean |got - emul| <= 3e-3 and max <= 0.06 (fp32 summation
    order and __expf only; an occasional flipped bf16 rounding propagates through the later blocks,
    so the max over thousands of boards is of the order of one bf16 step of the logits)."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden

pytestmark = pytest.mark.gpu

ATOL, RTOL = 0.05, 0.03
EMUL_MEAN, EMUL_MAX = 3e-3, 0.06
SCALE_REL = 0.08


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible: GPU tests must run on an MI355X")
    return torch.device("cuda:0")


def _golden_model(dev, fixture="urm.npz"):
    import agent
    g = golden(fixture)
    h, nl, heads, loops, trunc, k = (int(x) for x in g["config"])
    cfg = agent.GameURMConfig(hidden_dim=h, num_layers=nl, num_heads=heads, num_loops=loops, num_truncated_loops=trunc,
                              conv_kernel=k, dropout=0.0, expansion=float(g["expansion"]), rms_norm_eps=float(g["eps"]))
    m = agent.GameURM(cfg).eval()
    m.load_state_dict({kk[3:]: torch.from_numpy(g[kk]) for kk in g.files if kk.startswith("w::")}, strict=True)
    return m.to(dev), g


def _emulate(m, obs, fused=False):
    """torch fp32 restatement of g2048/urm.py with bf16 rounding where the kernels round: GEMM
    operands, the qkv output, attention probabilities and output, the SwiGLU-conv output, and (only
    on the library path, fused=False) the o_proj / gate_up / down_proj outputs -- the fused
    projections keep those in fp32 into their epilogues."""
    import torch.nn.functional as F
    r = lambda t: t.to(torch.bfloat16).float()  # noqa: E731
    ro = (lambda t: t) if fused else r  # noqa: E731
    c = m.config
    n, h, heads = obs.shape[0], c.hidden_dim, c.num_heads
    hd = h // heads
    with torch.no_grad():
        emb = F.silu(m.stem[1](obs.float().view(n, 16, 3) @ m.stem[0].weight.t()))
        x = m.init_hidden + emb
        for loop in range(c.num_loops):
            for li, blk in enumerate(m.layers):
                qkv = r(r(x) @ r(blk.attn.qkv_proj.weight).t())
                q, k, v = qkv.view(n, 16, 3, heads, hd).permute(2, 0, 3, 1, 4)
                p = r(((q @ k.transpose(-1, -2)) / hd ** 0.5).softmax(-1))
                o = r(p @ v).transpose(1, 2).reshape(n, 16, h)
                x = x + ro(o @ r(blk.attn.o_proj.weight).t())
                x = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.rms_norm_eps)
                ga, up = ro(r(x) @ r(blk.mlp.gate_up_proj.weight).t()).chunk(2, -1)
                a = F.silu(ga) * up
                w, b = blk.mlp.dwconv.weight.view(-1, 2), blk.mlp.dwconv.bias
                prev = torch.cat([torch.zeros_like(a[:, :1]), a[:, :-1]], 1)
                act = r(F.silu(prev * w[:, 0] + a * w[:, 1] + b))
                x = x + ro(act @ r(blk.mlp.down_proj.weight).t())
                x = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.rms_norm_eps)
                if li == len(m.layers) - 1 and loop < c.num_loops - 1:
                    x = x + emb
        pooled = x.mean(1)
        return m.action_head(pooled), m.value_head(pooled).view(-1)


def _check_emul(got_l, got_v, m, obs, fused=False):
    el, ev = _emulate(m, obs, fused)
    d = torch.cat([(got_l - el).abs().reshape(-1), (got_v - ev).abs().reshape(-1)])
    print(f"vs bf16-rounding restatement: mean {d.mean().item():.3g} max {d.max().item():.3g}")
    assert d.mean().item() <= EMUL_MEAN and d.max().item() <= EMUL_MAX


def _check(got, want, what):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    err = np.abs(got - want)
    bound = ATOL + RTOL * np.abs(want)
    assert (err <= bound).all(), f"{what}: max err {err.max():.4g}, worst excess {(err - bound).max():.4g}"
    return err.max()


@pytest.mark.parametrize("fixture", ["urm.npz", "urm64.npz"])
def test_urm_policy_matches_reference_golden(dev, fixture):
    """URMPolicy (the rollout forward; at the default config of urm64.npz the one-launch kernel the
    bench's URM leg times) vs the reference's own fp32 forward: the small h 32 fixture and the
    default GameURMConfig (h 64, BASELINE config 5's policy), 512 boards of the golden games."""
    from g2048.urm import URMPolicy
    m, g = _golden_model(dev, fixture)
    assert URMPolicy.supports(m)
    pol = URMPolicy(m)
    logits, value = pol(torch.from_numpy(g["obs"]).to(dev))
    _check(logits.cpu().numpy(), g["logits"], "logits")
    _check(value.cpu().numpy(), g["value"].reshape(-1), "value")
    _check_emul(logits, value, m, torch.from_numpy(g["obs"]).to(dev), pol.fused)
    # bf16 obs (the rollout's obs buffer) stays within the same bound
    lb, vb = pol(torch.from_numpy(g["obs"]).to(dev).to(torch.bfloat16))
    _check(lb.cpu().numpy(), g["logits"], "logits (bf16 obs)")
    _check(vb.cpu().numpy(), g["value"].reshape(-1), "value (bf16 obs)")


@pytest.mark.parametrize("h,heads,layers,loops,n", [(64, 4, 2, 4, 4096), (64, 2, 2, 4, 1000), (196, 4, 2, 2, 2048),
                                                     (128, 8, 1, 3, 333)])
def test_urm_policy_matches_fp32_module(dev, h, heads, layers, loops, n):
    """Default config (h 64, inter 120, head_dim 16), head_dim 32, head_dim 49 (zero-padded MFMA
    k-steps, unaligned head columns), head_dim 16 with 8 heads; ragged board counts."""
    import agent
    from g2048 import _lib as L
    from g2048.urm import URMPolicy
    torch.manual_seed(h + heads + n)
    m = agent.GameURM(agent.GameURMConfig(hidden_dim=h, num_heads=heads, num_layers=layers, num_loops=loops,
                                          num_truncated_loops=1, dropout=0.0)).to(dev).eval()
    rng = np.random.default_rng(n)
    boards = rng.integers(0, 14, size=(n, 16)).astype(np.int8)
    boards[rng.random(boards.shape) < 0.4] = 0
    obs = torch.empty(n, 48, dtype=torch.float32, device=dev)
    L.obs_encode(torch.from_numpy(boards).to(dev), obs)
    with torch.no_grad():
        ref_l, ref_v = m(obs)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            ac_l, ac_v = m(obs)
    pol = URMPolicy(m)
    got_l, got_v = pol(obs)
    ea = max((ac_l.float() - ref_l).abs().max().item(), (ac_v.float() - ref_v).abs().max().item())
    eg = max((got_l - ref_l).abs().max().item(), (got_v - ref_v.view(-1)).abs().max().item())
    print(f"h={h} heads={heads}: max err vs fp32 {eg:.4g} (torch bf16 autocast {ea:.4g}), "
          f"max |logit| {ref_l.abs().max().item():.3g}")
    _check_emul(got_l, got_v, m, obs, pol.fused)
    assert eg <= SCALE_REL * ref_l.abs().max().item(), eg


def test_urm_policy_weight_sync_and_graph(dev):
    """sync() refreshes the bf16 copies in place; a captured forward replays with the new weights."""
    import agent
    from g2048.urm import URMPolicy
    torch.manual_seed(3)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev).eval()
    pol = URMPolicy(m)
    obs = torch.rand(512, 48, device=dev) * 5
    pol(obs)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        pol(obs)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out_l, out_v = pol(obs)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.01 * torch.randn_like(p))
    pol.sync()
    g.replay()
    torch.cuda.synchronize()
    want_l, want_v = [t.clone() for t in pol(obs)]
    assert torch.equal(out_l, want_l) and torch.equal(out_v, want_v)
    with torch.no_grad():
        ref_l, _ = m(obs)
    _check(want_l.cpu().numpy(), ref_l.cpu().numpy(), "logits after sync")


def test_urm_rollout_drives_envs(dev):
    """Rollout with the URM policy (per-step path: obs -> URM -> sampler -> env step): legal actions,
    finite log-probs, logp rows of the sampler consistent with the URM logits."""
    import agent
    from g2048 import _lib as L
    from g2048.rollout import Rollout, make_policy
    from g2048.urm import URMPolicy
    torch.manual_seed(5)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev).eval()
    pol = make_policy(m)
    assert isinstance(pol, URMPolicy)
    ro = Rollout(2048, 24, dev, seed=9)
    ro.reset()
    b = ro.collect(pol, graph=True)
    torch.cuda.synchronize()
    legal = b.flags[:24] & L.FLAG_LEGAL
    a = b.actions.long()
    assert ((legal.long() >> a) & 1).all()  # every action legal on its board
    assert torch.isfinite(b.logp.gather(2, a.unsqueeze(2))).all()
    assert torch.isfinite(b.value).all() and (b.entropy >= 0).all()
    # the step-0 log-probs are the masked log-softmax of the URM logits of boards[0]
    obs = torch.empty(2048, 48, dtype=torch.bfloat16, device=dev)
    L.obs_encode(b.boards[0], obs)
    lg, _ = pol(obs)
    mask = ((b.flags[0].long().unsqueeze(1) >> torch.arange(4, device=dev)) & 1).bool()
    want = torch.where(mask, lg, torch.tensor(-torch.inf, device=dev)).log_softmax(-1)
    got = b.logp[0]
    np.testing.assert_allclose(torch.where(mask, got, 0).cpu().numpy(), torch.where(mask, want, 0).cpu().numpy(),
                               rtol=1e-5, atol=1e-5)


def test_urm_kernels_reject_bad_arguments(dev):
    from g2048 import _lib as L
    qkv = torch.zeros(32, 3 * 66, dtype=torch.bfloat16, device=dev)
    out = torch.zeros(32, 66, dtype=torch.bfloat16, device=dev)
    with pytest.raises(L.G2048Error):
        L.urm_attention(qkv, out, 4)  # h % 4 != 0
    qkv = torch.zeros(32, 3 * 256, dtype=torch.bfloat16, device=dev)
    out = torch.zeros(32, 256, dtype=torch.bfloat16, device=dev)
    with pytest.raises(L.G2048Error):
        L.urm_attention(qkv, out, 2)  # head_dim 128 > 64


@pytest.mark.parametrize("horizon", [16, 0])
def test_urm_trainer_steps(dev, horizon):
    """VecTrainer with --model-type urm: URMPolicy rollouts, autograd bf16 update with Muon on the
    2-D weights and AdamW on the rest (the conv kernels; init_hidden only with num_truncated_loops 0:
    it has no gradient otherwise, and torch's AdamW skips it); parameters move, metrics finite;
    fixed-horizon and episodic modes."""
    import math
    from g2048.rollout import Rollout  # noqa: F401
    from g2048.trainer import TrainConfig, VecTrainer
    from g2048.urm import URMPolicy
    cfg = TrainConfig(steps=4, episodes=256, horizon=horizon, max_steps=48 if horizon == 0 else None, batch_size=1024,
                      hidden=64, model_type="urm", points=0.1, mono=1.0, rtg_beta=0.99, gamma=0.99, entropy=0.02,
                      critic=0.2, warmup_steps=0)
    tr = VecTrainer(cfg, dev)
    assert isinstance(tr.policy, URMPolicy)
    before = {k: v.detach().clone() for k, v in tr.model.named_parameters()}
    for s in range(2):
        m = tr.train_step(s)
        for k in ("loss", "entropy", "grad_norm", "avg_score", "explained_var"):
            assert math.isfinite(m[k]), (k, m[k])
        assert m["samples"] > 0
    moved = {k for k, v in tr.model.named_parameters() if not torch.equal(v, before[k])}
    assert "layers.0.attn.qkv_proj.weight" in moved and "layers.1.mlp.dwconv.weight" in moved
    assert "init_hidden" not in moved  # num_truncated_loops = 1: no gradient, not in the optimizer


def test_urm_graphed_update_equals_eager(dev):
    """The GameURM minibatch step captured in one hipGraph (urm.training_graph_ok: every op a device
    Function) replays to the same parameters, bitwise, as the eager autograd step: two train steps
    of two trainers from the same seed (dropout 0: the masks are the only draw that differs between
    the capture warm-up and the eager run), 3 minibatches per step incl. a ragged last one."""
    from g2048.trainer import TrainConfig, VecTrainer
    res = []
    for graph in (True, False):
        cfg = TrainConfig(steps=4, episodes=256, horizon=10, batch_size=1024, hidden=64, model_type="urm",
                          dropout=0.0, points=0.1, mono=1.0, rtg_beta=0.99, gamma=0.99, entropy=0.02, critic=0.2,
                          warmup_steps=0, seed=11)
        torch.manual_seed(5)
        tr = VecTrainer(cfg, dev)
        assert tr.ppo.graph and tr.paths["update_graph"]
        tr.ppo.graph = graph  # the eager run keeps the same (graph-safe) MuonAdamW optimizer
        ms = [tr.train_step(s) for s in range(2)]
        res.append(({k: v.detach().clone() for k, v in tr.model.named_parameters()}, ms))
    (pg, mg), (pe, me) = res
    for k in pg:
        assert torch.equal(pg[k], pe[k]), k
    for a, b in zip(mg, me):
        for k in ("loss", "entropy", "grad_norm", "kl_average"):
            assert a[k] == b[k], (k, a[k], b[k])


@pytest.mark.parametrize("h,inter,rows", [(64, 120, 16 * 4097), (32, 64, 16 * 33)])
def test_urm_fused_projection_kernels(dev, h, inter, rows):
    """g2048_urm_linear / _rms / _swiglu vs torch on the same bf16 operands (fp32 reference of the
    same math): bf16 output rounding (2^-8 relative) plus accumulation order."""
    import torch.nn.functional as F
    from g2048 import _lib as L
    g = torch.Generator(device=dev).manual_seed(h)
    xb = torch.randn(rows, h, generator=g, device=dev).to(torch.bfloat16)
    wq = (torch.randn(3 * h, h, generator=g, device=dev) / h ** 0.5).to(torch.bfloat16)
    out = torch.empty(rows, 3 * h, dtype=torch.bfloat16, device=dev)
    L.urm_linear(xb, wq, out)
    ref = xb.float() @ wq.float().t()
    assert ((out.float() - ref).abs() <= 2.0 ** -8 * ref.abs() + 1e-3).all()
    # o_proj + residual + RMSNorm (+ emb)
    wo = (torch.randn(h, h, generator=g, device=dev) / h ** 0.5).to(torch.bfloat16)
    x0 = torch.randn(rows, h, generator=g, device=dev)
    emb = torch.randn(rows, h, generator=g, device=dev)
    for e in (None, emb):
        x = x0.clone()
        xo = torch.empty(rows, h, dtype=torch.bfloat16, device=dev)
        L.urm_linear_rms(xb, wo, x, e, xo, 1e-5)
        v = x0 + xb.float() @ wo.float().t()
        want = v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + 1e-5) + (0 if e is None else e)
        torch.testing.assert_close(x, want, rtol=1e-4, atol=1e-4)
        assert torch.equal(xo, x.to(torch.bfloat16))
    # gate_up + SwiGLU + depthwise conv (kernel 2, per board of 16 tokens) + SiLU
    wgu = (torch.randn(2 * inter, h, generator=g, device=dev) / h ** 0.5).to(torch.bfloat16)
    cw = torch.randn(inter, 2, generator=g, device=dev) * 0.5
    cb = torch.randn(inter, generator=g, device=dev) * 0.1
    act = torch.empty(rows, inter, dtype=torch.bfloat16, device=dev)
    L.urm_linear_swiglu(xb, wgu, cw, cb, act)
    gate, up = (xb.float() @ wgu.float().t()).chunk(2, -1)
    a = (F.silu(gate) * up).view(rows // 16, 16, inter)
    prev = torch.cat([torch.zeros_like(a[:, :1]), a[:, :-1]], 1)
    want = F.silu(prev * cw[:, 0] + a * cw[:, 1] + cb).reshape(rows, inter)
    assert ((act.float() - want).abs() <= 2.0 ** -8 * want.abs() + 2e-3).all(), (act.float() - want).abs().max()
    assert L.urm_linear_supported(2, h, 2 * inter, inter) and not L.urm_linear_supported(0, 196, 588)


def test_urm_fused_and_library_paths_agree(dev):
    """The default config through the fused projections vs the torch.mm path of the same policy."""
    import agent
    from g2048.urm import URMPolicy
    torch.manual_seed(8)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev).eval()
    pol = URMPolicy(m)
    assert pol.fused
    pol.mega = False  # the per-op chain: fused projections vs library projections
    obs = torch.rand(2048, 48, device=dev) * 6
    lf, vf = [t.clone() for t in pol(obs)]
    pol.fused = False
    ll, vl = pol(obs)
    with torch.no_grad():
        ref_l, _ = m(obs)
    e_f, e_l = (lf - ref_l).abs().max().item(), (ll - ref_l).abs().max().item()
    print(f"fused {e_f:.4g} library {e_l:.4g} vs fp32")
    assert e_f <= SCALE_REL * ref_l.abs().max().item() and (lf - ll).abs().max().item() <= 0.1


@pytest.mark.parametrize("layers,loops,n", [(2, 4, 4096), (1, 3, 1001), (2, 2, 17)])
def test_urm_forward_megakernel_matches_kernel_chain(dev, layers, loops, n):
    """g2048_urm_forward (the whole forward in one launch) vs the per-op kernel chain of the same
    policy (same rounding points: bf16 GEMM operands / qkv / attention probabilities and output / act,
    fp32 projections into their epilogues): equal to accumulation-order noise, and within the fp32
    bound of the module; ragged board counts."""
    import agent
    from g2048 import _lib as L
    from g2048.urm import URMPolicy
    torch.manual_seed(layers * 10 + loops)
    m = agent.GameURM(agent.GameURMConfig(num_layers=layers, num_loops=loops, num_truncated_loops=1,
                                          dropout=0.0)).to(dev).eval()
    rng = np.random.default_rng(n)
    boards = rng.integers(0, 14, size=(n, 16)).astype(np.int8)
    boards[rng.random(boards.shape) < 0.4] = 0
    obs = torch.empty(n, 48, dtype=torch.bfloat16, device=dev)
    L.obs_encode(torch.from_numpy(boards).to(dev), obs)
    pol = URMPolicy(m)
    assert pol.mega and pol.fused
    lm, vm = [t.clone() for t in pol(obs)]
    pol.mega = False
    lc, vc = pol(obs)
    dd = torch.cat([(lm - lc).abs().reshape(-1), (vm - vc).abs().reshape(-1)])
    d = dd.max().item()
    with torch.no_grad():
        ref_l, ref_v = m(obs.float())
    e = max((lm - ref_l).abs().max().item(), (vm - ref_v.view(-1)).abs().max().item())
    print(f"megakernel vs chain: max {d:.3g} mean {dd.mean().item():.3g}; vs fp32 {e:.3g}")
    # a flipped bf16 rounding in one of the 8 blocks shows up as ~1e-2 at the logits
    assert d <= 0.04 and dd.mean().item() <= 2e-3 and e <= SCALE_REL * ref_l.abs().max().item()


@pytest.mark.parametrize("n,heads", [(4096, 4), (37, 2)])
def test_urm_attention_backward_matches_sdpa(dev, n, heads):
    """URMAttentionFn (g2048_urm_attention + g2048_urm_attention_bwd, head_dim 16) vs fp32 autograd
    of scaled_dot_product_attention on the same bf16 qkv: outputs and dq / dk / dv within bf16
    rounding (max error <= 2 % of the largest gradient, cosine >= 0.9995)."""
    import torch.nn.functional as F
    from g2048.urm import URMAttentionFn
    h = 16 * heads
    torch.manual_seed(n + heads)
    qkv = (torch.randn(16 * n, 3 * h, device=dev) * 1.5).bfloat16().requires_grad_(True)
    wt = torch.randn(16 * n, h, device=dev)
    out = URMAttentionFn.apply(qkv, heads)
    (out.float() * wt).sum().backward()
    ref_in = qkv.detach().float().requires_grad_(True)
    q, k, v = ref_in.view(n, 16, 3, heads, 16).permute(2, 0, 3, 1, 4).unbind(0)
    o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(16 * n, h)
    (o * wt).sum().backward()
    assert float((out.float() - o.detach()).abs().max()) <= 0.02 * float(o.abs().max())
    for name, sl in (("dq", slice(0, h)), ("dk", slice(h, 2 * h)), ("dv", slice(2 * h, 3 * h))):
        got, want = qkv.grad[:, sl].float().reshape(-1), ref_in.grad[:, sl].reshape(-1)
        assert float((got - want).abs().max()) <= 0.02 * float(want.abs().max()), name
        assert float(torch.nn.functional.cosine_similarity(got, want, dim=0)) >= 0.9995, name


def _attn_keep_oracle(n, heads, p, seed, counter):
    """The device attention-dropout multipliers [n, heads, 16 queries, 16 keys] from the oracle's
    Philox4x32-10 (include/g2048_urm.h: counter {board, head << 8 | query << 2 | key group, call
    counter}, key = seed, words x, y = four 16-bit uniforms, keep iff u >= round(p 2^16))."""
    from oracle import oracle
    thr = int(round(p * 65536))
    km = np.zeros((n, heads, 16, 16), np.float32)
    key = [seed & 0xFFFFFFFF, seed >> 32]
    for b in range(n):
        for hh in range(heads):
            for i in range(16):
                for g in range(4):
                    r = oracle.philox4x32_10([b, (hh << 8) | (i << 2) | g, counter & 0xFFFFFFFF, counter >> 32], key)
                    u = [int(r[0]) & 0xFFFF, int(r[0]) >> 16, int(r[1]) & 0xFFFF, int(r[1]) >> 16]
                    for j in range(4):
                        km[b, hh, i, 4 * g + j] = (1.0 / (1.0 - np.float32(p))) if u[j] >= thr else 0.0
    return km


@pytest.mark.parametrize("n,heads,p", [(64, 4, 0.1), (37, 2, 0.3)])
def test_urm_attention_dropout_matches_masked_autograd(dev, n, heads, p):
    """URMAttentionFn with attention dropout (training mode, game.py:1314) vs fp32 autograd of
    softmax(q k^T / 4) * keep @ v with the keep multipliers regenerated by the oracle's Philox at the
    call's counter: output and dq / dk / dv within the same bf16 bounds as the p = 0 test; the call
    counter advances by one per training forward; the keep fraction is 1 - p within 3 sigma."""
    from g2048 import urm
    from g2048.urm import URMAttentionFn
    h = 16 * heads
    torch.manual_seed(n + heads)
    seed, ctr = urm._attn_drop_state(dev)
    c0 = int(ctr.item())
    qkv = (torch.randn(16 * n, 3 * h, device=dev) * 1.5).bfloat16().requires_grad_(True)
    wt = torch.randn(16 * n, h, device=dev)
    out = URMAttentionFn.apply(qkv, heads, p)
    (out.float() * wt).sum().backward()
    assert int(ctr.item()) == c0 + 1
    km = torch.from_numpy(_attn_keep_oracle(n, heads, p, seed, c0)).to(dev)
    frac = float((km > 0).float().mean())
    sd = (p * (1 - p) / km.numel()) ** 0.5
    assert abs(frac - (1 - p)) <= 3 * sd + 1e-6, frac
    ref_in = qkv.detach().float().requires_grad_(True)
    q, k, v = ref_in.view(n, 16, 3, heads, 16).permute(2, 0, 3, 1, 4).unbind(0)
    pr = torch.softmax(q @ k.transpose(-1, -2) * 0.25, dim=-1) * km
    o = (pr @ v).transpose(1, 2).reshape(16 * n, h)
    (o * wt).sum().backward()
    assert float((out.float() - o.detach()).abs().max()) <= 0.02 * float(o.abs().max())
    for name, sl in (("dq", slice(0, h)), ("dk", slice(h, 2 * h)), ("dv", slice(2 * h, 3 * h))):
        got, want = qkv.grad[:, sl].float().reshape(-1), ref_in.grad[:, sl].reshape(-1)
        assert float((got - want).abs().max()) <= 0.02 * float(want.abs().max()), name
        assert float(torch.nn.functional.cosine_similarity(got, want, dim=0)) >= 0.9995, name


def test_urm_attention_dropout_graph_replay_draws_new_masks(dev):
    """Captured in a hipGraph, every replay reads the bumped device counter: two replays give
    different outputs (different masks), each equal to an eager call at that counter value."""
    from g2048 import urm
    from g2048.urm import URMAttentionFn
    torch.manual_seed(5)
    n, heads, p = 256, 4, 0.1
    qkv = (torch.randn(16 * n, 3 * 16 * heads, device=dev)).bfloat16()
    seed, ctr = urm._attn_drop_state(dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        URMAttentionFn.apply(qkv, heads, p)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = URMAttentionFn.apply(qkv, heads, p)
    outs = []
    for _ in range(2):
        c = int(ctr.item())
        g.replay()
        torch.cuda.synchronize()
        outs.append(out.clone())
        assert int(ctr.item()) == c + 1
        ref = torch.empty_like(out)
        from g2048 import _lib as L
        L.urm_attention(qkv, ref, heads, p, seed, torch.tensor([c], dtype=torch.int64, device=dev))
        torch.cuda.synchronize()
        assert torch.equal(ref, outs[-1])
    assert not torch.equal(outs[0], outs[1])


def test_urm_module_training_uses_device_attention(dev, monkeypatch):
    """GameURM fwd + bwd under bf16 autocast on the device paths (stem, projections with the device
    weight gradient, attention core, residual RMSNorm with the bf16 operand copies, fused gate_up +
    SwiGLU + conv) vs the same model on torch's Linear / SDPA / composite ops, both against the fp32
    module (no autocast) as the truth: every parameter has a gradient (init_hidden aside: the no-grad
    truncated loop overwrites it), and per parameter the device gradient is as close to fp32 as
    torch's own bf16 autocast -- cosine >= autocast's - 0.002 and >= 0.99 (measured in the log)."""
    import agent
    from g2048 import urm
    torch.manual_seed(3)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
    obs = torch.rand(512, 48, device=dev) * 8
    grads = []
    for run in ("device", "torch_bf16", "fp32"):
        m.zero_grad()
        if run == "torch_bf16":  # the reference run: torch's Linear, SDPA and composite ops
            for f in ("attention_supported", "rms_res_supported", "swiglu_conv_supported", "stem_supported",
                      "gate_up_swiglu_supported", "linear_supported"):
                monkeypatch.setattr(urm, f, lambda *a, **k: False)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=run != "fp32"):
            lg, v = m(obs)
        (lg.float().square().sum() + v.float().sum()).backward()
        grads.append({k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None})
    # including the projection weights, whose autocast casts must not come from the no-grad cache
    want = {k for k, _ in m.named_parameters()} - {"init_hidden"}
    assert all(set(g) == want for g in grads)
    cos = torch.nn.functional.cosine_similarity
    for k in sorted(want):
        d, t, f = (g[k].reshape(-1).float() for g in grads)
        if float(f.norm()) == 0:
            continue
        cd, ct = float(cos(d, f, dim=0)), float(cos(t, f, dim=0))
        print(f"{k}: cos(device, fp32) {cd:.5f}  cos(torch bf16, fp32) {ct:.5f}")
        assert cd >= ct - 0.002 and cd >= 0.99, k


@pytest.mark.parametrize("n", [65536, 37])
def test_urm_gate_up_swiglu_fn_matches_unfused(dev, n):
    """GateUpSwiGLUFn (one fused forward kernel) vs the unfused device path it replaces -- the
    autocast gate_up Linear + SwiGLUConvFn -- on the same bf16 input: gu enters both backward
    kernels identically up to the GEMM's fp32 summation order, so act differs by at most a flipped
    bf16 rounding (max <= 2 bf16 steps of |act|max, mean <= 1e-4) and the four gradients agree at
    cosine >= 0.9999 (max error <= 1 % of the largest component)."""
    import agent
    from g2048.urm import GateUpSwiGLUFn, SwiGLUConvFn
    torch.manual_seed(n)
    mlp = agent.GameConvSwiGLU(64, agent.GameURMConfig().expansion, 2).to(dev)
    with torch.no_grad():
        mlp.dwconv.weight.mul_(3.0)
        mlp.dwconv.bias.uniform_(-0.5, 0.5)
    x = torch.randn(16 * n, 64, device=dev).bfloat16()
    g = torch.randn(16 * n, mlp.inter, device=dev)
    params = [mlp.gate_up_proj.weight, mlp.dwconv.weight, mlp.dwconv.bias]
    outs, grads = [], []
    for fused in (True, False):
        mlp.zero_grad()
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                act = GateUpSwiGLUFn.apply(xi, params[0], params[1].view(-1, 2), params[2])
            else:
                gu = mlp.gate_up_proj(xi)
                act = SwiGLUConvFn.apply(gu, params[1].view(-1, 2), params[2])
        (act.float() * g).sum().backward()
        outs.append(act.detach().float())
        grads.append([xi.grad.float()] + [p.grad.detach().clone() for p in params])
    d = (outs[0] - outs[1]).abs()
    print(f"fused gate_up swiglu: act max {d.max().item():.3g} mean {d.mean().item():.3g}")
    assert d.max().item() <= 2 * 2 ** -7 * outs[1].abs().max().item() and d.mean().item() <= 1e-4
    for a, b in zip(*grads):
        a, b = a.reshape(-1).float(), b.reshape(-1).float()
        assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) >= 0.9999
        assert float((a - b).abs().max()) <= 0.01 * float(b.abs().max())


@pytest.mark.parametrize("bcast", [False, True])
def test_urm_add_cast_fn_is_bitwise_the_module_ops(dev, bcast):
    """AddCastFn (a loop start h + emb and its bf16 copy in one kernel; backward sums the fp32 and
    bf16 gradient halves in one kernel) vs the ops it replaces -- h + emb, .to(bfloat16), autograd's
    cast backward and accumulation: forward and every gradient bitwise equal; h contiguous or the
    expanded init_hidden."""
    from g2048.urm import AddCastFn
    torch.manual_seed(3)
    b = 4097
    h0 = torch.randn(1 if bcast else b, 16, 64, device=dev)
    e0 = torch.randn(b, 16, 64, device=dev)
    g1, g2 = torch.randn(b, 16, 64, device=dev), torch.randn(b, 16, 64, device=dev)
    res = []
    for fused in (True, False):
        h = h0.clone().requires_grad_(True)
        e = e0.clone().requires_grad_(True)
        hx = h.expand(b, -1, -1) if bcast else h
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                out, outb = AddCastFn.apply(hx, e)
            else:
                out = hx + e
                outb = out.to(torch.bfloat16)
        ((out * g1).sum() + (outb.float() * g2).sum()).backward()
        res.append((out.detach(), outb.detach(), h.grad, e.grad))
    for a, c in zip(*res):
        assert torch.equal(a, c)


@pytest.mark.parametrize("h,n", [(64, 65536), (32, 4096)])
def test_urm_heads_fn_matches_autocast_heads(dev, h, n):
    """URMHeadsFn (both heads as one projection on g2048_urm_linear, weight gradient on
    g2048_urm_wgrad) vs action_head / value_head under bf16 autocast: outputs at most one bf16 ulp
    apart (round 4: the bias joins the fp32 accumulator, one rounding like autocast; was: one extra bf16
    rounding (2^-7 relative + 1e-3), every gradient at cosine >= 0.9999 with max error <= 1 % of its
    largest component (dW fp32 here, bf16-rounded on the library path)."""
    from g2048.urm import URMHeadsFn
    torch.manual_seed(h + n)
    ha, hv = torch.nn.Linear(h, 4).to(dev), torch.nn.Linear(h, 1).to(dev)
    p = torch.randn(n, h, device=dev)
    ga, gv = torch.randn(n, 4, device=dev), torch.randn(n, 1, device=dev)
    res = []
    for fused in (True, False):
        ha.zero_grad()
        hv.zero_grad()
        pi = p.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            la, lv = (URMHeadsFn.apply(pi, ha.weight, ha.bias, hv.weight, hv.bias) if fused else (ha(pi), hv(pi)))
        assert la.dtype == torch.bfloat16 and lv.dtype == torch.bfloat16
        ((la.float() * ga).sum() + (lv.float() * gv).sum()).backward()
        res.append([la.float(), lv.float(), pi.grad, ha.weight.grad, ha.bias.grad, hv.weight.grad, hv.bias.grad])
    for a, b in zip(res[0][:2], res[1][:2]):
        assert bool(((a - b).abs() <= 2 ** -7 * b.abs() + 1e-6).all())  # one rounding: at most 1 ulp apart
    for a, b in zip(res[0][2:], res[1][2:]):
        a, b = a.reshape(-1).float(), b.reshape(-1).float()
        assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) >= 0.9999
        assert float((a - b).abs().max()) <= 0.01 * float(b.abs().max())


@pytest.mark.parametrize("n", [65536, 37])
def test_urm_gate_up_swiglu_nograd_matches_training_kernel(dev, n):
    """The no-grad truncated loops' gate_up + SwiGLU-conv (round 4: the training epilogue with no gu
    stored) vs the training kernel (gu rounded to bf16 first, autocast's rounding points):
    bitwise equal, and as close to an fp32 restatement as the training kernel."""
    import torch.nn.functional as F

    import agent
    from g2048.urm import GateUpSwiGLUFn, gate_up_swiglu_nograd
    torch.manual_seed(n + 1)
    mlp = agent.GameConvSwiGLU(64, agent.GameURMConfig().expansion, 2).to(dev)
    x = torch.randn(16 * n, 64, device=dev).bfloat16()
    args = (x, mlp.gate_up_proj.weight, mlp.dwconv.weight.view(-1, 2), mlp.dwconv.bias)
    with torch.no_grad():
        got = gate_up_swiglu_nograd(*args).float()
        trn = GateUpSwiGLUFn.apply(*args).float()
        gu = x.float() @ mlp.gate_up_proj.weight.bfloat16().float().t()
        g, u = gu.chunk(2, -1)
        a = (F.silu(g) * u).view(n, 16, -1)
        w = mlp.dwconv.weight.view(-1, 2)
        prev = torch.cat([torch.zeros_like(a[:, :1]), a[:, :-1]], 1)
        ref = F.silu(prev * w[:, 0] + a * w[:, 1] + mlp.dwconv.bias).view(16 * n, -1)
    # round 4: the no-grad path runs the training epilogue without the gu stores -- bitwise equal
    assert torch.equal(got, trn)
    assert (got - ref).abs().mean().item() <= (trn - ref).abs().mean().item() * 1.05


@pytest.mark.parametrize("m,n,k", [(65536 * 16, 192, 64), (65536 * 16, 240, 64), (16 * 37, 64, 120),
                                   (16 * 1001, 64, 64)])
def test_urm_wgrad_matches_fp64(dev, m, n, k):
    """g2048_urm_wgrad (dW = dy^T x over the token rows on MFMA, fp32 accumulate) vs the fp64 product
    of the same bf16 operands: max error <= 1e-5 of the largest |dW| + 1e-6 (fp32 summation of up to
    1 M products), and bitwise deterministic across calls."""
    from g2048.urm import _wgrad
    torch.manual_seed(m + n + k)
    dy = torch.randn(m, n, device=dev).bfloat16()
    x = torch.randn(m, k, device=dev).bfloat16()
    got = _wgrad(dy, x)
    ref = (dy.double().t() @ x.double()).float()
    err = (got - ref).abs().max().item()
    print(f"wgrad {m}x{n}x{k}: max err {err:.3g} of {ref.abs().max().item():.3g}")
    assert err <= 1e-5 * ref.abs().max().item() + 1e-6
    assert torch.equal(got, _wgrad(dy, x))


@pytest.mark.parametrize("k,n", [(64, 192), (64, 64), (120, 64), (32, 96), (32, 32), (64, 32)])
def test_urm_linear_fn_matches_autocast_linear(dev, k, n):
    """URMLinearFn (forward and input gradient on the MFMA projection kernel g2048_urm_linear, weight
    gradient on g2048_urm_wgrad) vs nn.Linear under bf16 autocast (hipBLASLt), for every projection
    shape of GameURM h = 64 / 32 (qkv, o_proj, down_proj).  y and dx are bf16(fp32 sum of bf16
    products) on both paths, only the summation order differs: each element is within one bf16
    rounding (2^-8 relative, + 1e-4 absolute for the fp32 summation where a sum nearly cancels) of
    the fp64 product of the same bf16 operands, and within 2^-7 of autocast's; the weight gradient within the autocast path's own bf16 rounding of dW (ours stays
    fp32): max <= 2^-8 of the largest component.  No library GEMM runs for these shapes."""
    from g2048 import urm as U
    assert U.gemm_supported(n, k)
    torch.manual_seed(7 + k + n)
    rows = 16 * 4099
    lin = torch.nn.Linear(k, n, bias=False).to(dev)
    x = torch.randn(rows, k, device=dev)
    g = torch.randn(rows, n, device=dev)
    res = []
    for fused in (True, False):
        lin.zero_grad()
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = U.URMLinearFn.apply(xi, lin.weight) if fused else lin(xi)
        (y.float() * g).sum().backward()
        res.append((y.detach(), xi.grad.clone(), lin.weight.grad.clone()))
    wb = lin.weight.detach().bfloat16().double()
    y_ref = x.bfloat16().double() @ wb.t()
    dx_ref = g.bfloat16().double() @ wb
    for got, ref, lib in ((res[0][0], y_ref, res[1][0]), (res[0][1], dx_ref, res[1][1])):
        got, lib = got.double(), lib.double()
        # + an absolute 1e-4 for the fp32 summation error where the sum nearly cancels
        assert bool(((got - ref).abs() <= 2 ** -8 * ref.abs() + 1e-4).all())
        assert bool(((got - lib).abs() <= 2 ** -7 * lib.abs() + 2e-4).all())
    d = (res[0][2] - res[1][2]).abs().max().item()
    assert d <= 2 ** -8 * res[1][2].abs().max().item()


def test_urm_train_nograd_forward_matches_module_with_dropout(dev):
    """The training-mode no-grad forward (the PPO update's KL re-forward) runs the one-launch kernel
    with attention dropout.  At the same counter its masks are the autograd module path's
    (URMAttentionFn at counters c .. c + 7 for the 8 block applications): its distance to the module
    output is that of the dropout-free pair (the two paths' different bf16 rounding points: fp32 vs
    bf16 stem, fused epilogues) -- mean within 1.5x + 1e-3 of it, max <= 0.08 of the logit scale like
    the module-vs-fp32 bound -- and well below the distance with the masks of another counter.
    The counter advances by 8 either way; eval mode keeps the module path."""
    import agent
    from g2048 import urm
    torch.manual_seed(11)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.1)).to(dev).train()
    obs = torch.rand(3000, 48, device=dev) * 8
    seed, ctr = urm._attn_drop_state(dev)

    def run(p, grad, c):
        m.config.dropout = p
        for blk in m.layers:
            blk.attn.dropout = p
        ctr.fill_(c)
        with torch.set_grad_enabled(grad), torch.autocast("cuda", dtype=torch.bfloat16):
            lg, v = m(obs)
        assert int(ctr.item()) == c + (8 if p > 0 else 0) or (p == 0 and not grad)
        return torch.cat([lg.float().reshape(-1), v.float().reshape(-1)]).detach()

    c = int(ctr.item()) + 100
    mod0, one0 = run(0.0, True, c), run(0.0, False, c)
    mod1, one1 = run(0.1, True, c), run(0.1, False, c)
    other = run(0.1, False, c + 1000)
    assert "_g2048_train_fwd" in m.__dict__
    d0, d1, dx = (one0 - mod0).abs(), (one1 - mod1).abs(), (other - mod1).abs()
    print(f"one-launch vs module: p=0 max {d0.max().item():.3g} mean {d0.mean().item():.3g}; p=0.1 same masks "
          f"max {d1.max().item():.3g} mean {d1.mean().item():.3g}; other masks mean {dx.mean().item():.3g}")
    assert d1.mean().item() <= 1.5 * d0.mean().item() + 1e-3
    assert d1.max().item() <= 0.08 * mod1.abs().max().item()
    assert dx.mean().item() >= 3 * d1.mean().item()
    m.eval()
    c2 = int(ctr.item())
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        m(obs)
    assert int(ctr.item()) == c2  # eval: no dropout, module path


@pytest.mark.parametrize("rows", [65536 * 16, 33])
def test_urm_residual_rms_fn_bf16_copy(dev, rows):
    """ResidualRMSFn(with_bf16=True): the bf16 copy equals out.bfloat16() bitwise, and the backward
    with gradients on both outputs equals the fp32-only backward of dout + float(doutb) bitwise (the
    kernel adds what autocast's cast backward would have added); only-bf16 and only-fp32 gradients."""
    from g2048.urm import ResidualRMSFn
    torch.manual_seed(rows)
    h = torch.randn(rows, 64, device=dev) * 2
    a = torch.randn(rows, 64, device=dev).bfloat16()
    g32 = torch.randn(rows, 64, device=dev)
    g16 = torch.randn(rows, 64, device=dev).bfloat16()
    for use32, use16 in ((True, True), (False, True), (True, False)):
        h1, a1 = h.clone().requires_grad_(True), a.clone().requires_grad_(True)
        out, outb = ResidualRMSFn.apply(h1, a1, 1e-6, True)
        assert torch.equal(outb, out.detach().bfloat16())
        loss = (out * g32).sum() if use32 else 0.0
        if use16:
            loss = loss + (outb.float() * g16.float()).sum()
        loss.backward()
        h2, a2 = h.clone().requires_grad_(True), a.clone().requires_grad_(True)
        out2 = ResidualRMSFn.apply(h2, a2, 1e-6)
        gt = (g32 if use32 else torch.zeros_like(g32)) + (g16.float() if use16 else 0.0)
        out2.backward(gt)
        assert torch.equal(out.detach(), out2.detach())
        assert torch.equal(h1.grad, h2.grad) and torch.equal(a1.grad, a2.grad)


@pytest.mark.parametrize("n,odt", [(65536, torch.float32), (37, torch.float32), (1000, torch.bfloat16)])
def test_urm_stem_fn_matches_autocast_module(dev, n, odt):
    """StemFn (g2048_urm_stem_fwd / _bwd) vs torch autograd of the stem module under the same bf16
    autocast (game.py:1376-1380): emb within one bf16 step of the pre-LayerNorm activation (the 3-term
    dot product may round the other way; measured max 7e-4, mean 2e-8), and the three parameter
    gradients at cosine >= 0.9999, max error <= 1 % of the largest component."""
    import agent
    from g2048.urm import StemFn
    torch.manual_seed(n)
    m = agent.GameURM(agent.GameURMConfig()).to(dev)
    with torch.no_grad():  # a non-trivial affine LayerNorm
        m.stem[1].weight.uniform_(0.5, 1.5)
        m.stem[1].bias.uniform_(-0.3, 0.3)
    obs = (torch.rand(n, 48, device=dev) * 8).to(odt)
    g = torch.randn(16 * n, 64, device=dev)
    outs, grads = [], []
    for use_dev in (True, False):
        m.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if use_dev:
                e = StemFn.apply(obs, m.stem[0].weight, m.stem[1].weight, m.stem[1].bias, m.stem[1].eps)
            else:
                e = m.stem(obs.view(n, 16, 3)).reshape(16 * n, 64)
        (e.float() * g).sum().backward()
        outs.append(e.detach().float())
        grads.append([p.grad.detach().clone() for p in m.stem.parameters()])
    d = (outs[0] - outs[1]).abs()
    print(f"stem emb: max {d.max().item():.3g} mean {d.mean().item():.3g}")
    assert d.max().item() <= 0.05 and d.mean().item() <= 2e-4
    for a, b in zip(*grads):
        a, b = a.reshape(-1).float(), b.reshape(-1).float()
        assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) >= 0.9999
        assert float((a - b).abs().max()) <= 0.01 * float(b.abs().max())


def test_urm_stem_fn_is_deterministic(dev):
    """Two backward passes on the same input give bitwise equal parameter gradients."""
    from g2048.urm import StemFn
    torch.manual_seed(1)
    w, lw, lb = torch.randn(64, 3, device=dev), torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1
    obs = torch.rand(4096, 48, device=dev) * 8
    g = torch.randn(4096 * 16, 64, device=dev)
    res = []
    for _ in range(2):
        ps = [t.clone().requires_grad_(True) for t in (w, lw, lb)]
        with torch.autocast("cuda", dtype=torch.bfloat16):
            e = StemFn.apply(obs, *ps, 1e-5)
        (e * g).sum().backward()
        res.append([p.grad.clone() for p in ps])
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rows,adt", [(65536 * 16, torch.bfloat16), (1000, torch.float32), (17, torch.bfloat16)])
def test_urm_residual_rms_fn_matches_autograd(dev, rows, adt):
    """ResidualRMSFn (g2048_urm_rms_res_fwd / _bwd) vs fp32 autograd of agent.rms_norm(h + a):
    output and both input gradients within fp32 rounding (the bf16 input gradient within its own
    rounding of the fp32 value)."""
    import agent
    from g2048.urm import ResidualRMSFn
    torch.manual_seed(rows)
    h = (torch.randn(rows, 64, device=dev) * 2).requires_grad_(True)
    a = torch.randn(rows, 64, device=dev).to(adt).requires_grad_(True)
    g = torch.randn(rows, 64, device=dev)
    out = ResidualRMSFn.apply(h, a, 1e-6)
    (out * g).sum().backward()
    hr, ar = h.detach().clone().requires_grad_(True), a.detach().float().requires_grad_(True)
    ref = agent.rms_norm(hr + ar, 1e-6)
    (ref * g).sum().backward()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(h.grad, hr.grad, rtol=1e-4, atol=1e-5)
    tol = 8e-3 if adt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(a.grad.float(), ar.grad, rtol=tol, atol=1e-5 if adt == torch.float32 else 1e-3)


@pytest.mark.parametrize("k,n", [(64, 65536), (120, 65536), (64, 37), (120, 1001)])
@pytest.mark.parametrize("with_bf16", [True, False])
def test_urm_linres_fn_matches_unfused(dev, k, n, with_bf16):
    """LinResRMSFn (o_proj / down_proj + residual + post-norm in one forward kernel) vs the unfused
    device pair it replaces -- URMLinearFn then ResidualRMSFn -- on the same inputs under bf16
    autocast: the projection output enters both as the same bf16 values, so out differs only by the
    RMS sum order (<= 1e-5 relative, the bf16 copy within one rounding); dh / dx / dW -- downstream
    of the bf16 da, where that order can flip a rounding -- at cosine >= 0.99999 with max error <= one
    bf16 step (2^-7) of the largest component."""
    from g2048.urm import LinResRMSFn, ResidualRMSFn, URMLinearFn
    torch.manual_seed(k + n)
    h0 = torch.randn(n, 16, 64, device=dev)
    x0 = (torch.randn(n, 16, k, device=dev)).bfloat16()
    w = torch.nn.Parameter(torch.randn(64, k, device=dev) * k ** -0.5)
    g1 = torch.randn(n, 16, 64, device=dev)
    g2 = torch.randn(n, 16, 64, device=dev)
    res = []
    for fused in (True, False):
        w.grad = None
        h = h0.clone().requires_grad_(True)
        x = x0.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if fused:
                r = LinResRMSFn.apply(h, x, w, 1e-6, with_bf16)
            else:
                a = URMLinearFn.apply(x.reshape(-1, k), w).view(n, 16, 64)
                r = ResidualRMSFn.apply(h, a, 1e-6, with_bf16)
        out, outb = r if with_bf16 else (r, None)
        loss = (out * g1).sum() + ((outb.float() * g2).sum() if with_bf16 else 0.0)
        loss.backward()
        res.append((out.detach(), None if outb is None else outb.detach().float(), h.grad, x.grad.float(), w.grad))
    (o1, b1, *gr1), (o2, b2, *gr2) = res
    assert float((o1 - o2).abs().max()) <= 1e-5 * float(o2.abs().max())
    if with_bf16:
        assert bool(((b1 - b2).abs() <= 2 ** -7 * b2.abs() + 1e-6).all())
    for a, b in zip(gr1, gr2):
        a, b = a.reshape(-1).float(), b.reshape(-1).float()
        assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) >= 0.99999
        assert float((a - b).abs().max()) <= 2 ** -7 * float(b.abs().max())


def test_urm_block_uses_fused_projection_norm(dev, monkeypatch):
    """GameURMBlock under bf16 autocast runs o_proj / down_proj through LinResRMSFn (two calls per
    block application, no ResidualRMSFn) and matches the unfused block within bf16 rounding."""
    import agent
    from g2048 import urm
    torch.manual_seed(11)
    blk = agent.GameURMBlock(agent.GameURMConfig()).to(dev).eval()  # eval: no attention dropout
    h = torch.randn(257, 16, 64, device=dev)
    calls = {"linres": 0, "rms": 0}
    orig_l, orig_r = urm.LinResRMSFn.apply, urm.ResidualRMSFn.apply

    def cnt_l(*a):
        calls["linres"] += 1
        return orig_l(*a)

    def cnt_r(*a):
        calls["rms"] += 1
        return orig_r(*a)

    monkeypatch.setattr(urm.LinResRMSFn, "apply", cnt_l)
    monkeypatch.setattr(urm.ResidualRMSFn, "apply", cnt_r)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        fused = blk(h)
    assert calls == {"linres": 2, "rms": 0}
    monkeypatch.setattr(urm, "linres_supported", lambda lin, hh: False)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        ref = blk(h)
    assert calls["rms"] == 2
    # equal up to the RMS sum order, i.e. at most a flipped bf16 rounding of the next operands
    assert float((fused - ref).abs().max()) <= 2 ** -7 * float(ref.abs().max())


@pytest.mark.parametrize("n,inter", [(65536, 120), (37, 64)])
def test_urm_swiglu_conv_fn_matches_autograd(dev, n, inter):
    """SwiGLUConvFn (g2048_urm_swiglu_conv_fwd / _bwd) vs autograd of the module's composite (bf16
    silu(gate) * up, fp32 kernel-2 conv, silu) on the same bf16 gate_up output: act within one bf16
    step, dgu / dw / db at cosine >= 0.999 and max error <= 2 % of the largest."""
    import torch.nn.functional as F
    from g2048.urm import SwiGLUConvFn
    torch.manual_seed(n + inter)
    gu = (torch.randn(16 * n, 2 * inter, device=dev) * 1.5).bfloat16().requires_grad_(True)
    w = (torch.randn(inter, 2, device=dev) * 0.5).requires_grad_(True)
    b = (torch.randn(inter, device=dev) * 0.1).requires_grad_(True)
    g = torch.randn(16 * n, inter, device=dev)
    act = SwiGLUConvFn.apply(gu, w, b)
    (act.float() * g).sum().backward()
    gr, wr, br = (t.detach().clone().requires_grad_(True) for t in (gu, w, b))
    gate, up = gr.view(n, 16, 2 * inter).chunk(2, dim=-1)
    y = F.silu(gate) * up                                     # bf16, as under autocast
    prev = F.pad(y, (0, 0, 1, 0))[:, :-1]
    ref = F.silu(prev * wr[:, 0] + y * wr[:, 1] + br).reshape(16 * n, inter)
    (ref * g).sum().backward()
    assert float((act.float() - ref.detach()).abs().max()) <= 2 ** -7 * float(ref.abs().max())
    for name, got, want in (("dgu", gu.grad, gr.grad), ("dw", w.grad, wr.grad), ("db", b.grad, br.grad)):
        got, want = got.float().reshape(-1), want.float().reshape(-1)
        assert float(F.cosine_similarity(got, want, dim=0)) >= 0.999, name
        assert float((got - want).abs().max()) <= 0.02 * float(want.abs().max()), name


def test_urm_config5_forward_full_shape(dev):
    """BASELINE config 5's per-GPU shape (65 536 boards of the default GameURM, game.py:1355-1458):
    the one-launch forward (g2048_urm_forward) against the per-op kernel chain on every board, and
    against the fp32 module on a 4 096-board subsample with the bounds stated at the top."""
    import agent
    from g2048 import _lib as L
    from g2048.urm import URMPolicy
    n = 65536
    torch.manual_seed(55)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev).eval()
    rng = np.random.default_rng(5)
    boards = rng.integers(0, 15, size=(n, 16)).astype(np.int8)
    boards[rng.random(boards.shape) < 0.4] = 0
    obs = torch.empty(n, 48, dtype=torch.bfloat16, device=dev)
    L.obs_encode(torch.from_numpy(boards).to(dev), obs)
    pol = URMPolicy(m)
    assert pol.mega and pol.fused
    lm, vm = [t.clone() for t in pol(obs)]
    pol.mega = False
    lc, vc = [t.clone() for t in pol(obs)]
    dd = torch.cat([(lm - lc).abs().reshape(-1), (vm - vc).abs().reshape(-1)])
    print(f"65536 boards, megakernel vs chain: max {dd.max().item():.3g} mean {dd.mean().item():.3g}")
    assert torch.isfinite(lm).all() and torch.isfinite(vm).all()
    assert dd.max().item() <= 0.04 and dd.mean().item() <= 2e-3
    sub = torch.from_numpy(rng.choice(n, 4096, replace=False)).to(dev)
    with torch.no_grad():
        ref_l, ref_v = m(obs.index_select(0, sub).float())
    e = max((lm[sub] - ref_l).abs().max().item(), (vm[sub] - ref_v.view(-1)).abs().max().item())
    print(f"subsample vs fp32 module: {e:.3g} (max |logit| {ref_l.abs().max().item():.3g})")
    assert e <= SCALE_REL * ref_l.abs().max().item()
    _check_emul(lm[sub], vm[sub], m, obs.index_select(0, sub).float(), pol.fused)


def test_urm_config5_trainer_step_full_shape(dev):
    """One --model-type urm train step at config 5's per-GPU shape: 65 536 envs x T = 16, minibatch
    65 536 (16 minibatches of 1 M token rows), dropout 0.1: finite metrics and every parameter moves
    (init_hidden gets no gradient with num_truncated_loops >= 1, game.py:1437-1443, and stays)."""
    import math
    from g2048.trainer import TrainConfig, VecTrainer
    from g2048.urm import URMPolicy
    cfg = TrainConfig(steps=4, episodes=65536, horizon=16, batch_size=65536, hidden=64, model_type="urm",
                      points=0.1, mono=1.0, rtg_beta=0.99, gamma=0.99, entropy=0.02, critic=0.2, warmup_steps=0)
    tr = VecTrainer(cfg, dev)
    assert isinstance(tr.policy, URMPolicy)
    before = {k: v.detach().clone() for k, v in tr.model.named_parameters()}
    m = tr.train_step(1)
    for k in ("loss", "entropy", "grad_norm", "avg_score", "explained_var", "kl_average"):
        assert math.isfinite(m[k]), (k, m[k])
    assert m["samples"] == 65536 * 16
    still = {k for k, v in tr.model.named_parameters() if torch.equal(v, before[k])}
    assert still == {"init_hidden"}, still


# ------------------------------------------------------------------ round 5 ---------------------
@pytest.mark.parametrize("h,n", [(64, 65536), (64, 37), (32, 1000)])
def test_urm_gate_up_recompute_backward_matches_stored_gu(dev, h, n):
    """GateUpSwiGLUFn with gu recomputed in the backward (g2048_urm_gate_up_swiglu_bwd: the forward
    stores act only) vs the round-4 path that stores gu and runs g2048_urm_swiglu_conv_bwd on it:
    the forward is the same kernel (act bitwise), the recomputed gu is the stored one bit for bit, so
    dgu -- and with it dx and dW -- agrees up to the fma contraction of two separately compiled
    kernels (<= 1 bf16 step on a handful of elements); dw / db are summed in another fixed order
    (fp32 rounding: rtol 1e-4)."""
    import agent
    from g2048.urm import GateUpSwiGLUFn
    torch.manual_seed(h * n)
    mlp = agent.GameConvSwiGLU(h, agent.GameURMConfig().expansion, 2).to(dev)
    with torch.no_grad():
        mlp.dwconv.weight.mul_(3.0)
        mlp.dwconv.bias.uniform_(-0.5, 0.5)
    x = torch.randn(16 * n, h, device=dev).bfloat16()
    g = torch.randn(16 * n, mlp.inter, device=dev)
    params = [mlp.gate_up_proj.weight, mlp.dwconv.weight, mlp.dwconv.bias]
    res = []
    try:
        for rec in (True, False):
            GateUpSwiGLUFn.recompute = rec
            mlp.zero_grad()
            xi = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                act = GateUpSwiGLUFn.apply(xi, params[0], params[1].view(-1, 2), params[2])
            (act.float() * g).sum().backward()
            res.append([act.detach().float(), xi.grad.float()] + [p.grad.detach().clone() for p in params])
    finally:
        GateUpSwiGLUFn.recompute = True
    assert torch.equal(res[0][0], res[1][0])  # the same forward kernel
    for k, (a, b) in enumerate(zip(res[0][1:], res[1][1:])):
        a, b = a.reshape(-1).float(), b.reshape(-1).float()
        d = (a - b).abs()
        print(f"grad {k}: max {d.max().item():.3g} of {b.abs().max().item():.3g}, differing {(d > 0).float().mean().item():.2e}")
        if k == 0:  # dx = dgu W: a contraction flip in dgu moves an element by <= 1 bf16 step
            assert float(d.max()) <= 2 ** -7 * float(b.abs().max())
        elif k == 1:  # dW = dgu^T x over 16 n rows: the flips average out in the fp32 sum
            assert float(d.max()) <= 1e-4 * float(b.abs().max())
        else:      # dw0 / dw1 / db: another fixed summation order
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-6 * float(b.abs().max()))


@pytest.mark.parametrize("k,n", [(64, 64), (120, 64), (192, 64), (240, 64), (64, 120)])
def test_urm_linear_t_is_bitwise_the_transposed_copy(dev, k, n):
    """g2048_urm_linear_t (the input gradient dY W with W^T staged by the kernel itself) is bitwise
    g2048_urm_linear on W^T's contiguous copy (the round-4 path): same fragments, same MFMA order."""
    from g2048 import _lib as L
    torch.manual_seed(k + n)
    rows = 16 * 4099
    dy = torch.randn(rows, k, device=dev).bfloat16()
    w = torch.randn(k, n, device=dev).bfloat16()  # [k = out features, n = in features]
    a = torch.empty(rows, n, dtype=torch.bfloat16, device=dev)
    b = torch.empty_like(a)
    L.urm_linear_t(dy, w, a)
    L.urm_linear(dy, w.t().contiguous(), b)
    assert torch.equal(a, b)


def test_urm_emb_accumulation_and_mean_pool_are_bitwise_autograd(dev, monkeypatch):
    """The round-5 backward glue of GameURM: the loops' emb gradient summed inside the AddCastFn
    backward kernels (EmbGradAcc) and the mean-pool's gradient read as [b, h] by the last residual
    RMSNorm backward (MeanPoolFn + g2048_urm_rms_res_bwd3) vs autograd's own accumulation adds and
    materialised mean backward: every parameter gradient bitwise equal (the same sums in the same
    order), in a GameURM forward with 1 truncated and 3 gradient loops."""
    import agent
    from g2048 import urm
    torch.manual_seed(11)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
    obs = torch.randn(512, 48, device=dev)
    ga, gv = torch.randn(512, 4, device=dev), torch.randn(512, 1, device=dev)
    grads = []
    for fused in (True, False):
        if not fused:  # autograd's accumulation (no accumulator) and torch's mean
            monkeypatch.setattr(urm, "EmbGradAcc", lambda: None)
            monkeypatch.setattr(urm.MeanPoolFn, "apply", staticmethod(lambda h: h.mean(dim=1)))
        m.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            la, lv = m(obs)
        ((la.float() * ga).sum() + (lv.float() * gv).sum()).backward()
        grads.append({k: p.grad.clone() for k, p in m.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 10
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


def test_urm_bf16_weight_cache_tracks_the_optimizer(dev):
    """Bf16Weights (round 5): the fused Muon step writes the projection weights' bf16 copies with the
    weights themselves, so after steps the copies equal weight.to(bfloat16) bitwise, and the training
    Functions read them instead of casting."""
    import agent
    from g2048 import urm
    from g2048.dist import GradBucket
    from g2048.optim import FusedMuonAdamW
    torch.manual_seed(5)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
    opt = FusedMuonAdamW(m, 1e-3, 1e-4)
    assert opt.supported
    order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
    bk = GradBucket(order)
    cache = urm.attach_bf16_weights(m, opt)
    assert cache is not None and len(cache.pairs) == 4 * len(m.layers)
    for s in range(3):
        bk.flat.copy_(torch.randn(bk.flat.shape, generator=torch.Generator().manual_seed(s)).to(dev) * 1e-2)
        opt.step_clipped(bk.flat, 1.0)
    torch.cuda.synchronize()
    for w, t in cache.pairs:
        assert torch.equal(t, w.detach().to(torch.bfloat16))
        assert urm.bf16_weight(w) is t
    cache.detach()


def _urm_columns(dev, M, seed=0):
    """Random trajectory columns of M rows (boards, a legal action, logp, adv, ret) as the update reads them."""
    from oracle import oracle as O
    g = np.random.default_rng(seed)
    boards = g.integers(0, 10, size=(M, 16)).astype(np.int8)
    legal = O.legal_mask(boards)
    legal[legal == 0] = 1
    acts = np.array([g.choice([a for a in range(4) if m >> a & 1]) for m in legal], np.uint8)
    logp = np.log(g.dirichlet(np.ones(4), size=M)).astype(np.float32)
    return {"boards": torch.from_numpy(boards).to(dev), "actions": torch.from_numpy(acts).to(dev),
            "legal": torch.from_numpy(legal).to(dev), "logp": torch.from_numpy(logp).to(dev),
            "adv": torch.from_numpy(g.normal(size=M).astype(np.float32)).to(dev),
            "ret": torch.from_numpy(g.normal(size=M).astype(np.float32)).to(dev)}


@pytest.mark.parametrize("m,pdt", [(4096, torch.float32), (3001, torch.float32), (1000, torch.bfloat16)])
def test_urm_head_loss_fn_matches_torch_loss(dev, m, pdt):
    """URMHeadLossFn (g2048_urm_head_loss / _bwd, round 5) vs the round-4 path it replaces -- URMHeadsFn
    under bf16 autocast + ppo.ppo_losses + autograd -- on the same pooled features and columns: the
    logits follow autocast's rounding points in both (bf16 operands, one rounding of the biased fp32
    sum), so they differ only where the two dot-product orders round across a bf16 step; measured
    bounds: loss / loss sums within 1e-4 relative, masked logits within one bf16 step, dpooled and
    the head gradients at cosine >= 0.9999 and max error <= 1 % of their scale."""
    import agent
    from g2048 import _lib as L
    from g2048.ppo import invalid_from_legal, ppo_losses
    from g2048.urm import URMHeadsFn
    from g2048.urmppo import URMHeadLossFn
    torch.manual_seed(m)
    mod = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
    with torch.no_grad():
        mod.action_head.weight.mul_(4.0)
        mod.action_head.bias.uniform_(-0.5, 0.5)
        mod.value_head.bias.uniform_(-0.5, 0.5)
    cols = _urm_columns(dev, 3 * m, seed=m)
    idx = torch.randperm(3 * m, device=dev)[:m].contiguous()
    pooled = (torch.randn(m, 64, device=dev) * 1.5).to(pdt)
    beta = torch.tensor(0.02, device=dev)
    heads = [mod.action_head.weight, mod.action_head.bias, mod.value_head.weight, mod.value_head.bias]
    # reference: the round-4 modules + torch loss
    p_ref = pooled.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        if m % 16 == 0:
            lg, v = URMHeadsFn.apply(p_ref, *heads)
        else:  # (URMHeadsFn takes whole boards of 16 rows: autocast's own Linear, the same rounding points)
            lg, v = mod.action_head(p_ref), mod.value_head(p_ref)
    inv = invalid_from_legal(cols["legal"][idx])
    loss_ref, parts = ppo_losses(lg.float(), v.float(), cols["actions"][idx], inv, cols["logp"][idx], cols["adv"][idx],
                                 cols["ret"][idx], beta, 0.2, 0.2)
    loss_ref.backward()
    g_ref = [p.grad.clone() for p in heads]
    for p in heads:
        p.grad = None
    # the device loss
    sync = torch.zeros(1, dtype=torch.int32, device=dev)
    run = {"batch": L.make_ppo_batch(idx, cols["actions"], cols["legal"], cols["logp"], cols["adv"], cols["ret"]),
           "beta": beta, "critic": 0.2, "clip": 0.2, "sync": sync}
    p_dev = pooled.clone().requires_grad_(True)
    loss = URMHeadLossFn.apply(p_dev, *heads, run)
    loss.backward()
    torch.cuda.synchronize()
    assert int(sync.item()) == 0  # the ticket is back at zero after both kernels
    assert abs(float(loss) - float(loss_ref)) <= 1e-4 * abs(float(loss_ref)) + 1e-6, (float(loss), float(loss_ref))
    want = torch.stack([parts["ppo"].sum(), parts["entropy"].sum(), parts["vloss"].sum()])
    torch.testing.assert_close(run["sums"], want, rtol=1e-4, atol=1e-3)
    mk, mk_ref = run["masked"], parts["masked"]
    assert torch.equal(torch.isinf(mk), torch.isinf(mk_ref))
    fin = torch.isfinite(mk_ref)
    assert float((mk[fin] - mk_ref[fin]).abs().max()) <= 2 ** -7 * float(mk_ref[fin].abs().max())
    for name, a, b in [("dpooled", p_dev.grad, p_ref.grad)] + [(n, p.grad, r) for n, p, r in
                                                                zip(("dwa", "dba", "dwv", "dbv"), heads, g_ref)]:
        a, b = a.float().reshape(-1), b.float().reshape(-1)
        print(f"{name}: max {float((a - b).abs().max()):.3g} of {float(b.abs().max()):.3g}")
        assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) >= 0.9999, name
        assert float((a - b).abs().max()) <= 0.01 * float(b.abs().max()) + 1e-7, name


def test_urm_kl_stats_matches_torch(dev):
    """g2048_urm_kl_stats vs the torch statistics of PPOUpdater._post (ppo.kl_old_new + the stacked
    minibatch statistics) on the same masked / new logits, sums and grad norm: every entry of the
    accumulated statistics within 1e-5 relative, kl_max as the max."""
    from g2048 import _lib as L
    from g2048.ppo import kl_old_new
    torch.manual_seed(9)
    m = 5000
    legal = torch.randint(1, 16, (m,), device=dev, dtype=torch.int32)
    inv = ((legal.unsqueeze(-1) >> torch.arange(4, device=dev)) & 1) == 0
    old = (torch.randn(m, 4, device=dev) * 2).masked_fill(inv, float("-inf"))
    new = torch.randn(m, 4, device=dev) * 2
    sums = torch.tensor([12.5, 3000.0, 800.0], device=dev)
    gn = torch.tensor(0.75, device=dev)
    beta = torch.tensor(0.02, device=dev)
    stats = torch.zeros(9, device=dev)
    sync = torch.zeros(1, dtype=torch.int32, device=dev)
    part = torch.empty(2 * ((m + 255) // 256), device=dev)
    for _ in range(2):
        L.urm_kl_stats(old, new, sums, gn, beta, 0.2, stats, part, sync)
    kl = kl_old_new(old, new, inv)
    s_ppo, s_ent, s_v = (sums / m).tolist()
    one = torch.tensor([-(s_ppo - 0.2 * s_v + 0.02 * s_ent), -s_ppo, -0.02 * s_ent, 0.2 * s_v, 0.75, s_ent,
                        float(kl.sum()), float(kl.mean()), 0.0], device=dev)
    want = 2 * one
    want[8] = kl.max()
    torch.testing.assert_close(stats, want, rtol=1e-5, atol=1e-6)
    assert int(sync.item()) == 0


def test_urm_direct_weight_grads_are_bitwise_autograd(dev):
    """urm.direct_weight_grads (round 5): the shared weights' gradients added into .grad inside the
    producing kernels (g2048_urm_wgrad_acc, g2048_urm_gate_up_swiglu_bwd_acc) equal, bit for bit,
    autograd's accumulation of the returned gradients -- every parameter, with attention dropout (both
    runs at the same mask counter) and a truncated loop."""
    import agent
    from g2048 import urm
    torch.manual_seed(3)
    mod = agent.GameURM(agent.GameURMConfig(dropout=0.1)).to(dev).train()
    obs = (torch.rand(2048, 48, device=dev) * 8).bfloat16()
    wt = torch.randn(2048, 64, device=dev)
    _, ctr = urm._attn_drop_state(dev)
    c0 = int(ctr.item())
    grads = []
    for direct in (False, True):
        ctr.fill_(c0)
        for p in mod.parameters():
            p.grad = torch.zeros_like(p)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            if direct:
                with urm.direct_weight_grads():
                    pooled = mod.features(obs)
                    (pooled.float() * wt).sum().backward()
            else:
                pooled = mod.features(obs)
                (pooled.float() * wt).sum().backward()
        grads.append({k: p.grad.clone() for k, p in mod.named_parameters()})
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k
    assert float(grads[1]["layers.0.mlp.gate_up_proj.weight"].abs().sum()) > 0


def test_urm_attention_forward_scope_draws_the_per_application_masks(dev):
    """urm.attn_forward (round 5): inside one GameURM forward the attention applications read the
    forward's counter snapshot + their index and the counter is bumped once at the end -- the same
    masks as round 4's snapshot-and-bump per application (the Function outside a scope): pooled
    features and every gradient bitwise equal, the counter advanced by the same count."""
    import agent
    from g2048 import urm
    torch.manual_seed(4)
    mod = agent.GameURM(agent.GameURMConfig(dropout=0.2)).to(dev).train()
    obs = (torch.rand(1024, 48, device=dev) * 8).bfloat16()
    wt = torch.randn(1024, 64, device=dev)
    _, ctr = urm._attn_drop_state(dev)
    c0 = int(ctr.item())
    res = []
    for scoped in (True, False):
        ctr.fill_(c0)
        mod.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            pooled = mod.features(obs) if scoped else mod._features(obs)
            (pooled.float() * wt).sum().backward()
        res.append((pooled.detach().clone(), int(ctr.item()),
                    {k: p.grad.clone() for k, p in mod.named_parameters() if p.grad is not None}))
    assert torch.equal(res[0][0], res[1][0])
    assert res[0][1] == res[1][1] == c0 + 8
    for k in res[0][2]:
        assert torch.equal(res[0][2][k], res[1][2][k]), k


def test_urm_ppo_updater_matches_generic_updater(dev):
    """URMPPOUpdater (device loss kernels, direct weight gradients, one-launch KL statistics) vs
    PPOUpdater (torch loss + autograd) from the same weights on the same minibatches (torch-op
    MuonAdamW for both, dropout 0): the update directions agree (cosine >= 0.999 per 2-D weight, norm
    within 2 %; 1-D parameters within 2e-3 of their step) and the statistics within 1e-3 relative
    (the KL statistics: kl_total / kl_average 1e-2, kl_max 5e-2, see below) --
    what is left is the heads' dot-product order and the kernels' summation orders, amplified by
    Muon's bf16 Newton-Schulz."""
    import math

    import agent
    from g2048.dist import GradBucket
    from g2048.optim import MuonAdamW
    from g2048.ppo import PPOConfig, PPOUpdater
    from g2048.urmppo import URMPPOUpdater
    cols = _urm_columns(dev, 4096, seed=7)

    def enc(b):
        from g2048 import _lib as L
        o = torch.empty(b.shape[0], 48, dtype=torch.float32, device=dev)
        L.obs_encode(b.contiguous(), o)
        return o
    res = []
    for cls in (URMPPOUpdater, PPOUpdater):
        torch.manual_seed(2)
        mod = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
        opt = MuonAdamW(mod, 1e-3, 1e-4)
        order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
        gen = torch.Generator(device=dev)
        gen.manual_seed(5)
        init = {k: p.detach().clone() for k, p in mod.named_parameters()}
        up = cls(mod, opt, PPOConfig(batch_size=2048, critic=0.2), GradBucket(order), gen, graph=False)
        st = {k: float(v) for k, v in up.update(cols, 0.02, enc).items()}
        res.append(({k: p.detach() - init[k] for k, p in mod.named_parameters()}, st))
    (d0, s0), (d1, s1) = res
    for k in d0:
        a, b = d0[k].reshape(-1), d1[k].reshape(-1)
        if d0[k].ndim == 2 and b.norm() > 0:
            assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) >= 0.999, k
            assert math.isclose(float(a.norm()), float(b.norm()), rel_tol=0.02), k
        else:
            assert float((a - b).abs().max()) <= 2e-3 * float(b.abs().max()) + 1e-9, k
    # the KL statistics measure the update itself, and Muon's orthogonalisation (U V^T of the
    # gradient) amplifies rounding in the gradient's weak singular directions: with the one-pass
    # residual-RMSNorm backward in both updaters (round 5) the gradients agree with the three-launch
    # ones at cosine >= 0.9999998 while the weakest matrix's update turns to cosine 0.963
    # (tools/urm_grad_fused_check.py, tools/urm_stats_spread.py) -- so the KL statistics of two
    # updaters that differ only in the heads' / loss kernels' summation orders carry that noise:
    # measured kl_total / kl_average 0.33 %, kl_max 2.5 % (0.06 / 0.9 % with the three-launch
    # backward); the first-order statistics stay within 1e-3
    for k in s0:
        tol = 5e-2 if k == "kl_max" else 1e-2 if k.startswith("kl") else 1e-3
        assert math.isclose(s0[k], s1[k], rel_tol=tol, abs_tol=1e-6), (k, s0[k], s1[k])


def test_urm_ppo_updater_minibatch_gradients_match_autocast(dev):
    """One minibatch's gradients (before clipping / the optimizer) of URMPPOUpdater -- device loss
    and head kernels, fused projections, direct weight gradients -- against PPOUpdater under bf16
    autocast (torch loss + autograd) and PPOUpdater in fp32, same weights, same rows, dropout 0.  Bound
    derived from bf16 rounding: per parameter, the URM updater's relative distance to the fp32
    gradient is at most 1.1 x autocast's own + 1e-4 (autocast is the arithmetic the URM kernels
    restate: the same bf16 operands and rounding points, other summation orders), and the two bf16
    paths within URM_GRAD_REL of each other (relative L2)."""
    import agent
    from g2048.dist import GradBucket
    from g2048.optim import MuonAdamW
    from g2048.ppo import PPOConfig, PPOUpdater
    from g2048.urmppo import URMPPOUpdater
    cols = _urm_columns(dev, 2048, seed=11)
    idx = torch.randperm(2048, device=dev, generator=torch.Generator(device=dev).manual_seed(3))

    def enc(b):
        from g2048 import _lib as L
        o = torch.empty(b.shape[0], 48, dtype=torch.float32, device=dev)
        L.obs_encode(b.contiguous(), o)
        return o
    grads = {}
    for name, cls, amp in (("urm", URMPPOUpdater, torch.bfloat16), ("autocast", PPOUpdater, torch.bfloat16),
                           ("fp32", PPOUpdater, None)):
        torch.manual_seed(2)
        mod = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev).train()
        with torch.no_grad():  # heads away from their init scale: a loss gradient in every head row
            mod.action_head.weight.mul_(4.0)
            mod.action_head.bias.uniform_(-0.5, 0.5)
        opt = MuonAdamW(mod, 1e-3, 1e-4)
        order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
        up = cls(mod, opt, PPOConfig(batch_size=2048, critic=0.2, amp_dtype=amp), GradBucket(order), None,
                 graph=False)
        up._pre(idx, cols, torch.tensor(0.02, device=dev), enc)
        torch.cuda.synchronize()
        grads[name] = {k: p.grad.detach().double().reshape(-1).clone() for k, p in mod.named_parameters()
                       if p.grad is not None and float(p.grad.abs().sum()) > 0}
    assert set(grads["urm"]) == set(grads["autocast"]) == set(grads["fp32"])
    rows, bad = [], []
    for k in grads["fp32"]:
        u, a, f = grads["urm"][k], grads["autocast"][k], grads["fp32"][k]
        e_u, e_a = float((u - f).norm() / f.norm()), float((a - f).norm() / f.norm())
        d_ua = float((u - a).norm() / a.norm())
        rows.append(f"{k}: |urm - fp32| {e_u:.3e}  |autocast - fp32| {e_a:.3e}  |urm - autocast| {d_ua:.2e}")
        if e_u > 1.1 * e_a + 1e-4 or d_ua > URM_GRAD_REL:
            bad.append(rows[-1])
    print("\n".join(rows))
    assert not bad, bad


# the URM updater's minibatch gradients against autocast's: measured on MI355X (profiles/r06n/
# urm_grads2.log) within 5.7e-6 relative of each other for every parameter (the heads within 2.3e-7,
# value_head.bias equal), each at the same distance (4 digits) from the fp32 gradient as autocast's
# own (0.26-2.3 % for the bf16 paths): the head / loss kernels and the autograd loss differ only in
# summation order.  Bound: ~10 x the largest measured difference
URM_GRAD_REL = 5e-5


@pytest.mark.parametrize("n,heads,p", [(4099, 4, 0.0), (1000, 4, 0.1), (333, 2, 0.2)])
def test_urm_attention_board_kernels_are_bitwise_the_head_kernels(dev, n, heads, p):
    """The one-wave-per-board attention kernels (round 5: the board's qkv / dO rows staged in LDS by
    16-byte loads) vs the per-(board, head) kernels they replace for head_dim 16 -- which still run on
    8-byte-aligned (not 16) buffers: forward output and dq / dk / dv bitwise equal, with and without
    dropout (the same mask counter)."""
    from g2048 import _lib as L
    from g2048 import urm
    torch.manual_seed(n)
    h = 16 * heads
    qkv = (torch.randn(16 * n, 3 * h, device=dev) * 1.5).bfloat16()
    dout = torch.randn(16 * n, h, device=dev).bfloat16()
    seed, _ = urm._attn_drop_state(dev)
    ctr = torch.tensor([77], dtype=torch.int64, device=dev)

    def shifted(t):  # the same values at an address 8 bytes past a 16-byte boundary
        buf = torch.empty(t.numel() + 8, dtype=t.dtype, device=dev)
        v = buf[4:4 + t.numel()].view(t.shape)
        v.copy_(t)
        assert v.data_ptr() % 16 == 8
        return v
    res = []
    for aligned in (True, False):
        q = qkv if aligned else shifted(qkv)
        d = dout if aligned else shifted(dout)
        out = torch.empty(16 * n, h, dtype=torch.bfloat16, device=dev)
        dq = torch.empty_like(qkv) if aligned else shifted(torch.zeros_like(qkv))
        if aligned:
            out_t = out
        else:
            out_t = shifted(torch.zeros_like(out))
        L.urm_attention(q, out_t, heads, p, seed, ctr, offset=3)
        L.urm_attention_bwd(q, d, dq, heads, p, seed, ctr, offset=3)
        res.append((out_t.clone(), dq.clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("k,n", [(64, 65536), (120, 65536), (64, 37), (120, 1001)])
@pytest.mark.parametrize("grad_src", ["dout", "dout+bf16", "bf16", "pool"])
def test_urm_linres_fused_backward(dev, k, n, grad_src):
    """LinResRMSFn's one-pass backward (g2048_urm_linres_bwd: residual-RMSNorm backward, dX and dW from
    the bf16 da held on chip) vs its three-launch backward (g2048_urm_rms_res_bwd2, g2048_urm_linear_t,
    g2048_urm_wgrad) on the same forward: dh within fp32 rounding (the row mean summed in another
    order, <= 1e-5 of the largest component); dx BITWISE the projection kernel's dx of the fused
    path's own bf16(dh) (same fragments, same k order); dW within fp32 summation order of the
    unfused weight-gradient kernel on that bf16(dh); and fused vs three-launch dx / dW at cosine
    >= 0.99999 with max error <= one bf16 step (2^-7) of the largest component (da can flip a
    rounding).  Gradient sources: fp32 dout, fp32 + the bf16 copy's gradient, the bf16 one alone, and
    the mean-pool's broadcast [b, 64] gradient (odd board counts: the kernel's ragged row pair)."""
    from g2048 import _lib as L
    from g2048.urm import LinResRMSFn, MeanPoolFn
    torch.manual_seed(k + 7 * n)
    h0 = torch.randn(n, 16, 64, device=dev)
    x0 = torch.randn(n, 16, k, device=dev).bfloat16()
    w = torch.nn.Parameter(torch.randn(64, k, device=dev) * k ** -0.5)
    g1 = torch.randn(n, 16, 64, device=dev)
    g2 = torch.randn(n, 16, 64, device=dev)
    gp = torch.randn(n, 64, device=dev)
    want_b = grad_src in ("dout+bf16", "bf16")
    res = []
    for fused in (True, False):
        LinResRMSFn.fused_bwd = fused
        try:
            w.grad = None
            h = h0.clone().requires_grad_(True)
            x = x0.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                r = LinResRMSFn.apply(h, x, w, 1e-6, want_b)
            out, outb = r if want_b else (r, None)
            if grad_src == "pool":
                loss = (MeanPoolFn.apply(out) * gp).sum()
            else:
                loss = (outb.float() * g2).sum() if want_b else 0.0
                if grad_src != "bf16":
                    loss = loss + (out * g1).sum()
            loss.backward()
            res.append((h.grad.clone(), x.grad.float().clone(), w.grad.clone()))
        finally:
            LinResRMSFn.fused_bwd = True
    (dh1, dx1, dw1), (dh2, dx2, dw2) = res
    assert float((dh1 - dh2).abs().max()) <= 1e-5 * float(dh2.abs().max())
    # the fused pass's own products, recomputed from the dh it wrote
    da = dh1.reshape(-1, 64).to(torch.bfloat16).contiguous()
    wb = w.detach().to(torch.bfloat16).contiguous()
    dx_ref = torch.empty(16 * n, k, dtype=torch.bfloat16, device=dev)
    L.urm_linear_t(da, wb, dx_ref)
    assert torch.equal(dx1.reshape(-1, k).bfloat16(), dx_ref)
    dw_ref = torch.empty(64, k, dtype=torch.float32, device=dev)
    part = torch.empty(L.urm_wgrad_partials(16 * n, 64, k), dtype=torch.float32, device=dev)
    L.urm_wgrad(da, x0.reshape(-1, k).contiguous(), dw_ref, part)
    assert float((dw1 - dw_ref).abs().max()) <= 1e-5 * float(dw_ref.abs().max())
    for a, b in ((dx1, dx2), (dw1, dw2)):
        a, b = a.reshape(-1).float(), b.reshape(-1).float()
        assert float(torch.nn.functional.cosine_similarity(a, b, dim=0)) >= 0.99999
        assert float((a - b).abs().max()) <= 2 ** -7 * float(b.abs().max())
