"""No kernel of the GameMLP PPO update reads memory it did not write (reference
train.py:414-642): the deterministic form of the intermittent world-2 non-finite grad_norm hunt
(DESIGN.md §7).

Two ranks on one GPU interleave their kernels on the CUs, so between any two launches of one rank a
CU may have run the OTHER rank's kernel, and a stale LDS read then sees that kernel's bytes (env
tables, packed keep bits, Philox words: many are NaN / Inf patterns as fp32 or bf16).  Here that is
made exhaustive and repeatable in one process:

  * every library call of the update (train pass, backward, weight gradients, column sums, gradient
    sum of squares, Muon/AdamW, KL pass) is preceded by g2048_lds_poison on its stream: every CU's
    LDS holds the pattern when the kernel starts;
  * every scratch buffer the updater allocates with torch.empty (activations, dz, dG, keep bits,
    per-block partial rows, the head spill) is filled with the pattern too (stale HBM);
  * the world-size test of fastmlp._colsum is patched to 2, so the world > 1 norm path runs
    (g2048_colsum_batch, then g2048_grad_sumsq_tick into the optimizer's 64 partials, Muon with
    npartials 64) -- the only path of the 2-rank test that a world-1 test does not reach -- and the
    world-1 path (g2048_colsum_batch_sq) as a control;
  * the minibatches are 2 full ones and a ragged padded last one (rows < bs: the device row count).

Every run must be finite and BITWISE equal to the run with zero-filled scratch and no poison, for a
NaN, an Inf and a huge finite pattern: a kernel whose result depends on bytes it did not write
fails here on every box."""

import numpy as np
import pytest
import torch

from test_gpu_ppo_fused import _synthetic_data

pytestmark = pytest.mark.gpu

# fp32 NaN (= a bf16 NaN in each half); fp32 +Inf (bf16 halves +Inf and 0); fp32 / bf16 huge finite
PATTERNS = {"nan": 0x7FC07FC0, "inf": 0x7F800000, "huge": 0x7F7F7F7F}
# the host-side queries of the library (no kernel): no poison launch in front of them
_QUERIES = ("_bytes", "_supported", "_partials", "_blocks", "_offset", "build_info", "lds_poison", "_words")


class _PoisonLib:
    """Stands in for the loaded libg2048 (g2048._lib._lib): every compute entry point is preceded by an
    LDS poison launch on the current stream."""

    def __init__(self, real, word):
        self._real, self._word = real, word
        self.calls = 0

    def __getattr__(self, name):
        fn = getattr(self._real, name)
        if not name.startswith("g2048_") or name.endswith(_QUERIES) or not callable(fn):
            return fn
        real, word = self._real, self._word

        def wrapped(*args):
            real.g2048_lds_poison(torch.cuda.current_stream().cuda_stream, word)
            self.calls += 1
            return fn(*args)
        return wrapped


def _fill(t: torch.Tensor, word: int):
    """Every 32-bit word of t's storage := word (whatever t's dtype)."""
    b = t.view(torch.uint8).reshape(-1) if t.dtype != torch.uint8 else t.reshape(-1)
    n = b.numel() // 4 * 4
    if n:
        b[:n].view(torch.int32).fill_(int(np.array(word, dtype=np.uint32).view(np.int32)))
    if b.numel() > n:
        b[n:].fill_(word & 0xFF)


_SCRATCH = ("x0", "G", "H", "mean", "rstd", "masked", "dz", "dg", "P", "dres", "part_head", "part_kl", "part_ln",
            "part_wg", "dzb", "part_fwd", "part_klp", "part_wh", "wh_spill", "wh_out", "DG", "part_back", "keep",
            "part_pair", "part_mw")


def _run(dev, monkeypatch, word, world2, graph, dropout):
    """One update (3 minibatches, the last ragged) from a fixed state; returns every output bitwise."""
    import agent
    from g2048 import _lib as L
    from g2048 import fastmlp
    from g2048.dist import GradBucket
    from g2048.fastmlp import FusedPPOUpdater
    from g2048.optim import FusedMuonAdamW
    from g2048.ppo import PPOConfig
    if world2:
        monkeypatch.setattr(fastmlp, "world", lambda: (0, 2))
    bs = 2048
    data = _synthetic_data(dev, 2 * bs + 1000, seed=31)
    torch.manual_seed(8)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=196, num_layers=2, dropout=dropout)).to(dev)
    opt = FusedMuonAdamW(m, 1e-3, 1e-4)
    assert opt.supported and opt._cfg.parts == 13
    order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
    gen = torch.Generator(device=dev)
    gen.manual_seed(9)
    bk = GradBucket(order)
    up = FusedPPOUpdater(m, opt, PPOConfig(batch_size=bs, critic=0.2), bk, gen, graph=graph)
    up.force_split = graph  # graph: the 2-rank split capture (g1, eager all-reduce gap, g2)
    orig_alloc = up._alloc

    def alloc(n):
        fresh = up.bs != n
        orig_alloc(n)
        if fresh:  # the torch.empty buffers: poisoned (or zeroed for the reference run)
            for name in _SCRATCH:
                v = getattr(up, name, None)
                for t in (v if isinstance(v, (list, tuple)) else [v]):
                    if torch.is_tensor(t):
                        _fill(t, word or 0)
    monkeypatch.setattr(up, "_alloc", alloc)
    proxy = None
    if word is not None:
        real = L.load()
        proxy = _PoisonLib(real, word)
        monkeypatch.setattr(L, "_lib", proxy)
    try:
        sts = [{k: float(v) for k, v in up.update(data, 0.02).items()} for _ in range(2)]
    finally:
        if proxy is not None:
            monkeypatch.setattr(L, "_lib", proxy._real)
    torch.cuda.synchronize()
    assert up.fused_back and up.wgrad_one_launch and up._sq_done == (not world2)
    if word is not None:
        assert proxy.calls > 0
    out = {"params": torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu(),
           "bucket": bk.flat.detach().cpu().clone(), "norm": float(opt.norm_t), "coef": float(opt.coef_t),
           "state": [t.cpu() for t in _tensors(opt.snapshot())], "stats": sts}
    up.close()
    return out


def _tensors(x):
    if torch.is_tensor(x):
        return [x]
    return [t for y in (x if isinstance(x, (list, tuple)) else []) for t in _tensors(y)]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    return torch.device("cuda:0")


@pytest.mark.parametrize("world2,graph,dropout", [(True, False, 0.0), (True, True, 0.0), (False, False, 0.0),
                                                  (True, False, 0.1)])
def test_update_reads_no_stale_memory(dev, monkeypatch, world2, graph, dropout):
    ref = _run(dev, monkeypatch, None, world2, graph, dropout)
    assert np.isfinite(ref["norm"]) and torch.isfinite(ref["params"]).all()
    assert all(np.isfinite(v) for st in ref["stats"] for v in st.values())
    for name, word in PATTERNS.items():
        got = _run(dev, monkeypatch, word, world2, graph, dropout)
        assert torch.isfinite(got["params"]).all() and np.isfinite(got["norm"]), name
        assert torch.equal(got["params"], ref["params"]), (name, (got["params"] - ref["params"]).abs().max())
        assert torch.equal(got["bucket"], ref["bucket"]), name
        assert got["norm"] == ref["norm"] and got["coef"] == ref["coef"], name
        assert all(torch.equal(a, b) for a, b in zip(got["state"], ref["state"])), name
        assert got["stats"] == ref["stats"], name


def test_clip_coefficient_keeps_a_nan_norm(dev):
    """clip_grad_norm_'s coefficient is torch.clamp(max_norm / (norm + 1e-6), max=1): a NaN norm gives a
    NaN coefficient (torch propagates it into the step), where fminf(c, 1) returned 1 -- an unclipped
    step with finite weights that hid the fault (round-5 verdict).  One NaN gradient entry: the norm
    and the coefficient come out NaN from both clip entry points; an Inf norm clips to 0."""
    import agent
    from g2048 import _lib as L
    from g2048.dist import GradBucket
    from g2048.optim import FusedMuonAdamW
    torch.manual_seed(2)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=64, num_layers=2, dropout=0.0)).to(dev)
    opt = FusedMuonAdamW(m, 1e-3, 1e-4)
    order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
    bk = GradBucket(order)
    bk.flat.normal_()
    bk.flat[17] = float("nan")
    opt.step_clipped(bk.flat, 1.0)
    torch.cuda.synchronize()
    assert np.isnan(float(opt.norm_t)) and np.isnan(float(opt.coef_t))
    norm = torch.zeros((), device=dev)
    coef = torch.zeros((), device=dev)
    part = torch.zeros(64, device=dev)
    L.grad_clip(bk.flat, 1.0, norm, coef, part)
    assert np.isnan(float(norm)) and np.isnan(float(coef))
    bk.flat.normal_()
    bk.flat[5] = float("inf")
    L.grad_clip(bk.flat, 1.0, norm, coef, part)
    assert float(norm) == float("inf") and float(coef) == 0.0
