"""Micro-timings of the pieces of one fused PPO minibatch step (GPU only): the GEMM shapes, the
Muon+AdamW optimizer step and the fused kernels, each in a captured graph replayed many times.

    python tools/micro_update.py
"""

from __future__ import annotations

import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "2048-ppo_amd"))

import torch  # noqa: E402


def timed(fn, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * 10) * 1e3  # us per call


def main():
    import agent
    from g2048 import _lib as L
    from g2048.optim import MuonAdamW
    dev = torch.device("cuda:0")
    M, h = 65536, 196
    bf = torch.bfloat16
    X = torch.randn(M, h, device=dev, dtype=bf)
    X0 = torch.randn(M, 48, device=dev, dtype=bf)
    W = torch.randn(h, h, device=dev, dtype=bf)
    Ws = torch.randn(h, 48, device=dev, dtype=bf)
    G = torch.empty(M, h, device=dev, dtype=bf)
    out = {}
    out["fwd X W^T [65536x196x196]"] = timed(lambda: torch.mm(X, W.t(), out=G))
    out["fwd stem X0 Ws^T [65536x48->196]"] = timed(lambda: torch.mm(X0, Ws.t(), out=G))
    out["bwd dG W [65536x196x196]"] = timed(lambda: torch.mm(X, W, out=G))
    dW = torch.empty(h, h, device=dev)
    part = torch.empty(L.wgrad_partials(M, h, h), device=dev)
    out["wgrad dG^T X (MFMA kernel)"] = timed(lambda: L.wgrad(X, X, part, dW))
    out["wgrad torch.mm out_dtype f32"] = timed(lambda: dW.copy_(torch.mm(X.t(), X, out_dtype=torch.float32)))
    A = torch.randn(h, h, device=dev, dtype=bf)
    C = torch.empty(h, h, device=dev, dtype=bf)
    out["ns gemm 196^3 bf16"] = timed(lambda: torch.mm(A, A, out=C))
    A2 = torch.randn(2, h, h, device=dev, dtype=bf)
    C2 = torch.empty(2, h, h, device=dev, dtype=bf)
    out["ns bmm 2x196^3 bf16"] = timed(lambda: torch.bmm(A2, A2, out=C2))
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=h, num_layers=2, dropout=0.1)).to(dev)
    opt = MuonAdamW(m, 1e-3, 1e-4)
    for p in m.parameters():
        p.grad = torch.randn_like(p) * 1e-2
    out["MuonAdamW.step (all params)"] = timed(opt.step, reps=10)
    g = torch.randn(h, h, device=dev)
    out["newton_schulz 196x196"] = timed(lambda: opt._newton_schulz(g), reps=10)
    y = torch.empty(M, h, device=dev, dtype=bf)
    mean = torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    ln = m.backbone[0].mlp[1]
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    drop = L.make_dropout(0.1, 1, 0, 7, 0, ctr)
    gm_ = torch.empty(M, h, device=dev, dtype=bf)
    out["mlp_fwd fused (res, drop)"] = timed(lambda: L.mlp_fwd(X, W, ln.weight, ln.bias, True, gm_, y, mean, rstd, drop))
    out["mlp_fwd fused (res, no drop)"] = timed(lambda: L.mlp_fwd(X, W, ln.weight, ln.bias, True, gm_, y, mean, rstd,
                                                                  None))
    out["mlp_fwd fused stem (48->196)"] = timed(lambda: L.mlp_fwd(X0, Ws, ln.weight, ln.bias, False, gm_, y, mean, rstd,
                                                                  None))
    out["ln_act_fwd (res, drop)"] = timed(lambda: L.ln_act_fwd(X, ln.weight, ln.bias, X, y, mean, rstd, drop))
    dres = torch.randn(M, h, device=dev)
    pb = torch.empty(L.ln_act_bwd_partials(M, h), device=dev)
    dgam = torch.empty(h, device=dev)
    dbet = torch.empty(h, device=dev)
    out["ln_act_bwd (res, p, drop)"] = timed(lambda: L.ln_act_bwd(dres, X, X, mean, rstd, ln.weight, ln.bias, G, dres, pb,
                                                                  dgam, dbet, drop))
    from g2048.optim import FusedMuonAdamW
    fo = FusedMuonAdamW(m, 1e-3, 1e-4)
    from g2048.dist import GradBucket
    order = [p for p, _ in fo.muon] + [p for grp in fo.adam_groups for p in grp["params"]]
    bk = GradBucket(order)
    bk.flat.normal_()
    out["FusedMuonAdamW.step_clipped"] = timed(lambda: fo.step_clipped(bk.flat, 1.0), reps=10)
    xa = torch.randn(M, h, device=dev, dtype=bf)
    wa, ba, wv, bv = (torch.randn(4, h, device=dev) * 0.05, torch.zeros(4, device=dev), torch.randn(1, h, device=dev),
                      torch.zeros(1, device=dev))
    idx = torch.arange(M, device=dev)
    act = torch.zeros(M, dtype=torch.uint8, device=dev)
    leg = torch.full((M,), 15, dtype=torch.uint8, device=dev)
    olp = torch.full((M, 4), -1.3862944, device=dev)
    adv = torch.randn(M, device=dev)
    ret = torch.randn(M, device=dev)
    batch = L.make_ppo_batch(idx, act, leg, olp, adv, ret)
    beta_t = torch.tensor(0.02, device=dev)
    masked = torch.empty(M, 4, device=dev)
    dx = torch.empty(M, h, device=dev)
    hp = torch.empty(L.ppo_head_partials(M, h), device=dev)
    dwa, dba, dwv, dbv = (torch.empty_like(t) for t in (wa, ba, wv, bv))
    sums = torch.empty(3, device=dev)
    out["ppo_head_loss"] = timed(lambda: L.ppo_head_loss(xa, wa, ba, wv, bv, batch, beta_t, 0.2, 0.2, False, masked, dx,
                                                         hp, dwa, dba, dwv, dbv, sums))
    klo = torch.empty(2, device=dev)
    dzb = torch.empty(M, 8, device=dev)
    out["ppo_head_loss (dz only)"] = timed(lambda: L.ppo_head_loss(xa, wa, ba, wv, bv, batch, beta_t, 0.2, 0.2, False,
                                                                   masked, None, hp, dwa, dba, dwv, dbv, sums, dz=dzb))
    hg = (dzb, wa, wv)
    out["ln_act_bwd (head, drop)"] = timed(lambda: L.ln_act_bwd(None, None, X, mean, rstd, ln.weight, ln.bias, G, dres,
                                                                pb, dgam, dbet, drop, head=hg))
    out["ppo_head_kl"] = timed(lambda: L.ppo_head_kl(xa, wa, ba, masked, hp, klo))
    for k, v in out.items():
        print(f"{k:40s} {v:9.1f} us")


if __name__ == "__main__":
    main()
