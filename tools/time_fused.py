"""HIP-event timings of the fused GameMLP minibatch kernels at the bench's minibatch (65 536 rows,
h 196, dropout 0.1): the train pass (g2048_ppo_forward_loss), the KL pass (g2048_ppo_forward_kl),
the fused backward (g2048_ppo_backward), each replayed from a hipGraph of 10 launches.  GPU only.

    python tools/time_fused.py [m] [h]
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def timed(fn, reps=30):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(10):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * 10) * 1e3


def main():
    import os
    from g2048 import _lib as L
    if os.environ.get("G2048_LIB"):  # A/B timing against another build of the library
        L._lib = L.load(os.environ["G2048_LIB"])  # every wrapper then calls this build
    ms = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536").split(",")]
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 196
    for m in ms:
        run(L, m, h)


def run(L, m, h):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    bf, f32 = torch.bfloat16, torch.float32
    rnd = lambda *s: torch.randn(*s, generator=g, device=dev)  # noqa: E731
    w = [(rnd(h, 48) / 48 ** 0.5).to(bf)] + [(rnd(h, h) / h ** 0.5).to(bf) for _ in range(2)]
    gam = [torch.rand(h, generator=g, device=dev) + 0.5 for _ in range(3)]
    bet = [rnd(h) * 0.1 for _ in range(3)]
    wa, ba, wv, bv = rnd(4, h) * 0.1, rnd(4) * 0.1, rnd(1, h) * 0.1, rnd(1) * 0.1
    M = 2 * m
    rng = np.random.default_rng(0)
    boards = torch.from_numpy(rng.integers(0, 12, size=(M, 16)).astype(np.int8)).to(dev)
    legal = torch.full((M,), 15, dtype=torch.uint8, device=dev)
    actions = torch.from_numpy(rng.integers(0, 4, size=M).astype(np.uint8)).to(dev)
    logp = torch.full((M, 4), -1.3862944, device=dev)
    adv, ret = rnd(M), rnd(M)
    idx = torch.randperm(M, generator=g, device=dev)[:m]
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    rows = torch.tensor([m], dtype=torch.int64, device=dev)
    batch = L.make_ppo_batch(idx, actions, legal, logp, adv, ret, rows=rows)
    frag = torch.empty(L.head_split_bytes(h), dtype=torch.uint8, device=dev)
    L.head_split(wa, wv, frag)
    beta = torch.tensor(0.02, device=dev)
    G = [torch.empty(m, h, dtype=bf, device=dev) for _ in range(3)]
    H = [torch.empty(m, h, dtype=bf, device=dev) for _ in range(3)]
    mu = [torch.empty(m, device=dev) for _ in range(3)]
    rs = [torch.empty(m, device=dev) for _ in range(3)]
    masked = torch.empty(m, 4, device=dev)
    dz = torch.empty(m, 8, device=dev)
    out = dict(x0=torch.empty(m, 48, dtype=bf, device=dev), g=G, h=H, mean=mu, rstd=rs, masked=masked, dz=dz,
               dz_bf16=torch.empty(m, 16, dtype=bf, device=dev),
               partials=torch.empty(L.mlp_pass_partials(m, True), device=dev))
    drops = [L.make_dropout(0.1, l, 0, 321, 0, ctr) for l in (1, 2)]
    keep = torch.empty(2, m, 4, dtype=torch.int64, device=dev)  # the blocks' keep bits, as FusedPPOUpdater
    args = L.make_mlp_pass(boards, batch, m, w[0], w[1:], gam, bet, frag, ba, bv, drops=drops, beta_dev=beta,
                           critic=0.2, clip_eps=0.2, keep=keep, **out)
    dba, dbv, sums = torch.empty(4, device=dev), torch.empty(1, device=dev), torch.empty(3, device=dev)
    j = L.ColsumJob()
    res = {}
    res["train pass (ppo_forward_loss, deferred colsum)"] = timed(lambda: L.ppo_forward_loss(args, dba, dbv, sums, defer=j))
    kdrops = [L.make_dropout(0.1, l, 1, 321, 0, ctr) for l in (1, 2)]
    kargs = L.make_mlp_pass(boards, batch, m, w[0], w[1:], gam, bet, frag, ba, drops=kdrops, masked=masked,
                            partials=torch.empty(L.mlp_pass_partials(m, False), device=dev))
    kl = torch.empty(2, device=dev)
    jk = L.ColsumJob()
    res["KL pass (ppo_forward_kl, deferred colsum)"] = timed(lambda: L.ppo_forward_kl(kargs, kl, defer=jk))
    dg = [torch.empty(m, h, dtype=bf, device=dev) for _ in range(3)]
    dgam = [torch.empty(h, device=dev) for _ in range(3)]
    dbet = [torch.empty(h, device=dev) for _ in range(3)]
    bargs = L.make_mlp_back(m, w[1:], gam, bet, wa, wv, dz, G, mu, rs, drops=drops, dg=dg,
                            partials=torch.empty(L.mlp_back_partials(m, h), device=dev), keep=keep)
    jobs = [L.ColsumJob() for _ in range(3)]
    res["backward (ppo_backward, deferred colsums)"] = timed(lambda: L.ppo_backward(bargs, dgam, dbet, defer=jobs))
    # the weight gradients: one g2048_mlp_wgrad launch vs g2048_wgrad (head, stem) + g2048_wgrad_pair
    if hasattr(L, "mlp_wgrad_partials") and L.mlp_wgrad_partials(m, h) > 0:
        dzb = out["dz_bf16"]
        pw = torch.empty(L.mlp_wgrad_partials(m, h), device=dev)
        oh, ow = torch.empty(16, h, device=dev), [torch.empty(h, 48, device=dev)] + [torch.empty(h, h, device=dev) for _ in range(2)]
        jw = [L.ColsumJob() for _ in range(4)]
        res["weight gradients (g2048_mlp_wgrad, deferred colsums)"] = timed(
            lambda: L.mlp_wgrad(m, dzb, H[2], dg, [out["x0"], H[0], H[1]], pw, oh, ow, defer=jw))
    ph, ps = torch.empty(L.wgrad_partials(m, 16, h), device=dev), torch.empty(L.wgrad_partials(m, h, 48), device=dev)
    pp = [torch.empty(L.wgrad_pair_partials(m, h, h), device=dev) for _ in range(2)]
    oh, ow = torch.empty(16, h, device=dev), [torch.empty(h, 48, device=dev)] + [torch.empty(h, h, device=dev) for _ in range(2)]
    j3 = [L.ColsumJob() for _ in range(4)]

    def split():
        L.wgrad(out["dz_bf16"], H[2], ph, oh, defer=j3[0])
        L.wgrad(dg[0], out["x0"], ps, ow[0], defer=j3[1])
        L.wgrad_pair(dg[1], H[0], dg[2], H[1], pp[0], pp[1], ow[1], ow[2], defer=j3[2:])
    res["weight gradients (2 x g2048_wgrad + g2048_wgrad_pair)"] = timed(split)
    for k, v in res.items():
        print(f"{k:55s} {v:8.1f} us   (m={m}, h={h})")


if __name__ == "__main__":
    main()
