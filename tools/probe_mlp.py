"""Runs the fused minibatch kernels repeatedly, eagerly (for rocprofv3 counter passes, one record per
dispatch): probe_mlp.py [fwd|stem|bwd|wgrad|head|all]."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "2048-ppo_amd"))
import torch  # noqa: E402
from g2048 import _lib as L  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "all"
dev = torch.device("cuda:0")
M, h = 65536, 196
bf = torch.bfloat16
X = torch.randn(M, h, device=dev, dtype=bf)
X0 = torch.randn(M, 48, device=dev, dtype=bf)
W = torch.randn(h, h, device=dev, dtype=bf) * 0.07
Ws = torch.randn(h, 48, device=dev, dtype=bf) * 0.1
gam, bet = torch.ones(h, device=dev), torch.zeros(h, device=dev)
G, Y = torch.empty(M, h, device=dev, dtype=bf), torch.empty(M, h, device=dev, dtype=bf)
mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
ctr = torch.zeros(1, dtype=torch.int64, device=dev)
drop = L.make_dropout(0.1, 1, 0, 7, 0, ctr)
dres = torch.randn(M, h, device=dev)
part = torch.empty(max(L.ln_act_bwd_partials(M, h), L.wgrad_partials(M, h, h), L.ppo_head_partials(M, h)), device=dev)
dgam, dbet = torch.empty(h, device=dev), torch.empty(h, device=dev)
dW = torch.empty(h, h, device=dev)
wa, ba, wv, bv = (torch.randn(4, h, device=dev) * 0.05, torch.zeros(4, device=dev), torch.randn(1, h, device=dev) * 0.05,
                  torch.zeros(1, device=dev))
idx = torch.randperm(M, device=dev)
batch = L.make_ppo_batch(idx, torch.zeros(M, dtype=torch.uint8, device=dev),
                         torch.full((M,), 15, dtype=torch.uint8, device=dev),
                         torch.full((M, 4), -1.3862944, device=dev), torch.randn(M, device=dev),
                         torch.randn(M, device=dev))
beta_t = torch.tensor(0.02, device=dev)
masked, dz, sums = torch.empty(M, 4, device=dev), torch.empty(M, 8, device=dev), torch.empty(3, device=dev)
dwa, dba, dwv, dbv = (torch.empty_like(t) for t in (wa, ba, wv, bv))
hg = (dz, wa, wv)
for _ in range(10):
    if which in ("fwd", "all"):
        L.mlp_fwd(X, W, gam, bet, True, G, Y, mean, rstd, drop)
    if which in ("stem", "all"):
        L.mlp_fwd(X0, Ws, gam, bet, False, G, Y, mean, rstd, None)
    if which in ("bwd", "all"):
        L.ln_act_bwd(dres, X, G, mean, rstd, gam, bet, Y, dres, part, dgam, dbet, drop)
        L.ln_act_bwd(None, None, G, mean, rstd, gam, bet, Y, dres, part, dgam, dbet, drop, head=hg)
    if which in ("wgrad", "all"):
        L.wgrad(X, Y, part, dW)
    if which in ("head", "all"):
        L.ppo_head_loss(X, wa, ba, wv, bv, batch, beta_t, 0.2, 0.2, False, masked, None, part, dwa, dba, dwv, dbv,
                        sums, dz=dz)
        L.ppo_head_kl(X, wa, ba, masked, part, sums)
torch.cuda.synchronize()
print("done")
