"""Runs one fused layer kernel repeatedly (for rocprofv3 counter passes): probe_mlp.py [fwd|stem|bwd|head]."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "2048-ppo_amd"))
import torch  # noqa: E402
from g2048 import _lib as L  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
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
for _ in range(10):
    if which == "fwd":
        L.mlp_fwd(X, W, gam, bet, True, G, Y, mean, rstd, drop)
    elif which == "stem":
        L.mlp_fwd(X0, Ws, gam, bet, False, G, Y, mean, rstd, None)
torch.cuda.synchronize()
print("done")
