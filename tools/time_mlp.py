"""Event-timed variants of g2048_mlp_fwd at the training shape (65 536 x 196): stem, block with
G + dropout (training pass), block without G (KL re-forward), block inference (rollout policy)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "2048-ppo_amd"))
import torch  # noqa: E402
from g2048 import _lib as L  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] != "-":  # an alternative build of the library (A/B timing)
    L._lib = L.load(sys.argv[1])  # load(path) alone does not replace the module's library

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
cases = {
    "stem (G, stats)": (lambda: L.mlp_fwd(X0, Ws, gam, bet, False, G, Y, mean, rstd, None), 6.3 + 2 * 25.7),
    "block train (G, stats, dropout, residual)": (lambda: L.mlp_fwd(X, W, gam, bet, True, G, Y, mean, rstd, drop),
                                                  3 * 25.7),
    "block KL (dropout, residual)": (lambda: L.mlp_fwd(X, W, gam, bet, True, None, Y, None, None, drop), 2 * 25.7),
    "block inference (residual)": (lambda: L.mlp_fwd(X, W, gam, bet, True, None, Y, None, None, None), 2 * 25.7),
}
print("library:", L.load()._name)
only = sys.argv[2] if len(sys.argv) > 2 else None  # substring: time one case only (PMC passes)
for name, (fn, mb) in cases.items():
    if only and only not in name:
        continue
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"{name:45s} {us:7.1f} us  {mb / us:6.2f} TB/s ({mb:.0f} MB)")
