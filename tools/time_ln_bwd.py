"""Event-timed g2048_ln_act_bwd at the training shape (65 536 x 196) in the three configurations of
the h = 196 GameMLP update (FusedPPOUpdater.loss_backward): the last block (heads' gradient,
dropout), the first block (heads + P_2, dropout), the stem (heads + P_1 + P_2, no dropout).

    python tools/time_ln_bwd.py [alternative libg2048.so]
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "2048-ppo_amd"))
import torch  # noqa: E402
from g2048 import _lib as L  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] != "-":
    L._lib = L.load(sys.argv[1])

dev = torch.device("cuda:0")
M, h = 65536, 196
bf = torch.bfloat16
G = torch.randn(M, h, device=dev, dtype=bf)
mean, rstd = G.float().mean(1), 1 / G.float().std(1)
P = [torch.randn(M, h, device=dev, dtype=bf) * 1e-2 for _ in range(2)]
dz = torch.randn(M, 8, device=dev) * 1e-3
wa, wv = torch.randn(4, h, device=dev), torch.randn(1, h, device=dev)
gam, bet = torch.rand(h, device=dev) + 0.5, torch.randn(h, device=dev) * 0.1
dg = torch.empty(M, h, device=dev, dtype=bf)
part = torch.empty(L.ln_act_bwd_partials(M, h), device=dev)
dgam, dbet = torch.empty(h, device=dev), torch.empty(h, device=dev)
ctr = torch.zeros(1, dtype=torch.int64, device=dev)
drop = L.make_dropout(0.1, 1, 0, 7, 0, ctr)
head = (dz, wa, wv)
cases = {  # name: (dy, dropout, HBM MB: G + P's read, dG written, mean/rstd/dz)
    "last block (heads, dropout)": (L.make_dy(None, [], head), drop, 2 * 25.7 + 2.6),
    "block 1 (heads + P2, dropout)": (L.make_dy(None, P[1:], head), drop, 3 * 25.7 + 2.6),
    "stem (heads + P1 + P2)": (L.make_dy(None, P, head), None, 4 * 25.7 + 2.6),
}
print("library:", L.load()._name)
for name, (dy, dr, mb) in cases.items():
    fn = lambda: L.ln_act_bwd(None, None, G, mean, rstd, gam, bet, dg, None, part, dgam, dbet, dr, dy=dy)  # noqa: E731
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"{name:35s} {us:7.1f} us  {mb / us:6.2f} TB/s ({mb:.0f} MB, incl. the column-sum launch)")
