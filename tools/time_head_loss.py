"""Event-timed g2048_ppo_head_loss at the training shape (65 536 x 196, dz output, column sums
deferred like FusedPPOUpdater) -- PMC: TAG=hl bash tools/pmc_kernel.sh python3 tools/time_head_loss.py"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "2048-ppo_amd"))
import torch  # noqa: E402
from g2048 import _lib as L  # noqa: E402

dev = torch.device("cuda:0")
M, h, N = 65536, 196, 1 << 20
torch.manual_seed(0)
x = torch.randn(M, h, device=dev, dtype=torch.bfloat16)
wa, ba = torch.randn(4, h, device=dev) * 0.05, torch.zeros(4, device=dev)
wv, bv = torch.randn(1, h, device=dev) * 0.05, torch.zeros(1, device=dev)
idx = torch.randint(0, N, (M,), device=dev)
act = torch.randint(0, 4, (N,), device=dev, dtype=torch.uint8)
legal = torch.full((N,), 15, device=dev, dtype=torch.uint8)
logp = torch.full((N,), -1.3, device=dev)
adv, ret = torch.randn(N, device=dev), torch.randn(N, device=dev)
batch = L.make_ppo_batch(idx, act, legal, logp, adv, ret)
beta = torch.tensor([0.01], device=dev)
masked = torch.empty(M, 4, device=dev)
dz = torch.empty(M, 8, device=dev)
part = torch.empty(L.ppo_head_partials(M, h), device=dev)
gwa, gba, gwv, gbv = torch.empty_like(wa), torch.empty_like(ba), torch.empty_like(wv), torch.empty_like(bv)
sums = torch.zeros(3, device=dev)


def fn():
    job = L.ColsumJob()
    L.ppo_head_loss(x, wa, ba, wv, bv, batch, beta, 0.5, 0.2, False, masked, None, part, gwa, gba, gwv, gbv, sums,
                    dz=dz, defer=job)


for _ in range(3):
    fn()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    fn()
e1.record()
torch.cuda.synchronize()
print(f"ppo_head_loss 65536 x 196: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us")
