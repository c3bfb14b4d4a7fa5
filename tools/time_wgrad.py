"""Event-timed g2048_wgrad (dW = dG^T X, 65 536 x 196 x 196, incl. the column-sum launch) with the
k-split 8-wave kernel and, with G2048_WGRAD_NW4=1 in the environment, the 4-wave kernel.
    python tools/time_wgrad.py"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "2048-ppo_amd"))
import torch  # noqa: E402
from g2048 import _lib as L  # noqa: E402

dev = torch.device("cuda:0")
M, h = 65536, 196
A = torch.randn(M, h, device=dev, dtype=torch.bfloat16)
B = torch.randn(M, h, device=dev, dtype=torch.bfloat16)
part = torch.empty(L.wgrad_partials(M, h, h), device=dev)
out = torch.empty(h, h, device=dev)
for _ in range(3):
    L.wgrad(A, B, part, out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    L.wgrad(A, B, part, out)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
ref = A.float().T @ B.float()
print(f"wgrad 65536x196x196: {us:.1f} us, max |err| {float((out - ref).abs().max()):.3e} (|ref| max {float(ref.abs().max()):.1f})")
