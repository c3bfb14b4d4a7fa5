"""Probe g2048_urm_wgrad's output mapping with structured inputs (debug tool)."""
import sys
sys.path[:0] = ['.', '2048-ppo_amd']
import torch
from g2048.urm import _wgrad
dev = torch.device('cuda', 0)
m, n, k = 64, 16, 16
# dy[m][i] = 1 iff i == m % 16 ; x[m][j] = m (row id)  -> dW[i][j] = sum_{m: m%16==i} m
dy = torch.zeros(m, n, device=dev)
for r in range(m):
    dy[r, r % 16] = 1.0
x = torch.arange(m, device=dev, dtype=torch.float32)[:, None].repeat(1, k) + torch.arange(k, device=dev)[None, :] * 0
got = _wgrad(dy.bfloat16(), x.bfloat16())
ref = dy.t() @ x
torch.set_printoptions(linewidth=200)
print("ref col0", ref[:, 0].tolist())
print("got col0", got[:, 0].tolist())
print("got row0", got[0].tolist())
# second probe: x[m][j] = j  -> dW[i][j] = count(m%16==i) * j = 4 j
x2 = torch.arange(k, device=dev, dtype=torch.float32)[None, :].repeat(m, 1)
got2 = _wgrad(dy.bfloat16(), x2.bfloat16())
print("probe2 row0", got2[0].tolist())
print("probe2 col1", got2[:, 1].tolist())
