import sys
sys.path.insert(0, "2048-ppo_amd")
import torch
from g2048 import _lib as L
dev = torch.device("cuda:0")
torch.set_printoptions(linewidth=200, precision=1)
for (m, n1, n2) in [(64, 16, 16), (64, 32, 16), (128, 16, 16)]:
    # a[r][i] = 1 if r == i (+ offset) ; b[r][j] = r*100 + j  -> out[i][j] = sum_r a[r][i] b[r][j] = b[i][j]
    a = torch.zeros(m, n1, device=dev)
    for i in range(min(m, n1)):
        a[i, i] = 1
    b = torch.tensor([[r * 0 + (r % 16) * 16 + j for j in range(n2)] for r in range(m)], device=dev, dtype=torch.float32)
    a, b = a.bfloat16(), b.bfloat16()
    part = torch.empty(L.wgrad_partials(m, n1, n2), device=dev)
    out = torch.empty(n1, n2, device=dev)
    L.wgrad(a, b, part, out)
    ref = a.float().T @ b.float()
    print(m, n1, n2, "maxerr", (out - ref).abs().max().item())
    print(out[:16, :16])
    print(ref[:16, :16])
