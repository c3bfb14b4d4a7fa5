"""URM attention core fwd + bwd at 65 536 boards (h 64, 4 heads): URMAttentionFn vs torch SDPA (bf16)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "2048-ppo_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from g2048.urm import URMAttentionFn  # noqa: E402

dev = torch.device("cuda:0")
n, heads, h = 65536, 4, 64
qkv = torch.randn(16 * n, 3 * h, device=dev).bfloat16().requires_grad_(True)
g = torch.randn(16 * n, h, device=dev).bfloat16()


def dev_path():
    URMAttentionFn.apply(qkv, heads).backward(g)


def sdpa_path():
    q, k, v = qkv.view(n, 16, 3, heads, 16).permute(2, 0, 3, 1, 4).unbind(0)
    F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(16 * n, h).backward(g)


for name, fn in (("URMAttentionFn", dev_path), ("torch SDPA", sdpa_path)):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:16s} fwd+bwd {e0.elapsed_time(e1) / 5:.2f} ms")
