"""Time g2048_linear_dgrad (P = dG W, bf16 MFMA) against torch.mm (hipBLASLt) at the minibatch shape.
    python tools/time_dgrad.py [m] [h]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    from g2048 import _lib as L
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 196
    dev = torch.device("cuda", 0)
    dg = torch.randn(m, h, device=dev).to(torch.bfloat16)
    w = torch.randn(h, h, device=dev).to(torch.bfloat16)
    out = torch.empty(m, h, dtype=torch.bfloat16, device=dev)
    t_k = timed(lambda: L.linear_dgrad(dg, w, out))
    t_b = timed(lambda: torch.mm(dg, w, out=out))
    gb = (2 * m * h * 2) / 1e9
    print(f"dgrad m={m} h={h}: kernel {t_k:.1f} us ({gb / t_k * 1e6:.0f} GB/s), torch.mm {t_b:.1f} us")


if __name__ == "__main__":
    main()
