"""Per-variant timing of the fused URM projection kernels at N boards (h = 64, inter = 120).
    python tools/time_urm_linear.py [boards]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def timed(fn, reps=20):
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    h, i = 64, 120
    r = 16 * n
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    xb = torch.randn(r, h, device=dev).to(bf)
    act = torch.randn(r, i, device=dev).to(bf)
    x = torch.randn(r, h, device=dev)
    emb = torch.randn(r, h, device=dev)
    wq, wo, wg, wd = (torch.randn(a, b, device=dev).to(bf) * 0.1 for a, b in ((3 * h, h), (h, h), (2 * i, h), (h, i)))
    cw, cb = torch.randn(i, 2, device=dev), torch.randn(i, device=dev)
    qkv = torch.empty(r, 3 * h, dtype=bf, device=dev)
    out_a = torch.empty(r, i, dtype=bf, device=dev)
    xo = torch.empty(r, h, dtype=bf, device=dev)
    cases = {
        "qkv (store)": (lambda: L.urm_linear(xb, wq, qkv), r * (h + 3 * h) * 2),
        "o_proj + rms": (lambda: L.urm_linear_rms(xb, wo, x, None, xo, 1e-5), r * (h * 2 + h * 4 * 2 + h * 2)),
        "gate_up + swiglu": (lambda: L.urm_linear_swiglu(xb, wg, cw, cb, out_a), r * (h + i) * 2),
        "down + rms + emb": (lambda: L.urm_linear_rms(act, wd, x, emb, xo, 1e-5), r * (i * 2 + h * 4 * 3 + h * 2)),
        "torch.mm qkv": (lambda: torch.mm(xb, wq.t(), out=qkv), r * (h + 3 * h) * 2),
    }
    for name, (fn, nbytes) in cases.items():
        us = timed(fn)
        print(f"{name:20s} {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s")


if __name__ == "__main__":
    main()
