"""HIP-event timings of the GameURM training update's projection-kernel calls (urm_linear_kernel
instances) at N boards, h = 64, inter = 120: the forwards (qkv store, o_proj / down_proj + residual
RMSNorm training epilogue, gate_up + SwiGLU-conv training epilogue with and without gu) and the
input gradients dX = dY W (qkv, gate_up), and the gate_up + SwiGLU-conv backward (gu recomputed).  G2048_LIB=<path> times another build (A/B).  Each line
also prints a checksum of the outputs, so two builds can be compared for identical results.

    python tools/time_urm_train_linear.py [boards]
"""
import os
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


def csum(*ts):
    return sum(float(t.float().double().abs().sum()) for t in ts)


def main():
    from g2048 import _lib as L
    if os.environ.get("G2048_LIB"):
        L._lib = L.load(os.environ["G2048_LIB"])
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    h, i = 64, 120
    r = 16 * n
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(7)
    xb = torch.randn(r, h, device=dev, generator=g).to(bf)
    act = torch.randn(r, i, device=dev, generator=g).to(bf)
    hres = torch.randn(r, h, device=dev, generator=g)
    dqkv = torch.randn(r, 3 * h, device=dev, generator=g).to(bf)
    dgu = torch.randn(r, 2 * i, device=dev, generator=g).to(bf)
    wq, wo, wg, wd = (torch.randn(a, b, device=dev, generator=g).to(bf) * 0.1
                      for a, b in ((3 * h, h), (h, h), (2 * i, h), (h, i)))
    cw, cb = torch.randn(i, 2, device=dev, generator=g), torch.randn(i, device=dev, generator=g)
    qkv = torch.empty(r, 3 * h, dtype=bf, device=dev)
    out, outb, rstd = torch.empty(r, h, device=dev), torch.empty(r, h, dtype=bf, device=dev), torch.empty(r, device=dev)
    gu, a_out = torch.empty(r, 2 * i, dtype=bf, device=dev), torch.empty(r, i, dtype=bf, device=dev)
    dx = torch.empty(r, h, dtype=bf, device=dev)
    dact = torch.randn(r, i, device=dev, generator=g).to(bf)
    dgu2, dwc, dbc = torch.empty(r, 2 * i, dtype=bf, device=dev), torch.empty(i, 2, device=dev), torch.empty(i, device=dev)
    part = torch.empty(L.urm_swiglu_conv_partials(n, i), device=dev)
    cases = {
        "qkv fwd (store)": (lambda: L.urm_linear(xb, wq, qkv), r * (h + 3 * h) * 2, (qkv,)),
        "o_proj + rms_t": (lambda: L.urm_linear_res_rms(xb, wo, hres, out, outb, rstd, 1e-5),
                           r * (h * 2 + h * 4 * 2 + h * 2 + 4), (out, outb, rstd)),
        "down + rms_t": (lambda: L.urm_linear_res_rms(act, wd, hres, out, outb, rstd, 1e-5),
                         r * (i * 2 + h * 4 * 2 + h * 2 + 4), (out, outb, rstd)),
        "gate_up swiglu_t +gu": (lambda: L.urm_linear_swiglu_train(xb, wg, cw, cb, gu, a_out),
                                 r * (h + 2 * i + i) * 2, (gu, a_out)),
        "gate_up swiglu_t": (lambda: L.urm_linear_swiglu_train(xb, wg, cw, cb, None, a_out), r * (h + i) * 2, (a_out,)),
        "qkv dX (linear_t)": (lambda: L.urm_linear_t(dqkv, wq, dx), r * (3 * h + h) * 2, (dx,)),
        "gate_up dX (linear_t)": (lambda: L.urm_linear_t(dgu, wg, dx), r * (2 * i + h) * 2, (dx,)),
        "gate_up swiglu bwd": (lambda: L.urm_gate_up_swiglu_bwd(xb, wg, cw, cb, dact, dgu2, dwc, dbc, part),
                               r * (h + i + 2 * i) * 2, (dgu2, dwc, dbc)),
    }
    for name, (fn, nbytes, outs) in cases.items():
        us = timed(fn)
        print(f"{name:24s} {us:8.1f} us  {nbytes / us / 1e3:7.0f} GB/s  checksum {csum(*outs):.6e}", flush=True)


if __name__ == "__main__":
    main()
