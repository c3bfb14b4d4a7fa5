"""Time the fused MLP backward (g2048_ppo_backward) at the bench's minibatch (65 536 rows, h 196,
dropout 0.1) with HIP events.   python tools/time_back.py [m] [h]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from g2048 import _lib as L
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 196
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    w = [(torch.randn(h, h, generator=g, device=dev) / h ** 0.5).to(bf) for _ in range(2)]
    gam = [torch.rand(h, generator=g, device=dev) + 0.5 for _ in range(3)]
    bet = [torch.randn(h, generator=g, device=dev) * 0.1 for _ in range(3)]
    wa, wv = torch.randn(4, h, generator=g, device=dev) * 0.1, torch.randn(1, h, generator=g, device=dev) * 0.1
    G = [torch.randn(m, h, generator=g, device=dev).to(bf) for _ in range(3)]
    mu = [torch.zeros(m, device=dev) for _ in range(3)]
    rs = [torch.ones(m, device=dev) for _ in range(3)]
    dz = torch.randn(m, 8, generator=g, device=dev) / m
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    drops = [L.make_dropout(0.1, l, 0, 1, 0, ctr) for l in (1, 2)]
    dg = [torch.empty(m, h, dtype=bf, device=dev) for _ in range(3)]
    dgam = [torch.empty(h, device=dev) for _ in range(3)]
    dbet = [torch.empty(h, device=dev) for _ in range(3)]
    args = L.make_mlp_back(m, w, gam, bet, wa, wv, dz, G, mu, rs, drops=drops, dg=dg,
                           partials=torch.empty(L.mlp_back_partials(m, h), device=dev))
    jobs = [L.ColsumJob() for _ in range(3)]
    run = lambda: L.ppo_backward(args, dgam, dbet, defer=jobs)  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"g2048_ppo_backward m={m} h={h}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us")


if __name__ == "__main__":
    main()
