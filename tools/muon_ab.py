"""Multi-CU vs one-CU Muon equality with a given library build (bisecting builds of optim.hip):
    python tools/muon_ab.py LIB [parts] [poison]   GPU only; prints per-tensor equality and NaN counts.
poison: every CU's LDS filled with a NaN pattern before each step (g2048_lds_poison)."""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from g2048 import _lib as L
    L._lib = L.load(sys.argv[1])
    parts = sys.argv[2] if len(sys.argv) > 2 else "13"
    poison = len(sys.argv) > 3 and sys.argv[3] == "poison"
    import agent
    from g2048.dist import GradBucket
    from g2048.optim import FusedMuonAdamW
    dev = torch.device("cuda", 0)
    outs = []
    for p in ("1", parts):
        os.environ["G2048_MUON_PARTS"] = p
        torch.manual_seed(196)
        m = agent.GameMLP(agent.MLPConfig(hidden_dim=196, num_layers=2)).to(dev)
        opt = FusedMuonAdamW(m, 1e-3, 1e-4)
        order = [q for q, _ in opt.muon] + [q for grp in opt.adam_groups for q in grp["params"]]
        bk = GradBucket(order)
        for s in range(3):
            bk.flat.copy_(torch.randn(bk.flat.shape, generator=torch.Generator().manual_seed(s)).to(dev) * 1e-2)
            if poison:
                L.lds_poison(0x7FC07FC0, dev)
            opt.step_clipped(bk.flat, 1.0)
        torch.cuda.synchronize()
        outs.append([(n, q.detach().clone()) for n, q in m.named_parameters()])
    for (n, a), (_, b) in zip(*outs):
        print(f"{n:28s} equal {torch.equal(a, b)}  nan one-CU {int(a.isnan().sum())} multi {int(b.isnan().sum())}")


if __name__ == "__main__":
    main()
