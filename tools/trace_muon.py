"""Phase clocks of one Muon step from a MUON_TRACE build of the library (tools/alt/libg2048_mtrace.so:
`make -C 2048-ppo_amd/csrc` flags + -DMUON_TRACE): per block, the shader-clock deltas between the
trace points of muon_kernel (start, clip coefficient, prologue, normalise, per Newton-Schulz
iteration: G, U rows, X rows, drain, barrier wait, image copy; epilogue).  GPU only.

    python tools/trace_muon.py LIB [parts]
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from g2048 import _lib as L
    L._lib = L.load(sys.argv[1])
    os.environ["G2048_MUON_PARTS"] = sys.argv[2] if len(sys.argv) > 2 else "8"
    import agent
    from g2048.dist import GradBucket
    from g2048.optim import FusedMuonAdamW
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=196, num_layers=2)).to(dev)
    fo = FusedMuonAdamW(m, 1e-3, 1e-4)
    order = [p for p, _ in fo.muon] + [p for grp in fo.adam_groups for p in grp["params"]]
    bk = GradBucket(order)
    bk.flat.copy_(torch.randn_like(bk.flat) * 1e-2)
    for _ in range(4):
        fo.step_clipped(bk.flat, 1.0)
    torch.cuda.synchronize()
    ws = getattr(fo, "_ws", None)
    if ws is None:
        print("no workspace (parts <= 1): nothing traced")
        return
    nblk = 128  # kMuonMaxJobs
    nbytes = nblk * 64 * 8
    tr = ws[-nbytes:].view(torch.int64).view(nblk, 64).cpu().numpy()
    for b in range(nblk):
        k = int(tr[b, 0])
        if k == 0:
            continue
        t = tr[b, 1:k + 1].astype(np.int64)
        d = np.diff(t)
        print(f"block {b:2d}: total {t[-1] - t[0]:7d} clk  " + " ".join(str(int(x)) for x in d))


if __name__ == "__main__":
    main()
