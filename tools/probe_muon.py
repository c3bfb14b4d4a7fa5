"""Phase timing of the Newton-Schulz blocks from a -DMUON_PROBE build (tools/probe/libg2048.so):
wall-clock stamps (100 MHz) per block: start, LDS zeroed, norm, loaded, Newton-Schulz done, stored."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from g2048 import _lib as L
    L._lib = L.load(sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "tools/probe/libg2048.so"))
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
    for ns in (5, 0, 1):
        fo._cfg.ns_steps = ns
        for _ in range(5):
            fo.step_clipped(bk.flat, 1.0)
        torch.cuda.synchronize()
        off = fo._ws.numel() - 8 * 8 * 8
        st = fo._ws[off:].view(torch.int64).view(8, 8).cpu()
        for b in range(len(fo.muon)):
            t = st[b]
            d = [(int(t[k]) - int(t[0])) * 10 / 1000 for k in range(6)]
            print(f"ns={ns} block {b} {tuple(fo.muon[b][0].shape)}: " + " ".join(f"{x:.2f}" for x in d) + " us")


if __name__ == "__main__":
    main()
