"""GameURM parameter gradients of one fwd + bwd with LinResRMSFn's one-pass vs three-launch backward
(diagnostic; GPU only): per parameter the cosine and the max error relative to the largest entry."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    import agent
    from g2048 import urm
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    mod = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev).train()
    obs = (torch.rand(2048, 48, device=dev) * 8).bfloat16()
    wt = torch.randn(2048, 64, device=dev)
    grads = []
    for fused in (True, False):
        urm.LinResRMSFn.fused_bwd = fused
        for direct in (False, True):
            mod.zero_grad(set_to_none=False)
            for p in mod.parameters():
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            ctx = urm.direct_weight_grads() if direct else torch.autograd.graph.saved_tensors_hooks(lambda x: x, lambda x: x)
            with torch.autocast("cuda", dtype=torch.bfloat16), ctx:
                pooled = mod.features(obs)
                (pooled.float() * wt).sum().backward()
            grads.append({k: p.grad.detach().clone() for k, p in mod.named_parameters()})
    urm.LinResRMSFn.fused_bwd = True
    names = ["fused", "fused+direct", "unfused", "unfused+direct"]
    for i, j in ((0, 2), (0, 1), (2, 3)):
        print(f"== {names[i]} vs {names[j]}")
        for k in grads[i]:
            a, b = grads[i][k].reshape(-1).float(), grads[j][k].reshape(-1).float()
            if b.norm() == 0:
                continue
            c = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
            e = float((a - b).abs().max() / b.abs().max())
            print(f"  {k:40s} cos {c:.7f}  maxerr/max {e:.2e}")


if __name__ == "__main__":
    main()
