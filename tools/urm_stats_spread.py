"""Spread of the PPO minibatch statistics under rounding-order changes alone (diagnostic for the
tolerance of tests/test_gpu_urm.py::test_urm_ppo_updater_matches_generic_updater): the same update
of the same GameURM on the same minibatches with URMPPOUpdater / PPOUpdater, each with LinResRMSFn's
one-pass and three-launch backward.  GPU only.   python tools/urm_stats_spread.py"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd"), str(ROOT / "tests")]


def main():
    import agent
    from g2048 import _lib as L
    from g2048.dist import GradBucket
    from g2048.optim import MuonAdamW
    from g2048.ppo import PPOConfig, PPOUpdater
    from g2048.urm import LinResRMSFn
    from g2048.urmppo import URMPPOUpdater
    from test_gpu_urm import _urm_columns
    dev = torch.device("cuda", 0)
    cols = _urm_columns(dev, 4096, seed=7)

    def enc(b):
        o = torch.empty(b.shape[0], 48, dtype=torch.float32, device=dev)
        L.obs_encode(b.contiguous(), o)
        return o
    out, deltas = {}, {}
    for cls in (URMPPOUpdater, PPOUpdater):
        for fused in (True, False):
            LinResRMSFn.fused_bwd = fused
            torch.manual_seed(2)
            mod = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
            opt = MuonAdamW(mod, 1e-3, 1e-4)
            order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
            gen = torch.Generator(device=dev)
            gen.manual_seed(5)
            init = {k: p.detach().clone() for k, p in mod.named_parameters()}
            up = cls(mod, opt, PPOConfig(batch_size=2048, critic=0.2), GradBucket(order), gen, graph=False)
            out[(cls.__name__, fused)] = {k: float(v) for k, v in up.update(cols, 0.02, enc).items()}
            deltas[(cls.__name__, fused)] = {k: (p.detach() - init[k]).reshape(-1) for k, p in mod.named_parameters()}
    LinResRMSFn.fused_bwd = True
    cos = torch.nn.functional.cosine_similarity
    for a, b in ((("URMPPOUpdater", True), ("URMPPOUpdater", False)), (("PPOUpdater", True), ("PPOUpdater", False)),
                 (("URMPPOUpdater", True), ("PPOUpdater", True)), (("URMPPOUpdater", False), ("PPOUpdater", False))):
        worst = min((float(cos(deltas[a][k], deltas[b][k], dim=0)), k) for k in deltas[a] if deltas[b][k].norm() > 0)
        print(f"{a} vs {b}: min delta cosine {worst[0]:.6f} ({worst[1]})")
    keys = list(next(iter(out.values())).keys())
    for k in keys:
        vals = {f"{c[:3]}{'F' if f else 'U'}": round(v[k], 6) for (c, f), v in out.items()}
        ref = out[("PPOUpdater", False)][k]
        spread = max(abs(v[k] - ref) for v in out.values()) / max(abs(ref), 1e-12)
        print(f"{k:14s} {vals}  max rel spread {spread:.4f}")


if __name__ == "__main__":
    main()
