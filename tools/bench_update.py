"""Times one PPO update (all minibatches, graphed) of GameMLP h=196 with the autograd updater
(bf16 autocast) and with FusedPPOUpdater, on the same synthetic trajectory.  GPU only.

    python tools/bench_update.py [--samples 524288] [--batch 65536] [--iters 5]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "2048-ppo_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=524288)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--hidden", type=int, default=196)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--which", default="autograd,fused_torchopt,fused")
    a = ap.parse_args()
    import agent
    from g2048 import _lib as L
    import os
    if os.environ.get("G2048_LIB"):  # A/B timing against another build of the library
        L._lib = L.load(os.environ["G2048_LIB"])
    from g2048.dist import GradBucket
    from g2048.fastmlp import FusedPPOUpdater
    from g2048.optim import FusedMuonAdamW, MuonAdamW
    from g2048.ppo import PPOConfig, PPOUpdater
    dev = torch.device("cuda:0")
    g = np.random.default_rng(0)
    M = a.samples
    boards = torch.from_numpy(g.integers(0, 12, size=(M, 16)).astype(np.int8)).to(dev)
    legal = torch.empty(M, dtype=torch.uint8, device=dev)
    L.legal_mask(boards, legal)
    legal &= 0xF  # drop the done flag
    legal[legal == 0] = 1
    lg = torch.randn(M, 4, device=dev)
    inv = ((legal.to(torch.int32).unsqueeze(-1) >> torch.arange(4, device=dev)) & 1) == 0
    logp = lg.masked_fill(inv, float("-inf")).log_softmax(-1)
    acts = torch.multinomial(logp.exp(), 1).squeeze(1).to(torch.uint8)
    data = {"boards": boards, "actions": acts, "legal": legal, "logp": logp,
            "adv": torch.randn(M, device=dev), "ret": torch.randn(M, device=dev)}

    def enc(b):
        o = torch.empty(b.shape[0], 48, dtype=torch.float32, device=dev)
        L.obs_encode(b.contiguous(), o)
        return o
    out = {}
    for which in a.which.split(","):
        torch.manual_seed(0)
        m = agent.GameMLP(agent.MLPConfig(hidden_dim=a.hidden, num_layers=2, dropout=0.1)).to(dev)
        opt = (FusedMuonAdamW if which == "fused" else MuonAdamW)(m, 1e-3, 1e-4)
        order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
        gen = torch.Generator(device=dev)
        gen.manual_seed(1)
        cls = FusedPPOUpdater if which.startswith("fused") else PPOUpdater
        up = cls(m, opt, PPOConfig(batch_size=a.batch, critic=0.2), GradBucket(order), gen, graph=True)
        up.update(data, 0.02, enc)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            st = up.update(data, 0.02, enc)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        nmb = M // a.batch
        out[which] = {"ms_per_update": dt * 1e3, "ms_per_minibatch": dt * 1e3 / nmb,
                      "samples_per_s": M / dt, "loss": float(st["loss"]), "entropy": float(st["entropy"])}
        print(which, json.dumps(out[which]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
