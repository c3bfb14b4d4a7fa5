"""Time the policy rollout of one train step (65 536 envs x T steps, GameMLP h=196): the per-step
path (obs_encode + FusedPolicy + sample + env_step per step, one hipGraph) vs the fused persistent
kernel (g2048_policy_rollout, one launch).  GPU box only.
    python tools/time_rollout.py [--n 65536] [--T 64] [--reps 10]"""
import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--h", type=int, default=196)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import os
    if os.environ.get("G2048_LIB"):  # A/B timing against another build of the library
        from g2048 import _lib as L
        L._lib = L.load(os.environ["G2048_LIB"])
    import agent
    from g2048.rollout import FusedPolicy, Rollout
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=a.h, num_layers=2)).to(dev).eval()
    pol = FusedPolicy(m)
    for fused in (False, True):
        ro = Rollout(a.n, a.T, dev, seed=1)
        ro.use_fused = fused
        ro.reset()
        ro.collect(pol, graph=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            ro.buf.carry_over()
            ro.collect(pol, graph=True)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print(f"{'fused' if fused else 'per-step'}: {ms:.3f} ms per {a.T}-step rollout of {a.n} envs "
              f"({a.n * a.T / ms * 1e3:.3e} env-steps/s, {ms / a.T * 1e3:.1f} us/step)", flush=True)


if __name__ == "__main__":
    main()
