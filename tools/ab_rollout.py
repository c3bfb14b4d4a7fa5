"""A/B of the bench's rollout leg on one box: the same RolloutBench graphs with the counter advanced
by the launch itself (g2048_env_rollout_random_adv) vs a counter-bump kernel after every launch.

    python3 tools/ab_rollout.py [rounds] [launches]
"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from bench import RolloutBench
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda", 0)
    rb = RolloutBench(65536, 256, 0, dev)
    adv_launch = rb.launch

    def bump_launch():
        rb.L.env_rollout_random(rb.env.boards, rb.chunk, rb.tb, rb.ta, rb.tp, rb.tpot, rb.tf, rb.rng)
        rb.ctr.add_(rb.chunk)
    graphs = {}
    for name, fn in (("adv", adv_launch), ("bump", bump_launch)):
        rb.launch = fn
        rb.capture(8)
        graphs[name] = (rb.graph, rb.graph_g)
    res = {"adv": [], "bump": []}
    for r in range(rounds):
        for name in ("adv", "bump") if r % 2 == 0 else ("bump", "adv"):
            rb.graph, rb.graph_g = graphs[name]
            rb.run(16)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rb.run(k)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / k * 1e3)
    for name, v in res.items():
        print(f"{name}: us per launch {sorted(v)} -> median {sorted(v)[len(v) // 2]:.2f}")


if __name__ == "__main__":
    main()
