"""torch.profiler census of the train step's rollout metrics (VecTrainer._metrics) at the bench's
GameMLP configuration: which aten ops make up the ~1.2 ms metrics phase.
    python tools/prof_metrics.py [envs] [horizon]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from torch.profiler import ProfilerActivity, profile
    from g2048.trainer import TrainConfig, VecTrainer
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(steps=1000, lr=1e-3, critic_lr=1e-4, gamma=0.99, entropy=0.02, critic=0.2,
                      episodes=envs, batch_size=65536, epochs=1, hidden=196, num_layers=2,
                      points=0.1, mono=1.0, rtg_beta=0.99, warmup_steps=10, horizon=T,
                      upsample_ratio=0.25, seed=0x2048, graph=True, amp=True)
    tr = VecTrainer(cfg, dev)
    for s in range(3):
        tr.train_step(s)
    torch.cuda.synchronize()
    orig = tr._metrics
    caught = {}

    def wrapped(*a, **k):
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            r = orig(*a, **k)
            torch.cuda.synchronize()
        caught["p"] = prof
        return r
    tr._metrics = wrapped
    tr.train_step(3)
    ka = caught["p"].key_averages()
    print(ka.table(sort_by="device_time_total", row_limit=40, max_name_column_width=70))


if __name__ == "__main__":
    main()
