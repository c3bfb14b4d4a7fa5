"""Full training-iteration benchmark leg of bench.py (BASELINE.json configs[2]: 65 536 envs,
MLP h=196, return-to-go + entropy bonus, 1 MI355X; configs[3] when run on 8 ranks).

One iteration = fixed-horizon rollout of `--train-horizon` steps of every env with the bf16 policy
+ reward/RTG/advantage scan + D4 up-sampling (--upsample-ratio 0.25 of the README command, device
kernel) + PPO-clip update over all N x T samples and their copies in minibatches of `--train-batch`
(Muon + AdamW optimizer step per minibatch, the ragged last one padded; gradient all-reduce when
N > 1 GPU) + the metric reductions.  Reward weights / learning rates are the README command's.
"""

from __future__ import annotations

import time

import torch


def bench_train(args, rank: int, world: int, dev) -> dict:
    import torch.distributed as dist
    from g2048.trainer import TrainConfig, VecTrainer
    cfg = TrainConfig(steps=1000, lr=1e-3, critic_lr=1e-4, gamma=0.99, entropy=0.02, critic=0.2,
                      episodes=args.envs, batch_size=args.train_batch, epochs=1, hidden=196, num_layers=2,
                      points=0.1, mono=1.0, rtg_beta=0.99, warmup_steps=10, horizon=args.train_horizon,
                      upsample_ratio=args.train_upsample, seed=0x2048, graph=True, amp=True)
    tr = VecTrainer(cfg, dev)
    for s in range(args.train_warmup):
        tr.train_step(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.train_iters):
        m = tr.train_step(args.train_warmup + s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    # one more profiled iteration for the phase breakdown (not part of the timed region)
    tr.profile = True
    tr.timings = {}
    tr.train_step(args.train_warmup + args.train_iters)
    steps = args.envs * args.train_horizon * args.train_iters * world
    n_mb = -(-(args.envs * args.train_horizon + m["augmented_samples"]) // args.train_batch)
    return {
        "value": steps / wall, "unit": "env-steps/s", "ms_per_iter": wall / args.train_iters * 1e3,
        "iters": args.train_iters, "warmup": args.train_warmup,
        "config": {"workload": "65536 envs/GPU MLP h=196 bf16: rollout + RTG/entropy + PPO update",
                   "envs_per_gpu": args.envs, "horizon": args.train_horizon, "minibatch": args.train_batch,
                   "minibatches_per_iter": n_mb, "upsample_ratio": args.train_upsample, "optimizer": "Muon(2-D)+AdamW(1-D)", "dtype": "bf16 activations / fp32 master weights (MFMA kernels)"},
        "phase_ms_one_iter": {k: round(v, 3) for k, v in tr.timings.items()},
        "last_metrics": {k: m[k] for k in ("loss", "entropy", "avg_score", "episodes_finished", "grad_norm",
                                           "augmented_samples")},
    }
