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

MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 (MI355X_MICROARCH.md), not the 2:1-sparsity figure
HBM_PEAK_GBPS = 8000.0
# the update kernels' HBM bytes per 65 536-row minibatch from the committed PMC passes of this build
# (FETCH_SIZE / WRITE_SIZE, tools/pmc_train.sh -> tools/summarize_profile.py)
UPDATE_HBM = "profiles/r05m/train/update_hbm.json"
# the GameURM update's HBM bytes (every dispatch of one update, tools/urm_update_pmc.py under FETCH /
# WRITE passes -> tools/urm_update_hbm.py)
URM_UPDATE_HBM = "profiles/r06b/urm_update_hbm.json"


def mlp_flops_per_sample(h: int = 196, obs: int = 48, layers: int = 2, heads: int = 5) -> dict:
    """Algorithmic FLOP per sample of GameMLP (game.py:1049-1220): the forward's GEMMs, and the PPO
    update's train forward + backward (input and weight gradients: 2 x forward, the stem's input
    gradient excluded) + KL re-forward."""
    fwd = 2 * (obs * h + layers * h * h + h * heads)
    bwd = 2 * (obs * h + layers * h * h + h * heads) + 2 * (layers * h * h + h * heads)
    return {"forward": fwd, "update": fwd + bwd + fwd}


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
    # roofline of the two MFMA phases of the profiled iteration (one GPU's share): algorithmic FLOP
    # over the phase's wall time against the dense bf16 peak
    mc = tr.model.config
    fl = mlp_flops_per_sample(h=mc.hidden_dim, layers=len(tr.model.backbone))
    # the update's work is the real sample rows: the ragged last minibatch's padding is not counted
    rows_update = args.envs * args.train_horizon + int(m["augmented_samples"])
    paths, fallbacks, phases = tr.paths, tr.fallbacks, dict(tr.timings)
    tr.close()  # its graphs hold captured RCCL all-reduces at world > 1: released before the process group
    roof = {}
    for name, ms_key, flop in (("update", "update_ms", fl["update"] * rows_update),
                               ("policy_rollout", "rollout_ms", fl["forward"] * args.envs * args.train_horizon)):
        ms = phases.get(ms_key)
        if ms:
            ach = flop / (ms * 1e-3) / 1e12
            roof[name] = {"bound": "mfma", "achieved": ach, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": ach / MFMA_BF16_PEAK_TFLOPS, "flop_per_sample": fl["update" if name == "update" else "forward"],
                          "samples": rows_update if name == "update" else args.envs * args.train_horizon}
    # the same phase against HBM: the PMC-measured bytes of the update kernels per minibatch x the
    # minibatches of the iteration over the update's wall time
    try:
        import json
        from pathlib import Path
        hb = json.loads((Path(__file__).resolve().parents[2] / UPDATE_HBM).read_text())
        ms = phases.get("update_ms")
        if ms and hb.get("minibatch_rows") == args.train_batch:
            traffic = hb["bytes_per_minibatch"] * n_mb
            ach = traffic / (ms * 1e-3) / 1e9
            roof["update_hbm"] = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                  "frac": ach / HBM_PEAK_GBPS, "traffic_per_minibatch": hb["bytes_per_minibatch"],
                                  "minibatches": n_mb, "per_kernel_bytes": {k: v["hbm_bytes_per_launch"] * v["launches_per_minibatch"]
                                                                           for k, v in hb["kernels"].items()},
                                  "traffic_source": UPDATE_HBM}
    except (OSError, ValueError, KeyError):
        pass
    return {
        "value": steps / wall, "unit": "env-steps/s", "ms_per_iter": wall / args.train_iters * 1e3,
        "iters": args.train_iters, "warmup": args.train_warmup,
        "config": {"workload": "65536 envs/GPU MLP h=196 bf16: rollout + RTG/entropy + PPO update",
                   "envs_per_gpu": args.envs, "horizon": args.train_horizon, "minibatch": args.train_batch,
                   "minibatches_per_iter": n_mb, "upsample_ratio": args.train_upsample, "optimizer": "Muon(2-D)+AdamW(1-D)", "dtype": "bf16 activations / fp32 master weights (MFMA kernels)"},
        "phase_ms_one_iter": {k: round(v, 3) for k, v in phases.items()},
        "roofline": roof,
        "kernel_paths": paths, "fallbacks": fallbacks,
        "last_metrics": {k: m[k] for k in ("loss", "entropy", "avg_score", "episodes_finished", "grad_norm",
                                           "augmented_samples")},
    }


def bench_urm(args, rank: int, world: int, dev) -> dict:
    """BASELINE.json configs[4] on this GPU: the GameURM transformer policy (default GameURMConfig:
    h 64, 2 layers, 4 heads, 4 loops / 1 truncated, inter 120) driving 65 536 envs.  (1) rollout:
    `--urm-steps` policy steps (obs -> the one-launch URM forward g2048_urm_forward -> sampler -> env
    step), captured in one hipGraph, timed over replays; (2) one full training iteration at horizon
    `--urm-steps` (RTG + the bf16 update on the device autograd Functions of g2048/urm.py, one
    hipGraph per minibatch of --train-batch, fused Muon/AdamW)."""
    import agent
    import torch.distributed as dist
    from g2048.rollout import Rollout, make_policy
    from g2048.trainer import TrainConfig, VecTrainer
    torch.manual_seed(0x2048 + rank)
    m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
    pol = make_policy(m)
    T = args.urm_steps
    ro = Rollout(args.envs, T, dev, seed=0x2048 + rank, env_base=rank * args.envs)
    ro.reset()
    ro.collect(pol, graph=True)  # capture + first replay
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        ro.buf.carry_over()
        ro.collect(pol, graph=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # forward alone (one call of the policy on the obs buffer), events on the current stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pol(ro.buf.obs)
    e0.record()
    for _ in range(5):
        pol(ro.buf.obs)
    e1.record()
    torch.cuda.synchronize()
    fwd_ms = e0.elapsed_time(e1) / 5
    c = m.config
    flops_tok = 2 * c.num_loops * c.num_layers * (4 * c.hidden_dim ** 2 + 3 * m.layers[0].mlp.inter * c.hidden_dim
                                                  + 2 * 16 * c.hidden_dim)
    fwd_tflops = flops_tok * 16 * args.envs / (fwd_ms * 1e-3) / 1e12
    out = {"value": args.envs * T * reps * world / wall, "unit": "env-steps/s", "ms_per_step": wall / (reps * T) * 1e3,
           "forward_ms": fwd_ms, "forward_TFLOPs": fwd_tflops,
           "roofline": {"bound": "mfma", "kernel": "URM policy forward (one call, 16 tokens per board)",
                        "achieved": fwd_tflops, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": fwd_tflops / MFMA_BF16_PEAK_TFLOPS, "flop_per_token": flops_tok},
           "config": {"workload": f"{args.envs} envs/GPU, GameURM h={c.hidden_dim} L={c.num_layers} heads={c.num_heads} "
                                  f"loops={c.num_loops}/{c.num_truncated_loops} inter={m.layers[0].mlp.inter}, bf16",
                      "steps_per_graph": T, "replays": reps}}
    del ro, pol
    torch.cuda.empty_cache()
    cfg = TrainConfig(steps=1000, lr=1e-3, critic_lr=1e-4, gamma=0.99, entropy=0.02, critic=0.2, episodes=args.envs,
                      batch_size=args.train_batch, hidden=64, model_type="urm", points=0.1, mono=1.0, rtg_beta=0.99,
                      warmup_steps=10, horizon=T, seed=0x2048, graph=True, amp=True)
    tr = VecTrainer(cfg, dev)
    tr.train_step(0)  # warm-up: graph capture
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    iters = max(1, int(getattr(args, "urm_iters", 3)))
    t0 = time.perf_counter()  # profiling off: no per-phase syncs inside the timed iterations
    for s in range(iters):
        mt = tr.train_step(1 + s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    it = (time.perf_counter() - t0) / iters
    # one more profiled iteration for the phase breakdown (outside the timed region)
    tr.profile = True
    tr.timings = {}
    tr.train_step(1 + iters)
    paths, fallbacks, phases = tr.paths, tr.fallbacks, dict(tr.timings)
    tr.close()
    out["train_iter"] = {"value": args.envs * T * world / it, "unit": "env-steps/s", "ms_per_iter": it * 1e3,
                         "iters": iters,
                         "kernel_paths": paths, "fallbacks": fallbacks,
                         "phase_ms": {k: round(v, 3) for k, v in phases.items()},
                         "minibatch": args.train_batch, "loss": mt["loss"], "entropy": mt["entropy"],
                         "roofline": urm_update_roofline(c, args.envs * T, args.train_batch, phases.get("update_ms"),
                                                         flops_tok)}
    return out


def urm_update_roofline(c, rows: int, minibatch: int, update_ms, flops_tok: float) -> dict:
    """The GameURM update phase (one GPU's share of one train iteration) against both peaks.
    FLOP basis per token: the forward of every loop (flops_tok: projections 2 (4 h^2 + 3 inter h) and
    the 16-key attention products 2 x 2 x 16 h per layer application), the backward of the gradient
    loops (2 x forward x (loops - truncated) / loops: input and weight gradients) and the KL
    re-forward (one forward): flops_tok x (2 + 2 (L - Lt) / L); 16 tokens per sample, every sample of
    the iteration (no up-sampling in this leg).  HBM: the PMC bytes of one update (URM_UPDATE_HBM)
    over the update phase's wall time."""
    if not update_ms:
        return {}
    L_, Lt = c.num_loops, c.num_truncated_loops
    ftok = flops_tok * (2 + 2 * (L_ - Lt) / L_)
    ach = ftok * 16 * rows / (update_ms * 1e-3) / 1e12
    roof = {"update": {"bound": "mfma", "achieved": ach, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                       "frac": ach / MFMA_BF16_PEAK_TFLOPS, "flop_per_token": ftok, "tokens": 16 * rows,
                       "update_ms": update_ms}}
    try:
        import json
        from pathlib import Path
        hb = json.loads((Path(__file__).resolve().parents[2] / URM_UPDATE_HBM).read_text())
        if hb.get("minibatch") == minibatch and hb.get("rows") == rows:
            a = hb["bytes_per_update"] / (update_ms * 1e-3) / 1e9
            roof["update_hbm"] = {"bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                  "frac": a / HBM_PEAK_GBPS, "traffic_per_update": hb["bytes_per_update"],
                                  "top_kernels": {k: v["hbm_bytes"] for k, v in list(hb["kernels"].items())[:6]},
                                  "traffic_source": URM_UPDATE_HBM}
    except (OSError, ValueError, KeyError):
        pass
    return roof
