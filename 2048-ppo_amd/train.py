"""train.py -- CLI of the MI355X 2048 trainer, flag-compatible with the reference (train.py:1284-1456).

    python 2048-ppo_amd/train.py train --batch-size=4 --steps=20000 --lr 0.001 --critic-lr 1e-4 -h 196 \
        --gamma 0.99 --entropy 0.02 --points 0.10 --mono 1.0 --critic 0.2 --rtg-beta 0.99 --episodes 65536 --gpu

Every reference flag is accepted with the same default.  Flags that never reach the reference's
reward (--smoothness --tile-bonus --corner --adjacency --chain --topo --win-bonus) only weight the
printed breakdown table and the --viz-dir export, as in the reference; its dead flags
(--epsilon --momentum --workers) are accepted and ignored.  New flags: --horizon (0 = one full game per env per train step, the reference's
semantics; T > 0 = fixed-horizon auto-reset throughput mode), --seed, --no-graph, --fp32.
--model-type urm trains the GameURM transformer (the reference refuses it, train.py:1523-1532):
rollouts through g2048/urm.py's kernels, the update through autograd (bf16 autocast).
For several GPUs run it under `python -m torch.distributed.run --nproc-per-node N` (one rank per
GPU; --episodes is per rank).

The module also keeps the reference's Python-level API for this path: `calculate_advantage`
(train.py:651-904) and `model_optimize_step` (train.py:414-642) over list-of-dict episodes, and
`play_game_for_episode`, built on the same device kernels.
"""

from __future__ import annotations

import json
import math
import random
import sys
from pathlib import Path
from typing import Optional

import torch
import typer

sys.path.insert(0, str(Path(__file__).resolve().parent))

import agent  # noqa: E402
from agent import Direction, GameMLP, GameURM, GameURMConfig, MLPConfig  # noqa: E402,F401
from batched_rollout import play_games_batched  # noqa: E402
from g2048.logger import MetricLogger  # noqa: E402
from g2048.optim import MultiOptimizer, build_optimizer, cosine_with_warmup  # noqa: E402,F401

app = typer.Typer(help="Train and evaluate 2048 AI agents (MI355X-native)", add_completion=False)


# ------------------------------------------------------------------------------------------------
# Reference-compatible list-of-dict API
# ------------------------------------------------------------------------------------------------
def play_game_for_episode(model, max_steps: int | None = None, device=None, seed: int | None = None):
    """One game (train.py:213-345); seed -> CPython random.seed(seed) spawns, bit-exact on the GPU."""
    from g2048.episodes import play_games
    dev = device if device is not None and torch.device(device).type == "cuda" else torch.device("cuda", 0)
    res = play_games(model, 1, max_steps, dev, seeds=[seed] if seed is not None else None,
                     seed=random.getrandbits(63), record=True)
    return res["episodes"][0]


def _pack_episodes(episodes):
    """list[EpisodeData] -> time-major [T, N] arrays (N = episodes, padding flagged inactive)."""
    import numpy as np
    from g2048 import _lib as L
    eps = [ep for ep in episodes if ep.get("moves")]
    n = len(eps)
    T = max((len(ep["moves"]) for ep in eps), default=0)
    points = np.zeros((T, n), np.int32)
    pot = np.zeros((T, n, 4), np.int8)
    flags = np.full((T, n), L.FLAG_INACTIVE, np.uint8)
    value = np.zeros((T, n), np.float32)
    for e, ep in enumerate(eps):
        for t, m in enumerate(ep["moves"]):
            points[t, e] = int(m["points_earned"])
            pot[t, e] = (int(m["monotonicity_before"]), int(m["monotonicity_after"]), int(m["emptiness_before"]),
                         int(m["emptiness_after"]))
            flags[t, e] = 0
            value[t, e] = float(m["predicted_future_value"])
    return eps, T, n, points, pot, flags, value


def calculate_advantage(episodes, discount_rate, rtg_first_moment, points_weight=1.0, smoothness_weight=1.0,
                        max_tile_weight=1.0, corner_weight=1.0, adjacency_weight=1.0, chain_weight=1.0,
                        monotonicity_weight=1.0, emptiness_weight=1.0, topological_weight=1.0, win_bonus=1000.0,
                        rtg_beta=0.9, rtg_m2=1.0, rtg_mu=0.0, rtg_step=1, upsample_ratio=0.0, device=None):
    """train.py:651-904 on the GPU scan kernel.  Sets reward / future_reward_raw / future_reward /
    advantage (Python floats) on every move; returns (episodes, augmented_steps, first_moment, m2, mu)."""
    from g2048 import _lib as L
    from g2048.augment import augment_steps
    dev = torch.device(device) if device is not None else torch.device("cuda", 0)
    eps, T, n, points, pot, flags, value = _pack_episodes(episodes)
    if n == 0 or T == 0:  # the reference's early return (train.py:734-735)
        return episodes, [], rtg_first_moment, rtg_m2, rtg_mu
    t = lambda a, dt: torch.from_numpy(a).to(dev)  # noqa: E731
    st = torch.tensor([rtg_mu, rtg_m2, rtg_first_moment, float(rtg_step), 0, 1, 0, 0], dtype=torch.float64,
                      device=dev)
    cfg = L.RewardCfg(discount_rate, points_weight, monotonicity_weight, emptiness_weight, rtg_beta)
    g_raw, g_norm, adv = (torch.zeros(T, n, dtype=torch.float32, device=dev) for _ in range(3))
    reward = torch.zeros(T, n, dtype=torch.float64, device=dev)
    part = torch.zeros(3, dtype=torch.float64, device=dev)
    ws = torch.zeros(L.rtg_workspace_bytes(n), dtype=torch.uint8, device=dev)
    L.rtg_prepare(st, cfg)
    L.reward_rtg(t(points, None), t(pot, None), t(flags, None), t(value, None), st, g_raw, g_norm, adv, part, ws, cfg,
                 reward=reward)
    L.rtg_finalize(st, part, cfg)
    gr, gn, ad, s = g_raw.cpu().numpy(), g_norm.cpu().numpy(), adv.cpu().numpy(), st.tolist()
    rw = reward.cpu().numpy()
    for e, ep in enumerate(eps):
        for k, m in enumerate(ep["moves"]):
            m["reward"] = float(rw[k, e])  # the scan kernel's own float64 reward (train.py:702-719)
            m["future_reward_raw"] = float(gr[k, e])
            m["future_reward"] = float(gn[k, e])
            m["advantage"] = float(ad[k, e])
    augmented = augment_steps([m for ep in eps for m in ep["moves"]], upsample_ratio) if upsample_ratio > 0 else []
    return episodes, augmented, s[2], s[1], s[0]


def model_optimize_step(model, episodes, optimizer, lr_scheduler=None, kl_strength: float = 0.1,
                        critic_strength: float = 1.0, device=None, batch_size: int = 32, epochs: int = 1):
    """train.py:414-642: shuffled minibatches, PPO-clip + Huber value + entropy, clip 1.0, step,
    KL diagnostic; one scheduler step per call.  Runs wherever `model` lives (CPU or GPU)."""
    from g2048.ppo import kl_old_new, ppo_losses
    moves = [m for ep in episodes for m in ep["moves"]]
    dev = next(model.parameters()).device
    obs = torch.stack([m["game_state"] for m in moves]).to(dev, torch.float32)
    actions = torch.tensor([m["selected_direction"] for m in moves], device=dev)
    invalid = torch.tensor([m["action_mask"] for m in moves], device=dev)
    adv = torch.tensor([m["advantage"] for m in moves], dtype=torch.float32, device=dev)
    ret = torch.tensor([m["future_reward"] for m in moves], dtype=torch.float32, device=dev)
    old_lp = torch.tensor([m["policy_logprobs"] for m in moves], dtype=torch.float32, device=dev)
    tot = dict.fromkeys(("loss", "policy_loss", "entropy_loss", "value_loss", "grad_norm", "entropy", "kl_total",
                         "kl_average"), 0.0)
    kl_max, nb = 0.0, 0
    params = list(model.parameters())
    for _ in range(epochs):
        perm = torch.randperm(len(moves), device=dev)
        for s in range(0, len(moves), batch_size):
            idx = perm[s:s + batch_size]
            model.train()
            logits, value = model(obs[idx])
            loss, parts = ppo_losses(logits, value, actions[idx], invalid[idx], old_lp[idx], adv[idx], ret[idx],
                                     kl_strength, critic_strength)
            loss.backward()
            gn = torch.nn.utils.clip_grad_norm_(params, 1.0)
            optimizer.step()
            optimizer.zero_grad()
            with torch.no_grad():
                new_logits, _ = model(obs[idx])
                kl = kl_old_new(parts["masked"].detach(), new_logits, invalid[idx])
            tot["loss"] += loss.item()
            tot["policy_loss"] += -parts["ppo"].mean().item()
            tot["entropy_loss"] += -kl_strength * parts["entropy"].mean().item()
            tot["value_loss"] += critic_strength * parts["vloss"].mean().item()
            tot["grad_norm"] += gn.item()
            tot["entropy"] += parts["entropy"].mean().item()
            tot["kl_total"] += kl.sum().item()
            tot["kl_average"] += kl.mean().item()
            kl_max = max(kl_max, kl.max().item())
            nb += 1
    if hasattr(optimizer, "scheduler_step"):
        optimizer.scheduler_step()
    stats = {k: v / max(nb, 1) for k, v in tot.items()}
    stats["kl_max"] = kl_max
    stats["lr"] = lr_scheduler.get_last_lr()[0] if lr_scheduler is not None else 0.0
    return stats


def export_best_game_for_demo(episode, output_path: str) -> None:
    """train.py:81-120 (the docs/data/best_game.json schema)."""
    out = Path(output_path)
    out.parent.mkdir(parents=True, exist_ok=True)
    if not episode or not episode.get("moves"):
        print("Warning: No valid episode to export")
        return
    vals = lambda g: [[2 ** c if c > 0 else 0 for c in row] for row in g]  # noqa: E731
    names = ["UP", "DOWN", "LEFT", "RIGHT"]
    data = {"score": episode["total_points"], "total_steps": episode["total_steps"], "moves": [
        {"step": i + 1, "state_before": vals(m["state_before"]) if m.get("state_before") else [],
         "action": names[m["selected_direction"]],
         "state_after": vals(m["result_state"]) if m.get("result_state") else [],
         "points_earned": m.get("points_earned", 0), "entropy": m.get("entropy", 0.0)}
        for i, m in enumerate(episode["moves"])]}
    out.write_text(json.dumps(data, indent=2))
    print(f"Exported best game ({episode['total_points']} points, {episode['total_steps']} moves) to {out}")


# ------------------------------------------------------------------------------------------------
# CLI
# ------------------------------------------------------------------------------------------------
@app.command()
def train(
    steps: int = typer.Option(1000, "--steps", "-s"),
    model_path: Optional[Path] = typer.Option(None, "--model", "-m"),
    learning_rate: float = typer.Option(0.001, "--lr"),
    gamma: float = typer.Option(0.99, "--gamma"),
    entropy_strength: float = typer.Option(0.1, "--entropy"),
    critic_strength: float = typer.Option(1.0, "--critic"),
    epsilon: float = typer.Option(1.0, "--epsilon"),
    momentum: float = typer.Option(0.99, "--momentum"),
    num_episodes: int = typer.Option(1, "--episodes"),
    batch_size: int = typer.Option(1, "--batch-size"),
    ppo_epochs: int = typer.Option(1, "--epochs"),
    workers: int = typer.Option(1, "--workers", "-w"),
    max_steps: int = typer.Option(None, "--max-steps"),
    hidden_size: int = typer.Option(64, "-h", "--hidden"),
    num_layers: int = typer.Option(2, "--num-layers", "-l"),
    model_type: str = typer.Option("mlp", "--model-type", "-t"),
    num_heads: int = typer.Option(4, "--num-heads"),
    num_loops: int = typer.Option(4, "--num-loops"),
    num_truncated_loops: int = typer.Option(1, "--truncated-loops"),
    print_frequency: int = typer.Option(10, "--print-freq", "-p"),
    show_last_steps: int = typer.Option(0, "--show-last-steps"),
    points_weight: float = typer.Option(0.0, "--points"),
    smoothness_weight: float = typer.Option(0.0, "--smoothness"),
    max_tile_weight: float = typer.Option(0.0, "--tile-bonus"),
    corner_weight: float = typer.Option(0.0, "--corner"),
    adjacency_weight: float = typer.Option(0.0, "--adjacency"),
    chain_weight: float = typer.Option(0.0, "--chain"),
    monotonicity_weight: float = typer.Option(0.0, "--mono"),
    warmup_steps: int = typer.Option(200, "--warmup-steps"),
    emptiness_weight: float = typer.Option(0.0, "--emptiness"),
    topological_weight: float = typer.Option(0.0, "--topo"),
    win_bonus: float = typer.Option(0.0, "--win-bonus"),
    gpu: bool = typer.Option(False, "--gpu"),
    viz_dir: Optional[str] = typer.Option(None, "--viz-dir"),
    rtg_beta: float = typer.Option(0.9, "--rtg-beta"),
    log_dir: Optional[str] = typer.Option(None, "--log-dir"),
    use_wandb: bool = typer.Option(False, "--wandb"),
    wandb_project: Optional[str] = typer.Option("2048-rl", "--wandb-project"),
    wandb_run_name: Optional[str] = typer.Option(None, "--wandb-run"),
    eval_freq: Optional[int] = typer.Option(None, "--eval-freq"),
    eval_games: int = typer.Option(100, "--eval-games"),
    critic_lr: float = typer.Option(0.001, "--critic-lr"),
    decouple_critic: bool = typer.Option(False, "--decouple-critic"),
    upsample_ratio: float = typer.Option(0.0, "--upsample-ratio"),
    export_demo: bool = typer.Option(False, "--export-demo"),
    checkpoint_dir: Optional[str] = typer.Option("checkpoints", "--checkpoint-dir"),
    beta1: float = typer.Option(0.9, "--beta1"),
    beta2: float = typer.Option(0.999, "--beta2"),
    weight_decay: float = typer.Option(0.01, "--weight-decay"),
    adaptive_beta: bool = typer.Option(False, "--adaptive-beta"),
    target_entropy: float = typer.Option(0.7, "--target-entropy"),
    beta_min: float = typer.Option(0.001, "--beta-min"),
    beta_max: float = typer.Option(1.0, "--beta-max"),
    beta_lr: float = typer.Option(0.01, "--beta-lr"),
    horizon: int = typer.Option(0, "--horizon", help="0: one full game per env per step; T>0: fixed horizon"),
    seed: int = typer.Option(0x2048, "--seed"),
    no_graph: bool = typer.Option(False, "--no-graph", help="disable hipGraph capture of the rollout"),
    fp32: bool = typer.Option(False, "--fp32", help="fp32 rollouts/updates instead of bf16"),
):
    """Train the policy with vectorised GPU rollouts (one rank per GPU under torch.distributed.run)."""
    from g2048.dist import init_from_env
    from g2048.trainer import TrainConfig, VecTrainer
    rank, ws, local = init_from_env()
    if not torch.cuda.is_available():
        typer.echo("Error: no ROCm GPU visible; the vectorised trainer has no CPU path")
        raise typer.Exit(1)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    logger = MetricLogger(log_dir=log_dir if rank == 0 else None, experiment_name=f"train_{model_type}",
                          use_wandb=use_wandb and rank == 0, wandb_project=wandb_project,
                          wandb_run_name=wandb_run_name, quiet=rank != 0)
    logger.print(f"Using device: {device} (rank {rank}/{ws})")
    if model_path:
        logger.print(f"Loading model from: {model_path}")
        logger.print("this path is not available")  # train.py:1508-1514
        logger.close()
        raise typer.Exit(0)
    if model_type.lower() not in ("mlp", "urm"):
        logger.print(f"Unknown model type: {model_type}. Use 'mlp' or 'urm'.")
        logger.close()
        raise typer.Exit(1)
    cfg = TrainConfig(steps=steps, lr=learning_rate, critic_lr=critic_lr, gamma=gamma, entropy=entropy_strength,
                      critic=critic_strength, episodes=num_episodes, batch_size=batch_size, epochs=ppo_epochs,
                      max_steps=max_steps, hidden=hidden_size, num_layers=num_layers, decouple_critic=decouple_critic,
                      points=points_weight, mono=monotonicity_weight, emptiness=emptiness_weight, rtg_beta=rtg_beta,
                      warmup_steps=warmup_steps, beta1=beta1, beta2=beta2, weight_decay=weight_decay,
                      adaptive_beta=adaptive_beta, target_entropy=target_entropy, beta_min=beta_min,
                      beta_max=beta_max, beta_lr=beta_lr, upsample_ratio=upsample_ratio, horizon=horizon, seed=seed,
                      graph=not no_graph, amp=not fp32, model_type=model_type.lower(), num_heads=num_heads,
                      num_loops=num_loops, num_truncated_loops=num_truncated_loops)
    name = "GameURM" if model_type.lower() == "urm" else "GameMLP"
    extra = f", heads={num_heads}, loops={num_loops}/{num_truncated_loops}" if name == "GameURM" else ""
    logger.print(f"Creating {name} model (hidden={hidden_size}, layers={num_layers}{extra}); "
                 f"{num_episodes} envs/GPU x {ws}")
    tr = VecTrainer(cfg, device)
    logger.print("Kernel paths: " + ", ".join(f"{k}={v}" for k, v in tr.paths.items()))
    for msg in tr.fallbacks:
        logger.print(f"Fallback: {msg}")
    best_eval = 0.0
    highest = 0
    from tqdm import tqdm
    from g2048 import report
    weights = report.RewardWeights(points=points_weight, smoothness=smoothness_weight, max_tile=max_tile_weight,
                                   corner=corner_weight, adjacency=adjacency_weight, chain=chain_weight,
                                   monotonicity=monotonicity_weight, emptiness=emptiness_weight,
                                   topological=topological_weight)
    it = tqdm(range(steps), desc="Running RL training", disable=rank != 0)
    for step in it:
        m = tr.train_step(step)
        should_print = step % print_frequency == 0
        logger.log(m, step=step, verbose=should_print)
        new_high = m["peak_score"] > highest  # train.py:1754-1755
        highest = max(highest, m["peak_score"])
        if rank == 0 and (should_print or (new_high and viz_dir)):
            best = tr.best_episode()  # train.py:1800-1837: tables, last steps, final state, viz export
            if should_print:
                report.print_episode_breakdown(logger, best, weights, gamma)
                if show_last_steps > 0:
                    report.print_last_steps(logger, best, show_last_steps)
                report.print_final_state(logger, best)
            if viz_dir:
                report.export_episode_visualization(viz_dir, step, best, weights, gamma)
        if step > 0 and eval_freq and step % eval_freq == 0:
            ev = tr.evaluate(eval_games, max_steps)
            logger.log(ev, step=step)
            if rank == 0 and ev["eval/avg_score"] > best_eval:
                best_eval = ev["eval/avg_score"]
                path = Path(checkpoint_dir) / "best_model.pt"
                tr.save_checkpoint(path, best_eval, step)
                logger.print(f"New best model saved (avg score: {best_eval:.1f}) to {path}")
    if export_demo and rank == 0:
        from g2048.episodes import play_games
        res = play_games(tr.model.eval(), 32, max_steps, device, record=True)
        best = max(res["episodes"], key=lambda e: e["total_points"])
        export_best_game_for_demo(best, "docs/data/best_game.json")
        logger.print("ONNX export needs the `onnx` package, which is not installed")
    logger.close()
    # the captured graphs (with their RCCL all-reduce nodes at world > 1) go before the communicator
    tr.close()
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def load_checkpoint_model(ck) -> torch.nn.Module:
    """The policy of a best_model.pt (train.py:1893-1901 layout; a bare state_dict loads as GameMLP):
    GameURM when the saved config carries URM fields (num_loops / num_heads), else GameMLP."""
    cfg = ck["config"] if isinstance(ck, dict) and "config" in ck else {}
    sd = ck["model_state_dict"] if isinstance(ck, dict) and "model_state_dict" in ck else ck
    if "num_loops" in cfg or "num_heads" in cfg:
        model = GameURM(GameURMConfig(**cfg))
    else:
        model = GameMLP(MLPConfig(**cfg))
    model.load_state_dict(sd)
    return model


@app.command()
def evaluate(model_path: Path = typer.Argument(...), games: int = typer.Option(100, "--games", "-g")):
    """Evaluate a checkpoint on `games` seeded games (game i spawns like random.seed(i))."""
    from g2048.episodes import play_games
    model = load_checkpoint_model(torch.load(model_path, map_location="cpu", weights_only=True))
    dev = torch.device("cuda", 0)
    res = play_games(model.to(dev).eval(), games, None, dev, seeds=list(range(games)), record=False)
    s, tiles = res["scores"], res["max_tiles"]
    typer.echo(f"Eval Results - Max: {max(s):.0f}, Avg: {sum(s) / len(s):.1f}, Median: {sorted(s)[len(s) // 2]:.0f}")
    typer.echo("Tiles Reached - " + ", ".join(f"{v}: {sum(1 for t in tiles if t >= v) / len(tiles) * 100:.1f}%"
                                               for v in (512, 1024, 2048)))


@app.command("export-demo")
def export_demo_cmd(model_path: Path = typer.Option("checkpoints/best_model.pt", "--model", "-m"),
                    game_path: Optional[Path] = typer.Option(None, "--game", "-g"),
                    output_dir: Path = typer.Option("docs/data", "--output", "-o"),
                    num_games: int = typer.Option(10, "--num-games", "-n"),
                    gpu: bool = typer.Option(False, "--gpu"),
                    batch_size: int = typer.Option(32, "--batch-size", "-b")):
    """train.py:1946-2072: play games in batches with play_games_batched, export the best as JSON."""
    output_dir.mkdir(parents=True, exist_ok=True)
    if not model_path.exists():
        typer.echo(f"Error: Model checkpoint not found at {model_path}")
        raise typer.Exit(1)
    model = load_checkpoint_model(torch.load(model_path, map_location="cpu", weights_only=True))
    model.eval()
    dev = torch.device("cuda", 0)
    model = model.to(dev)
    if game_path and game_path.exists():
        data = json.loads(game_path.read_text())
        (output_dir / "best_game.json").write_text(json.dumps(
            {"score": data.get("score", 0), "total_steps": data.get("total_steps", len(data["moves"])),
             "moves": data["moves"]}, indent=2))
    else:
        episodes = []
        bs = min(batch_size, num_games)
        for i in range(0, num_games, bs):
            episodes.extend(play_games_batched(model, min(bs, num_games - i), None, dev))
        scores = sorted((ep["total_points"] for ep in episodes), reverse=True)
        typer.echo(f"Played {num_games} games — avg: {sum(scores) / len(scores):.0f}, best: {scores[0]}, "
                   f"worst: {scores[-1]}")
        export_best_game_for_demo(max(episodes, key=lambda e: e["total_points"]), str(output_dir / "best_game.json"))
    typer.echo("Error: Missing dependency - onnx (ONNX export is not available in this build)")
    raise typer.Exit(1)


if __name__ == "__main__":
    app()
