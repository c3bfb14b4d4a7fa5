"""Episode reports of the trainer CLI (the reference's stdout tables and viz export,
train.py:183-210 format_grid, :1043-1124 print_episode_breakdown, :1127-1152 print_last_steps /
print_final_state, :1155-1209 export_episode_visualization): same text layout and JSON schema,
fed by EpisodeData records whose info deltas come from the g2048_info_deltas kernel."""

from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path

DIRECTION_NAMES = ("UP", "DOWN", "LEFT", "RIGHT")


@dataclass
class RewardWeights:
    """train.py:907-919"""
    points: float = 0.0
    smoothness: float = 0.0
    max_tile: float = 0.0
    corner: float = 0.0
    adjacency: float = 0.0
    chain: float = 0.0
    monotonicity: float = 0.0
    emptiness: float = 0.0
    topological: float = 0.0


def _value(e: int) -> int:
    return 1 << e if e > 0 else 0


def format_grid(grid, indent: str = "  ") -> str:
    """A boxed 4x4 grid of tile values ('.' = empty), cells centred in max(4, digits+1) columns."""
    width = max(4, len(str(max(_value(c) for row in grid for c in row))) + 1)
    rule = "─" * (width * 4 + 3)
    out = [f"{indent}┌{rule}┐"]
    for i, row in enumerate(grid):
        out.append(indent + "│" + "│".join(("." if c == 0 else str(_value(c))).center(width) for c in row) + "│")
        out.append(f"{indent}├{rule}┤" if i < 3 else f"{indent}└{rule}┘")
    return "\n".join(out)


def print_episode_breakdown(logger, episode: dict, w: RewardWeights, gamma: float) -> None:
    moves = episode.get("moves") or []
    if not moves:
        return
    logger.print(f"\n  Best game this batch (score: {episode['total_points']}, steps: {episode['total_steps']}):")
    total = lambda key: sum(m.get(key, 0) for m in moves)  # noqa: E731
    rows = [("points_earned", total("points_earned"), w.points), ("smoothness", total("smoothness_delta"), w.smoothness),
            ("tile_bonus", total("max_tile_created"), w.max_tile), ("corner", total("corner_delta"), w.corner),
            ("adjacency", total("adjacency_delta"), w.adjacency), ("chain", total("chain_delta"), w.chain),
            ("topological", total("topological_delta"), w.topological)]
    logger.print("  Reward breakdown:")
    logger.print("    ┌─────────────────┬──────────┬────────┬──────────┐")
    logger.print("    │ Component       │      Raw │ Weight │ Weighted │")
    logger.print("    ├─────────────────┼──────────┼────────┼──────────┤")
    weighted_sum = 0.0
    for name, raw, weight in rows:
        weighted_sum += raw * weight
        logger.print(f"    │ {name:<15} │ {raw:>8.1f} │ {weight:>6.2f} │ {raw * weight:>8.1f} │")
    logger.print("    ├─────────────────┼──────────┼────────┼──────────┤")
    logger.print(f"    │ {'TOTAL':<15} │          │        │ {weighted_sum:>8.1f} │")
    logger.print("    └─────────────────┴──────────┴────────┴──────────┘")
    if w.monotonicity == 0.0 and w.emptiness == 0.0:
        return
    n = len(moves)
    gT = gamma ** n
    logger.print("")
    logger.print(f"  PBRS Reward Shaping (γ={gamma:.4f}, T={n}, γ^T={gT:.4f}):")
    logger.print("    ┌─────────────┬──────────┬──────────┬────────┬──────────┐")
    logger.print("    │ Potential   │    Φ(s₀) │   Φ(s_T) │ Weight │ γ^T·Φ_T-Φ₀│")
    logger.print("    ├─────────────┼──────────┼──────────┼────────┼──────────┤")
    pbrs = 0.0
    for label, key, weight in (("monotonicity", "monotonicity", w.monotonicity), ("emptiness   ", "emptiness", w.emptiness)):
        if weight == 0.0:
            continue
        phi0, phiT = moves[0].get(f"{key}_before", 0.0), moves[-1].get(f"{key}_after", 0.0)
        contrib = (gT * phiT - phi0) * weight
        pbrs += contrib
        logger.print(f"    │ {label}│ {phi0:>8.1f} │ {phiT:>8.1f} │ {weight:>6.2f} │ {contrib:>9.2f} │")
    logger.print("    ├─────────────┼──────────┼──────────┼────────┼──────────┤")
    logger.print(f"    │ TOTAL       │          │          │        │ {pbrs:>9.2f} │")
    logger.print("    └─────────────┴──────────┴──────────┴────────┴──────────┘")


def print_last_steps(logger, episode: dict, num_steps: int) -> None:
    moves = episode.get("moves") or []
    if not moves:
        return
    shown = moves[-num_steps:]
    first = len(moves) - len(shown)
    logger.print(f"\n  Last {len(shown)} steps (pts: {' → '.join(str(m.get('points_earned', 0)) for m in shown)}):")
    for k, m in enumerate(shown):
        logger.print(f"\n  Step {first + k + 1}: {DIRECTION_NAMES[m['selected_direction']]} (+{m.get('points_earned', 0)} pts)")
        if "result_state" in m:
            logger.print(format_grid(m["result_state"], indent="  "))


def print_final_state(logger, episode: dict) -> None:
    if "final_state" in episode:
        logger.print("\n  Final state:")
        logger.print(format_grid(episode["final_state"], indent="  "))


def export_episode_visualization(viz_dir: str, train_step: int, episode: dict, w: RewardWeights,
                                 gamma: float) -> Path | None:
    """viz_dir/step_XXXXXX.json in the reference's schema (train.py:1155-1209)."""
    moves = episode.get("moves") or []
    if not moves:
        return None
    grid = lambda g: [[_value(c) for c in row] for row in g] if g else []  # noqa: E731
    data = {"step": train_step, "score": episode["total_points"], "total_steps": episode["total_steps"], "moves": []}
    for k, m in enumerate(moves):
        g = m.get
        data["moves"].append({
            "step": k + 1, "state_before": grid(g("state_before", [])), "action": DIRECTION_NAMES[m["selected_direction"]],
            "state_after": grid(g("result_state", [])), "points_earned": g("points_earned", 0),
            "rewards": {
                "points": g("points_earned", 0) * w.points, "smoothness": g("smoothness_delta", 0) * w.smoothness,
                "tile_bonus": g("max_tile_created", 0) * w.max_tile, "corner": g("corner_delta", 0) * w.corner,
                "adjacency": g("adjacency_delta", 0) * w.adjacency, "chain": g("chain_delta", 0) * w.chain,
                "monotonicity": (gamma * g("monotonicity_after", 0) - g("monotonicity_before", 0)) * w.monotonicity,
                "topological": g("topological_delta", 0) * w.topological,
                "emptiness": (gamma * g("emptiness_after", 0) - g("emptiness_before", 0)) * w.emptiness},
            "entropy": g("entropy", 0.0), "advantage": g("advantage", 0.0)})
    path = Path(viz_dir)
    path.mkdir(parents=True, exist_ok=True)
    out = path / f"step_{train_step:06d}.json"
    out.write_text(json.dumps(data, indent=2))
    return out
