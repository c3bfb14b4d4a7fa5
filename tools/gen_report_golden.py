"""Generate tests/golden/report.json by running the REFERENCE's report functions in this container.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_report_golden.py

One game is played by the reference's play_game_for_episode (train.py:213-346) with the shipped
best_model.pt (weights_only=True), its advantages filled by calculate_advantage (train.py:651-904);
then print_episode_breakdown / print_last_steps / print_final_state (train.py:1043-1152) are run
with a capturing logger and export_episode_visualization (train.py:1155-1209) writes its JSON.
The fixture holds the episode records (inputs) and the printed text and viz JSON (outputs): data
only, no reference source.
"""

from __future__ import annotations

import json
import random
import sys
import tempfile
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
from refshim import REF, load_reference  # noqa: E402

OUT = Path(__file__).resolve().parent.parent / "tests" / "golden" / "report.json"
KEEP = ("state_before", "result_state", "selected_direction", "points_earned", "smoothness_delta",
        "max_tile_created", "corner_delta", "adjacency_delta", "chain_delta", "topological_delta",
        "monotonicity_before", "monotonicity_after", "emptiness_before", "emptiness_after", "entropy",
        "advantage")
CASES = [  # (weights, gamma, last_steps)
    (dict(points=0.1, smoothness=0.5, max_tile=0.2, corner=0.3, adjacency=0.4, chain=0.6, monotonicity=1.0,
          emptiness=0.7, topological=0.8), 0.99, 5),
    (dict(points=1.0), 0.95, 3),
]


class CaptureLogger:
    def __init__(self):
        self.lines = []

    def print(self, msg=""):
        self.lines.append(str(msg))


def main():
    game, train = load_reference()
    ck = torch.load(REF / "docs" / "data" / "best_model.pt", map_location="cpu", weights_only=True)
    model = game.GameMLP(game.MLPConfig(**ck["config"]))
    model.load_state_dict(ck["model_state_dict"])
    model.eval()
    torch.manual_seed(4)
    ep = train.play_game_for_episode(model, max_steps=160, seed=11)
    random.seed(0)
    eps, _, _, _, _ = train.calculate_advantage([ep], 0.99, 0.0, 0.1, 1, 1, 1, 1, 1, 1.0, 0.0, 1, 1000.0)
    ep = eps[0]
    rec = {"total_points": ep["total_points"], "total_steps": ep["total_steps"], "final_state": ep["final_state"],
           "moves": [{k: m[k] for k in KEEP} for m in ep["moves"]]}
    out = {"episode": rec, "cases": []}
    for ci, (w, gamma, last) in enumerate(CASES):
        weights = train.RewardWeights(**w)
        log = CaptureLogger()
        train.print_episode_breakdown(log, rec, weights, gamma)
        train.print_last_steps(log, rec, last)
        train.print_final_state(log, rec)
        with tempfile.TemporaryDirectory() as d:
            train.export_episode_visualization(d, 17 + ci, rec, weights, gamma)
            viz = json.loads((Path(d) / f"step_{17 + ci:06d}.json").read_text())
        out["cases"].append({"weights": w, "gamma": gamma, "last_steps": last, "train_step": 17 + ci,
                             "text": log.lines, "viz": viz})
    OUT.write_text(json.dumps(out))
    print(f"report.json: {len(rec['moves'])} moves, {len(CASES)} cases")


if __name__ == "__main__":
    main()
