"""The trainer's stdout tables and --viz-dir export (g2048/report.py) against the reference's own
output on one best_model.pt game (tests/golden/report.json, made by tools/gen_report_golden.py from
train.py:1043-1209): identical text lines and identical step_XXXXXX.json.  The info deltas in the
fixture's records are also replayed through the C oracle (game.py:981-1002)."""

import json

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def rep():
    return json.loads((GOLDEN / "report.json").read_text())


class _Log:
    def __init__(self):
        self.lines = []

    def print(self, msg=""):
        self.lines.append(str(msg))


@pytest.mark.parametrize("case", [0, 1])
def test_report_text_and_viz_match_reference(rep, case, tmp_path):
    from g2048 import report
    c = rep["cases"][case]
    ep = rep["episode"]
    w = report.RewardWeights(**c["weights"])
    log = _Log()
    report.print_episode_breakdown(log, ep, w, c["gamma"])
    report.print_last_steps(log, ep, c["last_steps"])
    report.print_final_state(log, ep)
    assert log.lines == c["text"]
    path = report.export_episode_visualization(str(tmp_path), c["train_step"], ep, w, c["gamma"])
    assert path.name == f"step_{c['train_step']:06d}.json"
    assert json.loads(path.read_text()) == c["viz"]


def test_report_empty_episode_prints_nothing(tmp_path):
    from g2048 import report
    log = _Log()
    ep = {"moves": [], "total_points": 0, "total_steps": 0}
    report.print_episode_breakdown(log, ep, report.RewardWeights(points=1.0), 0.99)
    report.print_last_steps(log, ep, 5)
    assert log.lines == []
    assert report.export_episode_visualization(str(tmp_path), 0, ep, report.RewardWeights(), 0.99) is None
    assert not any(tmp_path.iterdir())


def test_oracle_info_deltas_on_reference_episode(rep):
    """The reference game's recorded smoothness/corner/adjacency/chain/topological deltas equal the
    oracle's step(full_info) on the recorded state_before + action."""
    from oracle import oracle as O
    moves = rep["episode"]["moves"]
    boards = np.array([[c for row in m["state_before"] for c in row] for m in moves], np.int8)
    acts = np.array([m["selected_direction"] for m in moves], np.int64)
    after, f, info, _ = O.step(boards, acts, O.RNG_INJECT, inj_k=np.zeros(len(acts), np.int32),
                               inj_v=np.ones(len(acts), np.int32), full_info=True)
    want = np.array([[m[k] for k in ("smoothness_delta", "corner_delta", "adjacency_delta", "chain_delta",
                                     "topological_delta")] for m in moves])
    np.testing.assert_array_equal(info, want)
    assert np.array_equal(f["points"], [m["points_earned"] for m in moves])
