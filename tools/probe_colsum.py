"""Lists the deferred column-sum jobs of one GameMLP minibatch (fused update, h 196, 65 536 rows):
partial rows x columns x segments per job and the blocks of the one g2048_colsum_batch_sq launch.
Runs tools/bench_update.py's fused leg once with the launch wrapped.  GPU box only.

    python tools/probe_colsum.py
"""
import json
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]

from g2048 import _lib as L  # noqa: E402

_orig = L.colsum_batch_sq
_seen = []


def _wrap(jobs, *a, **k):
    if not _seen:
        _seen.append([(int(j.nb), int(j.cols), int(j.nseg)) for j in jobs])
        print("JOBS", json.dumps(_seen[0]), "blocks", L.colsum_batch_blocks(jobs), flush=True)
    return _orig(jobs, *a, **k)


L.colsum_batch_sq = _wrap
sys.argv = [str(ROOT / "tools" / "bench_update.py"), "--which", "fused", "--samples", "262144", "--iters", "1"]
runpy.run_path(sys.argv[0], run_name="__main__")
