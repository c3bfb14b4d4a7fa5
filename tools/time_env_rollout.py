"""HIP-event timing of the bench's rollout leg (65 536 boards, `chunk` env steps per launch, K launches
in one exact-count graph after a warm-up graph) for one library build.  G2048_LIB=<path> times another
build (A/B); the line ends with a checksum of the final boards and of the last launch's records, so
two builds can be compared for identical results.

    python tools/time_env_rollout.py [K] [chunk]
"""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from g2048 import _lib as L
    if os.environ.get("G2048_LIB"):
        L._lib = L.load(os.environ["G2048_LIB"])
    from bench import RolloutBench
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    dev = torch.device("cuda", 0)
    rb = RolloutBench(65536, chunk, 0, dev)
    rb.capture(1)
    rb.capture_exact(10)
    rb.capture_exact(k)
    rb.run(10)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rb.run(k)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / k * 1e3
    cs = [int(t.view(torch.uint8).to(torch.int64).sum()) for t in (rb.env.boards, rb.tb, rb.ta, rb.tp, rb.tpot, rb.tf)]
    print(f"rollout {chunk}-step launch {us:8.1f} us  {65536 * chunk / us * 1e6:.4e} env-steps/s  "
          f"checksum {' '.join(map(str, cs))}", flush=True)


if __name__ == "__main__":
    main()
