"""Time the GameURM policy forward (g2048/urm.py) at N boards; run under rocprofv3 --kernel-trace
--stats for the per-kernel split.   python tools/time_urm.py [N] [hidden] [reps]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    import os
    import agent
    from g2048 import _lib
    if os.environ.get("G2048_LIB"):  # time a variant build (tools/alt/...) instead of the in-tree library
        _lib._lib = _lib.load(os.environ["G2048_LIB"])
    from g2048.urm import URMPolicy
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    h = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = agent.GameURM(agent.GameURMConfig(hidden_dim=h, dropout=0.0)).to(dev).eval()
    pol = URMPolicy(m)
    obs = (torch.rand(n, 48, device=dev) * 8).to(torch.bfloat16)
    pol(obs)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        pol(obs)
    e1.record()
    torch.cuda.synchronize()
    print(f"URM forward n={n} h={h}: {e0.elapsed_time(e1) / reps:.3f} ms")


if __name__ == "__main__":
    main()
