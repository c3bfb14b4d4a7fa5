"""One GameURM training fwd+bwd (the device autograd Functions, bf16 autocast, dropout 0.1) and one
one-launch rollout forward at BASELINE config 5's per-GPU shape (65 536 boards), for rocprofv3 PMC
passes (tools/pmc_urm.sh): few dispatches, so counter collection stays short.

    python tools/urm_pmc_step.py
"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]

import torch  # noqa: E402

import agent  # noqa: E402
from g2048.urm import URMPolicy  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = agent.GameURM(agent.GameURMConfig(dropout=0.1)).to(dev)
obs = torch.rand(65536, 48, device=dev) * 8
for _ in range(2):
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg, v = m(obs)
    (lg.float().sum() + v.float().sum()).backward()
m.eval()
pol = URMPolicy(m)
for _ in range(2):
    pol(obs)
torch.cuda.synchronize()
print("urm pmc step done")
