"""Which GameURM parameters receive a gradient on the device under bf16 autocast (debug tool)."""
import sys
sys.path[:0] = ['.', '2048-ppo_amd']
import torch
import agent
from g2048 import urm
dev = torch.device('cuda', 0)
torch.manual_seed(3)
m = agent.GameURM(agent.GameURMConfig(dropout=0.0)).to(dev)
obs = torch.rand(512, 48, device=dev) * 8
for label in ("device", "nofused"):
    if label == "nofused":
        for f in ("attention_supported", "rms_res_supported", "swiglu_conv_supported", "stem_supported", "gate_up_swiglu_supported"):
            setattr(urm, f, lambda *a, **k: False)
    m.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lg, v = m(obs)
    (lg.float().square().sum() + v.float().sum()).backward()
    print(label, "no grad:", [k for k, p in m.named_parameters() if p.grad is None])
    print(label, "zero grad:", [k for k, p in m.named_parameters() if p.grad is not None and float(p.grad.abs().sum()) == 0])
