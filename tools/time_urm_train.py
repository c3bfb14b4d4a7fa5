import sys, time, torch
sys.path[:0]=['/root/repo','/root/repo/2048-ppo_amd']
import agent
from torch.nn.attention import sdpa_kernel, SDPBackend
dev=torch.device('cuda',0)
drop=float(sys.argv[1]) if len(sys.argv)>1 else 0.1
m=agent.GameURM(agent.GameURMConfig(dropout=drop)).to(dev)
print('dropout',drop)
obs=torch.rand(65536,48,device=dev)*8
def step():
    with torch.autocast('cuda',dtype=torch.bfloat16):
        l,v=m(obs)
    (l.float().sum()+v.float().sum()).backward()
for name, ctx in (("default", None), ("math", SDPBackend.MATH), ("efficient", SDPBackend.EFFICIENT_ATTENTION)):
    try:
        for rep in range(2):
            torch.cuda.synchronize(); t=time.perf_counter()
            if ctx is None: step()
            else:
                with sdpa_kernel([ctx]): step()
            torch.cuda.synchronize(); dt=time.perf_counter()-t
        print(name, f"{dt*1e3:.1f} ms per fwd+bwd of 65536 boards")
    except Exception as e:
        print(name, "failed", e)
