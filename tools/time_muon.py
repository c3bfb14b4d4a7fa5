"""Time the fused Muon + AdamW optimizer step (FusedMuonAdamW.step_clipped: grad clip, muon_kernel,
adamw_kernel) of GameMLP h=196 (or GameURM: hidden = "urm") with HIP events.
    python tools/time_muon.py [libpath|-] [hidden|urm] [quick]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from g2048 import _lib as L
    if len(sys.argv) > 1 and sys.argv[1] != "-":
        L._lib = L.load(sys.argv[1])  # every wrapper then calls this build
    import agent
    from g2048.dist import GradBucket
    from g2048.optim import FusedMuonAdamW
    urm = len(sys.argv) > 2 and sys.argv[2] == "urm"  # the default GameURMConfig's 11 matrices instead
    h = 64 if urm else int(sys.argv[2]) if len(sys.argv) > 2 else 196
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = (agent.GameURM(agent.GameURMConfig()) if urm else agent.GameMLP(agent.MLPConfig(hidden_dim=h, num_layers=2))).to(dev)
    fo = FusedMuonAdamW(m, 1e-3, 1e-4)
    order = [p for p, _ in fo.muon] + [p for grp in fo.adam_groups for p in grp["params"]]
    bk = GradBucket(order)
    bk.flat.copy_(torch.randn_like(bk.flat) * 1e-2)
    step = lambda: fo.step_clipped(bk.flat, 1.0)  # noqa: E731
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    e0.record()
    for _ in range(reps):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(f"FusedMuonAdamW.step_clipped h={h}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us per step (eager)")
    s = torch.cuda.Stream()  # the training path replays the step from a hipGraph: time that too
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(10):
                step()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps // 10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"FusedMuonAdamW.step_clipped h={h}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us per step (hipGraph)")
    for ns in (() if "quick" in sys.argv[3:] else (0, 1, 5)):  # split: prologue/epilogue (0 Newton-Schulz steps) vs per-step cost
        fo._cfg.ns_steps = ns
        e0.record()
        for _ in range(reps):
            step()
        e1.record()
        torch.cuda.synchronize()
        print(f"  ns_steps={ns}: {e0.elapsed_time(e1) / reps * 1e3:.1f} us")
    w = m.layers[0].attn.qkv_proj.weight if urm else m.backbone[0].mlp[0].weight
    print("checksum", float(w.double().sum()), float(w.double().abs().sum()))


if __name__ == "__main__":
    main()
