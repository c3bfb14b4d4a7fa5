"""torch.profiler census of the GameURM training iteration's torch-side ops (eager, no graph): which
aten ops launch the small elementwise / reduce / copy kernels between the device Functions.
    python tools/prof_urm_ops.py [envs] [horizon] [eager]   (eager: the update without its hipGraph --
    the same optimizer (the fused Muon/AdamW kernel) and device Functions as the captured update, so
    every launch is attributed to its aten op and input shapes)"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    from torch.profiler import ProfilerActivity, profile
    from g2048.trainer import TrainConfig, VecTrainer
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(steps=1000, lr=1e-3, critic_lr=1e-4, gamma=0.99, entropy=0.02, critic=0.2, episodes=envs,
                      batch_size=65536, hidden=64, model_type="urm", points=0.1, mono=1.0, rtg_beta=0.99,
                      warmup_steps=10, horizon=T, seed=0x2048, graph=False, amp=True)
    tr = VecTrainer(cfg, dev)
    if len(sys.argv) > 3 and sys.argv[3] == "eager":
        tr.ppo.graph = False  # the captured update's ops, launched one by one
    tr.train_step(0)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        tr.train_step(1)
        torch.cuda.synchronize()
    # every device kernel of the iteration: the library's (libg2048: urm_* / muon / colsum / env ...)
    # vs torch's own (at::native elementwise / reduce / copy, rocclr copy and fill blits), and torch's
    # per minibatch (minibatches = the loss launches, one urm_head_loss_kernel each; else the KL
    # re-forwards, the training-mode urm_forward_kernel<*, true>)
    kern = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    torch_k = [e for e in kern if "at::" in e.name or "rocclr" in e.name or "Memset" in e.name
               or "Memcpy" in e.name or e.name.startswith("void at_")]
    nmb = sum(1 for e in kern if "urm_head_loss_kernel" in e.name) or sum(
        1 for e in kern if "urm_forward_kernel" in e.name and ", true>" in e.name) or 1
    from collections import Counter
    print(f"device kernels: {len(kern)}; torch's: {len(torch_k)} over {nmb} minibatches + the rollout = "
          f"{len(torch_k) / nmb:.1f} per minibatch (upper bound: the rollout's are included)")
    for name, c in Counter(e.name[:90] for e in torch_k).most_common(12):
        print(f"  {c:6d}  {name}")
    ka = prof.key_averages()
    rows = sorted(ka, key=lambda e: -e.count)
    print(f"{'op':60s} {'count':>6s} {'dev_us':>10s}")
    for e in rows[:70]:
        if e.key.startswith("aten::") or "Function" in e.key or "Backward" in e.key:
            print(f"{e.key[:60]:60s} {e.count:6d} {e.device_time_total:10.0f}")
    print(ka.table(sort_by="device_time_total", row_limit=45, max_name_column_width=70))
    # the aten ops by input shape: which calls launch the small kernels
    ks = prof.key_averages(group_by_input_shape=True)
    rows = sorted((e for e in ks if e.key.startswith("aten::") and e.device_time_total > 0),
                  key=lambda e: -e.device_time_total)
    print(f"{'aten op':28s} {'count':>6s} {'dev_us':>9s}  input shapes")
    for e in rows[:40]:
        print(f"{e.key[:28]:28s} {e.count:6d} {e.device_time_total:9.0f}  {str(e.input_shapes)[:110]}")


if __name__ == "__main__":
    main()
