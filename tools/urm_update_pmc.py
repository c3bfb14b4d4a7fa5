"""GPU program for the GameURM update's HBM counters (BASELINE config 5 on one GPU, the bench's URM
training leg): a VecTrainer at the bench's configuration runs one train step (graph capture), then a
second one whose PPO update is bracketed by two marker dispatches (g2048_lds_poison with word 0, a
kernel no other code launches), each behind a device synchronize.  Run under rocprofv3 --pmc
FETCH_SIZE / --pmc WRITE_SIZE (tools/gpu/check.sh urmhbm); tools/urm_update_hbm.py sums the
dispatches between the markers into profiles/<tag>/urm_update_hbm.json, which bench.py's URM leg
reads for urm.train_iter.roofline.update_hbm.

    python3 tools/urm_update_pmc.py [envs] [horizon] [minibatch]
"""

import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "2048-ppo_amd")]


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    mb = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    from g2048 import _lib as L
    from g2048.trainer import TrainConfig, VecTrainer
    dev = torch.device("cuda", 0)
    cfg = TrainConfig(steps=1000, lr=1e-3, critic_lr=1e-4, gamma=0.99, entropy=0.02, critic=0.2, episodes=envs,
                      batch_size=mb, hidden=64, model_type="urm", points=0.1, mono=1.0, rtg_beta=0.99,
                      warmup_steps=10, horizon=T, seed=0x2048, graph=True, amp=True)  # = benchloop.bench_urm
    tr = VecTrainer(cfg, dev)
    tr.train_step(0)
    torch.cuda.synchronize()
    orig = tr.ppo.update
    seen = {}

    def update(data, beta, encode=None):
        seen["rows"] = int(data["actions"].shape[0])
        torch.cuda.synchronize()
        L.lds_poison(0)  # marker: start of the update
        torch.cuda.synchronize()
        r = orig(data, beta, encode)
        torch.cuda.synchronize()
        L.lds_poison(0)  # marker: end of the update
        torch.cuda.synchronize()
        return r
    tr.ppo.update = update
    m = tr.train_step(1)
    tr.close()
    print("URM_UPDATE_PMC " + json.dumps({"envs": envs, "horizon": T, "minibatch": mb, "rows": seen["rows"],
                                           "minibatches": -(-seen["rows"] // mb), "loss": m["loss"]}), flush=True)


if __name__ == "__main__":
    main()
