"""The RCCL ("nccl" backend) code path of the data-parallel update on the device (new
code -- the reference has no parallelism, /root/reference/train.py:1458).

A fresh child process initialises torch.distributed with the "nccl" backend (RCCL on ROCm) at world
size 1 BEFORE any other GPU call, the way bench.py / torch.distributed.run ranks do, then:
  * runs FusedPPOUpdater's minibatch step eagerly and captured: under RCCL the gradient all-reduce
    (a real one-rank RCCL all-reduce: GradBucket issues it whenever the backend is RCCL) is captured
    INSIDE the single minibatch hipGraph -- no split graph, no eager collective between replays --
    and the captured update is bitwise the eager one (parameters and statistics, 3 updates with a
    ragged padded last minibatch);
  * checks that the all-reduce really was issued during the capture (once per captured step);
  * runs two VecTrainer train steps (rollout, RTG, D4 up-sampling, graphed update) on that process
    group.
RCCL cannot put two ranks on one GPU, so the 2-rank case runs on gloo (tests/test_gpu_dist.py)."""

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child():
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)  # before any other GPU work
    sys.path[:0] = [str(ROOT), str(PKG)]
    from g2048 import _lib as L
    L.lds_poison(0x7FC07FC0)  # a fresh process: conftest's per-test LDS poison did not run here
    torch.cuda.synchronize()
    import numpy as np
    import agent
    from g2048.dist import GradBucket
    from g2048.fastmlp import FusedPPOUpdater
    from g2048.optim import FusedMuonAdamW
    from g2048.ppo import PPOConfig
    from g2048.trainer import TrainConfig, VecTrainer
    from test_gpu_ppo_fused import _synthetic_data
    rep = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    calls = {"captured": 0, "eager": 0}
    orig = dist.all_reduce

    def counting_all_reduce(t, *a, **k):
        calls["captured" if torch.cuda.is_current_stream_capturing() else "eager"] += 1
        return orig(t, *a, **k)
    dist.all_reduce = counting_all_reduce
    data = _synthetic_data(dev, 8192, seed=21)
    out = []
    for graph in (False, True):
        torch.manual_seed(3)
        m = agent.GameMLP(agent.MLPConfig(hidden_dim=196, num_layers=2, dropout=0.1)).to(dev)
        opt = FusedMuonAdamW(m, 1e-3, 1e-4)
        order = [p for p, _ in opt.muon] + [p for grp in opt.adam_groups for p in grp["params"]]
        gen = torch.Generator(device=dev)
        gen.manual_seed(5)
        bk = GradBucket(order)
        assert bk.capturable() and bk.rccl()
        up = FusedPPOUpdater(m, opt, PPOConfig(batch_size=3000, critic=0.2), bk, gen, graph=graph)
        before = dict(calls)
        sts = [{k: float(v) for k, v in up.update(data, 0.02).items()} for _ in range(3)]
        if graph:
            rep["split"] = up.graph_split
            rep["multi"] = up.MULTI
            rep["captured_allreduces"] = calls["captured"] - before["captured"]
            # replays issue no eager collective: only the capture warm-up's eager steps did
            rep["eager_allreduces_graph_run"] = calls["eager"] - before["eager"]
        else:
            rep["eager_allreduces"] = calls["eager"] - before["eager"]
        out.append((torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy(), sts))
    rep["params_equal"] = bool(np.array_equal(out[0][0], out[1][0]))
    rep["stats_equal"] = out[0][1] == out[1][1]
    rep["moved"] = bool(np.abs(out[1][0]).sum() > 0)
    cfg = TrainConfig(steps=10, episodes=1024, horizon=16, batch_size=4096, hidden=196, points=0.1, mono=1.0,
                      rtg_beta=0.99, gamma=0.99, entropy=0.02, critic=0.2, warmup_steps=0, upsample_ratio=0.25)
    tr = VecTrainer(cfg, dev)
    ms = [tr.train_step(s) for s in range(2)]
    rep["trainer_finite"] = all(np.isfinite(x["loss"]) and np.isfinite(x["grad_norm"]) for x in ms)
    rep["trainer_split"] = tr.ppo.graph_split
    torch.cuda.synchronize()
    print("RCCL_REPORT " + json.dumps(rep), flush=True)  # before the teardown: an abort there keeps it
    # teardown order: every graph holding a captured all-reduce goes before the communicator
    up.close()
    tr.close()
    del up, tr
    import gc
    gc.collect()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("RCCL_TEARDOWN_OK", flush=True)


@pytest.mark.gpu
def test_rccl_world1_captured_allreduce_graph_equals_eager(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env["PYTHONPATH"] = os.pathsep.join([str(ROOT / "tests"), str(ROOT), str(PKG), env.get("PYTHONPATH", "")])
    # the child's whole stdout / stderr go to a file (kept under gpurun_out/ on the GPU box, so a
    # failure's full C++ message -- which thread threw, and what -- survives the run)
    out_dir = ROOT / "gpurun_out" if os.environ.get("GRAFT_REPO_ROOT") else tmp_path
    out_dir.mkdir(parents=True, exist_ok=True)
    log = out_dir / "rccl_child_full.log"
    with open(log, "w") as f:
        r = subprocess.run([sys.executable, "-u", __file__, "--child"], env=env, stdout=f, stderr=subprocess.STDOUT,
                           text=True, timeout=300)
    text = log.read_text()
    lines = [x for x in text.splitlines() if x.startswith("RCCL_REPORT ")]
    if r.returncode != 0 or not lines or "RCCL_TEARDOWN_OK" not in text:
        pytest.fail(f"RCCL child exited {r.returncode} (full log: {log}):\n" + "\n".join(text.splitlines()[-80:]),
                    pytrace=False)
    rep = json.loads(lines[-1][len("RCCL_REPORT "):])
    print(rep)
    assert rep["backend"] == "nccl" and rep["world"] == 1
    assert rep["split"] is False and rep["trainer_split"] is False  # one graph per minibatch
    # the collective is a node of the captured minibatch steps: one in the one-step graph and one per
    # step of the MULTI-step graph (FusedPPOUpdater's offset path)
    assert rep["captured_allreduces"] == 1 + rep["multi"]
    assert rep["eager_allreduces"] == 3 * 3  # eager path: one per minibatch (3 updates x 3 minibatches)
    assert rep["params_equal"] and rep["stats_equal"] and rep["moved"]
    assert rep["trainer_finite"]


if __name__ == "__main__" and "--child" in sys.argv:
    _child()
