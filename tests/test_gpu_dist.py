"""The multi-rank training path on device tensors (new code: the reference has no
parallelism, /root/reference/train.py:1458): two fresh ranks on cuda:0 with the gloo backend run
VecTrainer with the kernel-written PPO step (fastmlp.FusedPPOUpdater: its hipGraph split in two
around the eager gradient all-reduce, g2048/ppo.py) for 2 fixed-horizon train steps, with
dropout 0 and D4 up-sampling (so the ranks' sample counts differ and dist.equal_rows trims them).

Checked across the ranks:
  * the replicas stay bitwise identical (same update from the same all-reduced gradient);
  * the all-reduced bucket of the first minibatches equals the mean of the two ranks' local buckets;
  * the RTG batch moments (advantage.RTGTracker's 24-byte partials reduce) equal those of the
    concatenated trajectories of both ranks;
  * equal_rows gave both ranks the same sample count, hence the same minibatch count.
Both policies: GameMLP (FusedPPOUpdater) and GameURM (PPOUpdater over g2048/urm.py's device
Functions, the reference's game.py:1355-1458 model).  RCCL cannot put two ranks on one GPU, so the
collectives here are gloo's CUDA-tensor all-reduces (host staged, hence the split graph); the RCCL
path -- the all-reduce captured inside the minibatch graph -- is tests/test_gpu_rccl.py."""

import os
import socket
import sys

import numpy as np
import pytest
import torch

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

STEPS = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, model_type="mlp"):
    for p in (str(ROOT), str(PKG)):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from g2048 import fastmlp
    from g2048.trainer import TrainConfig, VecTrainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from g2048 import _lib as L
    # a spawned rank is a fresh process: conftest's autouse poison ran only in the pytest process, so
    # each rank fills every CU's LDS with the NaN pattern itself before its first kernel (a kernel of
    # the path that reads LDS it did not write then turns it into NaN here, not on one box in ten)
    L.lds_poison(0x7FC07FC0)
    torch.cuda.synchronize()
    torch.manual_seed(rank)  # different local inits: VecTrainer must broadcast rank 0's replica
    if model_type == "urm":  # GameURM (default config: h 64, 2 layers, 4 heads, 4 / 1 loops) on its device Functions
        cfg = TrainConfig(steps=10, episodes=256, horizon=8, batch_size=1024, hidden=64, model_type="urm",
                          dropout=0.0, points=0.1, mono=1.0, rtg_beta=0.99, gamma=0.99, entropy=0.02, critic=0.2,
                          warmup_steps=0, upsample_ratio=0.25)
    else:
        cfg = TrainConfig(steps=10, episodes=512, horizon=16, batch_size=2048, hidden=196, dropout=0.0, points=0.1,
                          mono=1.0, rtg_beta=0.99, gamma=0.99, entropy=0.02, critic=0.2, warmup_steps=0,
                          upsample_ratio=0.25)
    tr = VecTrainer(cfg, dev)
    rec = {"before": [], "after": [], "rows": [], "nb": [], "g_raw": [], "moments": []}
    if model_type == "urm":
        from g2048 import urm as urm_mod
        assert not isinstance(tr.ppo, fastmlp.FusedPPOUpdater) and tr.ppo.graph == urm_mod.training_graph_ok(tr.model)
        assert tr.ppo.graph  # the captured (split) URM minibatch step
    else:
        assert isinstance(tr.ppo, fastmlp.FusedPPOUpdater) and tr.ppo.graph
    bucket = tr.grads
    orig_ar = bucket.allreduce_mean

    def allreduce_mean():
        keep = len(rec["before"]) < 3
        if keep:
            rec["before"].append(bucket.flat.cpu().numpy().copy())
        orig_ar()
        if keep:
            rec["after"].append(bucket.flat.cpu().numpy().copy())
    bucket.allreduce_mean = allreduce_mean
    orig_up = tr.ppo.update

    def update(data, beta, encode=None):
        m = int(data["actions"].shape[0])
        rec["rows"].append(m)
        rec["nb"].append(-(-m // cfg.batch_size))
        return orig_up(data, beta, encode)
    tr.ppo.update = update
    # every minibatch's gradient norm, read right after its step (the split path's g2 replay): an
    # intermittent non-finite grad_norm with a finite loss / KL was seen in this MLP test (r04c, r05d,
    # DESIGN.md §7); a recurrence names its minibatch and the non-finite bucket segments / parameters
    inner = getattr(tr.opt, "opt", tr.opt)
    rec["norms"] = []

    def checked(fn):  # the graphed minibatch (_replay) and the eager one (_minibatch: warm-ups, ragged URM)
        def run(*args):
            fn(*args)
            nt = getattr(inner, "norm_t", None)
            if nt is None:
                return
            v = float(nt)
            if not np.isfinite(v):
                raise AssertionError((rank, "minibatch", len(rec["norms"]), v, tr.nonfinite_report(),
                                      inner.norm_part.cpu().tolist()))
            rec["norms"].append(v)
        return run
    tr.ppo._replay = checked(tr.ppo._replay)
    tr.ppo._minibatch = checked(tr.ppo._minibatch)
    for s in range(STEPS):
        m = tr.train_step(s)  # raises FloatingPointError itself on a non-finite norm (trainer._metrics)
        assert np.isfinite(m["loss"]) and np.isfinite(m["grad_norm"]), (rank, s, m)
        T = tr.rollout.T
        rec["g_raw"].append(tr.rollout.buf.g_raw[:T].reshape(-1).double().cpu().numpy())
        rec["moments"].append(tr.rtg.state.cpu().numpy().copy())
    torch.cuda.synchronize()
    rec["params"] = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()]).cpu().numpy()
    out[rank] = rec
    tr.close()  # graphs before the process group (teardown order)
    dist.destroy_process_group()


@pytest.mark.parametrize("model_type", ["mlp", "urm"])
def test_two_ranks_fused_update_on_device(model_type):
    """GameMLP: the kernel-written FusedPPOUpdater; GameURM (BASELINE config 5's policy): PPOUpdater
    over the URM device autograd Functions, captured in the same split graph."""
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    port = _free_port()
    with mp.Manager() as man:
        out = man.dict()
        mp.start_processes(_worker, args=(2, port, out, model_type), nprocs=2, join=True, start_method="spawn")
        r0, r1 = out[0], out[1]
    # same sample count and minibatch count on both ranks, every train step
    assert r0["rows"] == r1["rows"] and r0["nb"] == r1["nb"] and len(r0["rows"]) == STEPS
    # the per-minibatch norms were read on every graphed minibatch and agree across the replicas
    # (the same all-reduced bucket)
    assert len(r0["norms"]) >= sum(r0["nb"]) and r0["norms"] == r1["norms"]
    assert len(r0["before"]) == 3 and len(r1["before"]) == 3
    # the all-reduced bucket is the mean of the two local ones (sum then / 2: exact in fp32)
    for k in range(3):
        want = (r0["before"][k] + r1["before"][k]) / np.float32(2)
        assert not np.array_equal(r0["before"][k], r1["before"][k])  # the shards' gradients differ
        np.testing.assert_array_equal(r0["after"][k], want)
        np.testing.assert_array_equal(r1["after"][k], want)
    # replicas bitwise identical after both train steps (and they did move)
    assert np.array_equal(r0["params"], r1["params"])
    # RTG batch moments of the concatenated trajectories (state[6:8] = batch mean, population var)
    for s in range(STEPS):
        g = np.concatenate([r0["g_raw"][s], r1["g_raw"][s]])
        for r in (r0, r1):
            mean, var = r["moments"][s][6], r["moments"][s][7]
            # g_raw is stored fp32 (the moments are of the fp64 values): 2^-24 relative per element
            np.testing.assert_allclose(mean, g.mean(), rtol=1e-6, atol=1e-6 * g.std())
            np.testing.assert_allclose(var, g.var(), rtol=2e-5)
        np.testing.assert_array_equal(r0["moments"][s], r1["moments"][s])
