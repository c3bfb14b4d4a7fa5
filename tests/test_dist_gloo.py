"""World-size-2 data parallelism on CPU (gloo): the sharded PPO update with ONE flat-gradient
all-reduce per optimizer step equals the single-process update on the concatenated batch, replicas
stay bit-identical, and the 3-scalar RTG moment reduction composes across ranks."""

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n, seed):
    g = np.random.default_rng(seed)
    boards = g.integers(0, 10, size=(n, 16)).astype(np.int8)
    boards[g.random(boards.shape) < 0.4] = 0
    from oracle import oracle as O
    legal = O.legal_mask(boards)
    legal[legal == 0] = 1
    actions = np.array([[a for a in range(4) if m >> a & 1][0] for m in legal], np.uint8)
    logp = np.log(np.full((n, 4), 0.25, np.float32)) + g.normal(scale=0.1, size=(n, 4)).astype(np.float32)
    return {"boards": torch.from_numpy(boards), "actions": torch.from_numpy(actions),
            "legal": torch.from_numpy(legal.astype(np.uint8)), "logp": torch.from_numpy(logp),
            "adv": torch.from_numpy(g.normal(size=n).astype(np.float32)),
            "ret": torch.from_numpy(g.normal(size=n).astype(np.float32))}


def _encode(b):
    from oracle import oracle as O
    return torch.from_numpy(O.obs_encode(b.numpy()))


def _make(seed=0):
    import agent
    from g2048.dist import GradBucket
    from g2048.optim import build_optimizer
    from g2048.ppo import PPOConfig, PPOUpdater
    torch.manual_seed(seed)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=32, num_layers=2, dropout=0.0))
    opt = build_optimizer(m, 1e-3, 1e-4, warmup_steps=0, total_steps=10, schedule=False)
    return m, PPOUpdater(m, opt, PPOConfig(batch_size=1 << 20, amp_dtype=None), GradBucket(m.parameters()))


def _worker(rank, world, port, out):
    import sys
    from conftest import ROOT
    sys.path.insert(0, str(ROOT / "2048-ppo_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = _data(512, 1)
    shard = {k: v[rank * 256:(rank + 1) * 256] for k, v in full.items()}
    m, up = _make()
    st = up.update(shard, beta=0.02, encode=_encode)
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    # RTG moment reduction: shifted sums of each shard add up
    g = np.random.default_rng(5).normal(loc=40, scale=7, size=1000)
    mine = g[rank * 500:(rank + 1) * 500]
    shift = 38.5
    part = torch.tensor([(mine - shift).sum(), ((mine - shift) ** 2).sum(), float(len(mine))], dtype=torch.float64)
    dist.all_reduce(part)
    out[rank] = {"params": flat.numpy(), "same": all(torch.equal(gathered[0], x) for x in gathered),
                 "part": part.numpy(), "loss": float(st["loss"])}
    dist.destroy_process_group()


def test_two_rank_update_equals_single_process():
    import sys
    from conftest import ROOT
    sys.path.insert(0, str(ROOT / "2048-ppo_amd"))
    port = _free_port()
    with mp.Manager() as man:
        out = man.dict()
        mp.start_processes(_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    assert res[0]["same"] and res[1]["same"]
    m, up = _make()
    up.update(_data(512, 1), beta=0.02, encode=_encode)
    single = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).numpy()
    np.testing.assert_allclose(res[0]["params"], single, rtol=1e-4, atol=2e-6)
    g = np.random.default_rng(5).normal(loc=40, scale=7, size=1000)
    s1, s2, n = res[0]["part"]
    m1 = s1 / n
    mean, var = 38.5 + m1, s2 / n - m1 * m1
    assert np.isclose(mean, g.mean(), rtol=1e-12) and np.isclose(var, g.var(), rtol=1e-9)


def _ragged_worker(rank, world, port, out):
    """Ranks with different sample counts (D4 copies / episodic games vary per rank): equal_rows trims
    to the smallest, so both run the same number of minibatches and the update completes."""
    import sys
    from conftest import ROOT
    sys.path.insert(0, str(ROOT / "2048-ppo_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import agent
    from g2048.dist import GradBucket, equal_rows
    from g2048.optim import build_optimizer
    from g2048.ppo import PPOConfig, PPOUpdater
    data = equal_rows(_data(300 if rank == 0 else 257, 3 + rank))
    torch.manual_seed(0)
    m = agent.GameMLP(agent.MLPConfig(hidden_dim=32, num_layers=2, dropout=0.0))
    opt = build_optimizer(m, 1e-3, 1e-4, warmup_steps=0, total_steps=10, schedule=False)
    up = PPOUpdater(m, opt, PPOConfig(batch_size=100, amp_dtype=None), GradBucket(m.parameters()))
    up.update(data, beta=0.02, encode=_encode)
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    out[rank] = {"rows": int(data["actions"].shape[0]), "same": all(torch.equal(gathered[0], x) for x in gathered)}
    dist.destroy_process_group()


def test_unequal_rank_sample_counts_are_equalized():
    port = _free_port()
    with mp.Manager() as man:
        out = man.dict()
        mp.start_processes(_ragged_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
        res = dict(out)
    assert res[0]["rows"] == res[1]["rows"] == 257
    assert res[0]["same"] and res[1]["same"]
