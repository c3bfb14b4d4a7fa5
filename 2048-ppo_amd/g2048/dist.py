"""Data parallelism: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm) or gloo (CPU tests).

The envs shard trivially (each rank owns its boards and its own Philox key), so the data path has
only two exchanges per train step:
  * the policy gradient: ONE all-reduce of a single flat fp32 bucket per optimizer step, issued
    before gradient clipping so every replica clips and steps identically; under RCCL it is captured
    inside the minibatch's hipGraph (one graph replay per minibatch, no host round trip);
  * the return-to-go batch statistics: one all-reduce of 3 float64 sums per train step.
"""

from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend: str | None = None) -> tuple[int, int, int]:
    """Initialise from torchrun's RANK/WORLD_SIZE/LOCAL_RANK (no-op for a single process)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, ws, local


def equal_rows(data: dict, n_real: int | None = None, generator: torch.Generator | None = None) -> dict:
    """Trim every rank's flat sample set to the smallest rank's row count (one MIN all-reduce), so all
    ranks run the same number of minibatches -- one gradient all-reduce each -- with equal minibatch
    sizes.  The first `n_real` rows are the real samples, D4 copies follow them:
    copies are dropped first (they are already a random subset); when a rank must also drop real
    rows (episodic mode) it keeps a uniformly random subset of them -- rows are time-major, so a
    tail trim would drop only the latest moves of every game."""
    m = next(iter(data.values())).shape[0]
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return data
    dev = next(iter(data.values())).device
    t = torch.tensor([m], dtype=torch.int64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return trim_rows(data, int(t.item()), n_real, generator)


def trim_rows(data: dict, k: int, n_real: int | None = None, generator: torch.Generator | None = None) -> dict:
    """Keep k rows of `data`: all real rows and the first copies when k >= n_real, else a random
    k-subset of the real rows (in their original order)."""
    m = next(iter(data.values())).shape[0]
    n_real = m if n_real is None else min(int(n_real), m)
    if k >= m:
        return data
    if k >= n_real:
        return {key: v[:k] for key, v in data.items()}
    dev = next(iter(data.values())).device
    gdev = generator.device if generator is not None else dev
    keep = torch.randperm(n_real, generator=generator, device=gdev)[:k].sort().values.to(dev)
    return {key: v.index_select(0, keep) for key, v in data.items()}


def graph(g, pool=None):
    """torch.cuda.graph(g, pool) for every capture of the package, in "thread_local" capture mode.

    torch's default "global" mode makes a capture-unsafe call from ANY thread of the process an
    error while the capture is open.  With a process group alive, ProcessGroupNCCL's watchdog thread
    polls the events of the eager collectives (hipEventQuery) every ~100 ms; a poll that lands inside
    one of our captures -- the minibatch graphs are captured right after two eager warm-up steps,
    whose all-reduces are still on the watchdog's list -- fails under "global" mode, and the
    watchdog turns the failure into an uncaught c10::DistBackendError on its own thread: SIGABRT with
    a C++ frame dump whose last frame is libc's thread start.  That is the shape of the RCCL child
    abort seen once in round 4.  "thread_local" keeps the capture-safety check for
    this thread, which issues all of the package's GPU work, and leaves the watchdog's queries
    alone."""
    import torch
    return torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local")


def _host_staged() -> bool:
    """gloo on device tensors (the CPU-backend tests of the device path: RCCL refuses two ranks on
    one GPU) goes through a host copy; RCCL ("nccl") takes the device tensor itself."""
    return dist.get_backend() == "gloo"


def allreduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if dist.is_initialized() and (dist.get_world_size() > 1 or dist.get_backend() == "nccl"):
        if t.is_cuda and _host_staged():
            h = t.cpu()
            dist.all_reduce(h)
            t.copy_(h)
        else:
            dist.all_reduce(t)
    return t


def allreduce_min_(t: torch.Tensor) -> torch.Tensor:
    """In-place MIN over the ranks (RCCL on the device tensor itself; gloo host-staged)."""
    if dist.is_initialized() and dist.get_world_size() > 1:
        if t.is_cuda and _host_staged():
            h = t.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MIN)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if dist.is_initialized() and dist.get_world_size() > 1:
        if t.is_cuda and _host_staged():
            h = t.cpu()
            dist.broadcast(h, src)
            t.copy_(h)
        else:
            dist.broadcast(t, src)
    return t


class GradBucket:
    """All parameter gradients as views of one flat fp32 buffer.

    Backward accumulates into the views in place, so the all-reduce is a single collective on a
    contiguous buffer (88 401 floats = 353 604 B for GameMLP h=196), and clipping is one norm.
    """

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        total = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n

    def zero(self):
        self.flat.zero_()

    @staticmethod
    def world() -> int:
        return dist.get_world_size() if dist.is_initialized() else 1

    @staticmethod
    def rccl() -> bool:
        return dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"

    @classmethod
    def capturable(cls) -> bool:
        """The gradient all-reduce can be captured into the minibatch hipGraph: RCCL ("nccl")
        collectives on device buffers are graph-capturable; gloo's host-staged path is not (the
        updater then splits its graph around an eager all-reduce)."""
        return cls.world() == 1 or cls.rccl()

    def allreduce_mean(self):
        """Mean of the flat bucket over the ranks.  Under RCCL the collective is issued even with a
        single rank (a one-rank all-reduce), so a world-size-1 RCCL run exercises -- and captures --
        the same call as the 8-GPU one."""
        w = self.world()
        if w > 1 or self.rccl():
            allreduce_sum_(self.flat)
            if w > 1:
                self.flat.div_(w)

    def clip_(self, max_norm: float) -> torch.Tensor:
        """torch.nn.utils.clip_grad_norm_ semantics on the flat buffer; returns the pre-clip norm."""
        norm = torch.linalg.vector_norm(self.flat)
        self.flat.mul_(torch.clamp(max_norm / (norm + 1e-6), max=1.0))
        return norm

    def check_views(self):
        """The bucket is only valid while every .grad still aliases it (zero_grad(set_to_none) breaks it)."""
        base = self.flat.data_ptr()
        return all(p.grad is not None and base <= p.grad.data_ptr() < base + self.flat.numel() * 4 for p in self.params)
