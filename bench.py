#!/usr/bin/env python3
"""bench.py -- env-steps/s of the 2048 hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 65536] [--chunk 1024]

For N > 1 either launch it under torch.distributed.run (one rank per GPU, RCCL; WORLD_SIZE must
equal --gpus) or let it hand itself to torch.distributed.run: without WORLD_SIZE in the
environment and --gpus N > 1, the parent starts N fresh ranks before it touches the GPU and exits
with their status.  Workload (BASELINE.md /
SURVEY.md §8d): `--envs` independent 4x4 boards per GPU, uniform random legal actions (Philox
keyed by 0x2048 + rank), auto-reset on done.  One bench "step" = one launch of the fused
rollout kernel `env_rollout_kernel` = `--chunk` consecutive env steps of every board, writing the
full per-step trajectory record (board, action, points, potentials, flags); the launch (which also
advances its device-side Philox counter, in its last workgroup) is replayed from a hipGraph (host issue
cost: one graph launch per step).  value = total legal transitions of all ranks / max-over-ranks wall time of the K timed
steps (weak scaling: the boards per GPU are fixed; the envs are independent, so no data-path
collective exists).

Also reported in the same JSON line:
  roofline       env_rollout_kernel: SURVEY.md §8(d)'s 42 algorithmic bytes per env-step x env-steps
                 per launch / avg launch time (HIP events on the launch stream, timed region only)
                 against the HBM peak; the bytes the kernel really moves (26 B per step + 32 B per
                 board per launch) as a separate field; the VALU issue rate from the committed SQ
                 counters of this build, and `bound` = whichever of the two is nearer its peak
  sweep          the same kernel at 2^20 / 2^22 / 2^24 boards (beyond the 256 MiB Infinity Cache)
  single_step    the one-launch-per-step kernel (env_step_kernel, 42 B/step, §8d) captured in a
                 hipGraph, its steps/s and roofline
  train_loop     full training iteration (policy rollout with the MLP h=196 + reward/RTG scan +
                 PPO update with Muon/AdamW) when --train-iters > 0
  cpu_baseline   the CPU restatement (oracle/, rank 0 only) on a bounded sample of the workload
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "2048-ppo_amd"))
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak (spec)
VALU_ISSUE_PEAK = 1024 * 2.4e9 / 2  # wave-instructions/s: 1 024 SIMDs, one 64-lane VALU op per 2 cycles
# what the step's instruction mix can reach: at 65 536 boards there is one wave per SIMD, and one
# wave alone issues an independent VALU op per 4 cycles at best (MI355X_MICROARCH.md constants,
# 'vector-instruction ISSUE cost'); a second wave does not double it for this VOP3-heavy mix
# (v_bitop3 / v_perm / v_bcnt / v_pk_* / v_mad_u64 sustain ~4.6 cycles per wave-instruction per
# SIMD with 2 or 4 waves, profiles/r01e/valu_rate.log; the producer/consumer two-wave split of the
# rollout measured slower, profiles/r02d)
VALU_SINGLE_WAVE_PEAK = 1024 * 2.4e9 / 4
STEP_BYTES = 42  # SURVEY.md §8(d) algorithmic bytes per env-step: board in 16 + action 1 + board out 16
                 # + points 4 + flags 1 + pot 4 (the roofline basis)
ROLLOUT_STEP_BYTES = 16 + 1 + 4 + 4 + 1  # bytes the fused rollout really writes per env-step
ROLLOUT_LAUNCH_BYTES = 32  # ... plus per board per launch: board in + board out
SINGLE_STEP_BYTES = STEP_BYTES


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--chunk", type=int, default=1024,
                   help="env steps per rollout launch (one bench step; 256 before round 6: the per-launch "
                        "prologue -- table staging, per-board setup -- is then 4x less of the time)")
    p.add_argument("--launches-per-graph", type=int, default=8,
                   help="rollout launches captured per hipGraph replay (the timed steps stay K launches)")
    p.add_argument("--single-steps", type=int, default=256, help="graph-captured one-launch-per-step steps (0=off)")
    p.add_argument("--train-iters", type=int, default=3, help="timed full training iterations (0=off)")
    p.add_argument("--train-warmup", type=int, default=2)
    p.add_argument("--train-horizon", type=int, default=64)
    p.add_argument("--train-batch", type=int, default=65536)
    p.add_argument("--train-upsample", type=float, default=0.25, help="--upsample-ratio of the README command")
    p.add_argument("--urm-steps", type=int, default=16, help="GameURM policy rollout leg: steps per graph (0=off)")
    p.add_argument("--urm-iters", type=int, default=3, help="timed GameURM training iterations")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of each CPU-baseline leg (0=off)")
    p.add_argument("--sweep", default="1048576,4194304,16777216",
                   help="comma list of board counts for the rollout-kernel sweep ('' = off)")
    p.add_argument("--sweep-chunk", type=int, default=64, help="env steps per launch in the sweep")
    return p.parse_args()


def hand_off_to_ranks(args):
    """`--gpus N` without a torch.distributed.run environment: start N fresh ranks (one per GPU)
    through torch.distributed.run as a child process -- before this process touches the GPU -- and
    exit with their status.  Under a launcher, WORLD_SIZE must equal --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}; launch one rank per GPU")
        return
    if args.gpus <= 1:
        return
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    raise SystemExit(subprocess.call(cmd, env=env))


def setup_dist(args):
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return rank, world, local


def barrier(world):
    import torch.distributed as dist
    if world > 1:
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int) -> float:
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t)
    return float(t.item())


def graph_capture(g):
    from g2048.dist import graph
    return graph(g)


class RolloutBench:
    """Fused random-legal rollout: `chunk` env steps of every board per launch."""

    def __init__(self, n, chunk, rank, dev):
        import torch
        from g2048 import _lib as L
        from g2048.env import VecEnv
        self.L, self.n, self.chunk = L, n, chunk
        self.env = VecEnv(n, dev, seed=0x2048 + rank, env_base=rank * n)
        self.env.reset()
        self.tb = torch.empty(chunk, n, 16, dtype=torch.int8, device=dev)
        self.ta = torch.empty(chunk, n, dtype=torch.uint8, device=dev)
        self.tp = torch.empty(chunk, n, dtype=torch.int32, device=dev)
        self.tpot = torch.empty(chunk, n, 4, dtype=torch.int8, device=dev)
        self.tf = torch.empty(chunk, n, dtype=torch.uint8, device=dev)
        # the Philox counter base lives on the device: the launch (and its counter bump) can be
        # replayed from a hipGraph, so the host issue cost per bench step is one graph launch
        self.ctr = torch.ones(1, dtype=torch.int64, device=dev)
        self.rng = L.make_rng(L.RNG_PHILOX, self.env.seed, 0, self.env.env_base, counter_dev=self.ctr)
        # the launch advances the counter itself (its last workgroup: g2048_env_rollout_random_adv), so
        # consecutive launches in a graph have no counter-bump kernel between them
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        self.graph = None

    def launch(self):
        self.L.env_rollout_random(self.env.boards, self.chunk, self.tb, self.ta, self.tp, self.tpot, self.tf, self.rng,
                                  ticket=self.ticket)

    def capture(self, per_graph=1):
        """Two hipGraphs: `per_graph` consecutive launches (each with its counter bump) and a single
        one for the remainder, so K bench steps are K launches with fewer graph-launch gaps."""
        import torch
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.launch()  # warm-up outside the capture
        torch.cuda.current_stream().wait_stream(s)
        self.per_graph = max(1, per_graph)
        self.graph = torch.cuda.CUDAGraph()
        with graph_capture(self.graph):
            self.launch()
        self.graph_g = self.graph
        if self.per_graph > 1:
            self.graph_g = torch.cuda.CUDAGraph()
            with graph_capture(self.graph_g):
                for _ in range(self.per_graph):
                    self.launch()

    def step(self):
        self.graph.replay()

    def capture_exact(self, k):
        """One more hipGraph holding exactly k consecutive launches (k <= 256): run_exact(k) is then a
        single graph launch -- no host graph-launch gap inside the timed region."""
        import torch
        if getattr(self, "graph_k", None) is None:
            self.graph_k = {}
        if k in self.graph_k or not 0 < k <= 256:
            return
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            for _ in range(k):
                self.launch()
        self.graph_k[k] = g

    def run(self, k):
        """Exactly k launches (k bench steps): one replay of a k-launch graph when one was captured,
        else `per_graph`-launch graphs and single launches for the remainder."""
        gk = getattr(self, "graph_k", None) or {}
        if k in gk:
            gk[k].replay()
            return
        for _ in range(k // self.per_graph):
            self.graph_g.replay()
        for _ in range(k % self.per_graph):
            self.graph.replay()

    def bytes_per_launch(self):
        return self.n * (self.chunk * ROLLOUT_STEP_BYTES + ROLLOUT_LAUNCH_BYTES)


def time_region(fn, k, world):
    """Barrier + sync on both sides; HIP events on the launch stream bracket the same region."""
    import torch
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(k):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    return wall, e0.elapsed_time(e1) / 1e3


def bench_single_step(n, steps, rank, dev, world):
    """One launch per env step (env_step_kernel, §8d's 42 B/step), captured in a hipGraph so host
    launch overhead is excluded; the Philox counter base lives on the device and the graph bumps it."""
    import torch
    from g2048 import _lib as L
    from g2048.env import VecEnv
    env = VecEnv(n, dev, seed=0x3048 + rank, env_base=rank * n)
    env.reset()
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    aout = torch.empty(n, dtype=torch.uint8, device=dev)
    pts = torch.empty(n, dtype=torch.int32, device=dev)
    pot = torch.empty(n, 4, dtype=torch.int8, device=dev)
    fl = torch.empty(n, dtype=torch.uint8, device=dev)
    per_graph = 64

    def body():
        for t in range(per_graph):
            rng = L.make_rng(L.RNG_PHILOX, env.seed, t, env.env_base, counter_dev=ctr)
            L.env_step(env.boards, env.boards, None, aout, pts, None, pot, fl, rng, L.OPT_AUTO_RESET)
        ctr.add_(per_graph)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()  # warm-up outside capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with graph_capture(g):
        body()
    reps = max(1, steps // per_graph)
    g.replay()
    torch.cuda.synchronize()
    wall, ev = time_region(g.replay, reps, world)
    total = reps * per_graph
    wall = max_over_ranks(wall, world)
    ev = max_over_ranks(ev, world)
    avg = ev / total  # includes the per-launch dispatch gap inside the graph (conservative)
    return {
        "kernel": "env_step_kernel<Philox>",
        "steps_per_s": n * total * world / wall,
        "ms_per_env_step": wall / total * 1e3,
        "avg_launch_us": avg * 1e6,
        "roofline": {"bound": "hbm", "achieved": n * SINGLE_STEP_BYTES / avg / 1e9, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": n * SINGLE_STEP_BYTES / avg / 1e9 / HBM_PEAK_GBPS,
                     "bytes_per_step": SINGLE_STEP_BYTES},
    }


def cpu_baselines(seconds):
    """CPU restatements (oracle/, rank 0 only), each bounded by `seconds`: (1) game.step's pure-Python
    restatement (incl. the 17 heuristic evaluations of game.py:981-1002), random legal actions,
    auto-reset, 1 core; (2) the same loop on P processes (aggregate); (3) the README train loop
    (oracle/pyloop.py), 1 process; (4) the C oracle on P cores.  (1)-(3) are also reported scaled to
    the reference's own speed by the port/reference ratios measured in the build container
    (profiles/<tag>/cpu_ref_ratio.json, tools/cpu_ref_ratio.py)."""
    out = {}
    try:
        from oracle import oracle as O  # noqa: F401
        from oracle import pyloop, pyref
    except Exception as e:  # pragma: no cover
        return {"error": f"oracle unavailable: {e}"}
    import multiprocessing as mp
    # every core this job may use: the GPU box's CPU share is its OMP_NUM_THREADS (16 per GPU; nproc
    # there shows the whole machine), capped by the affinity mask
    visible = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cores = min(visible, share) if share > 0 else visible
    out["cores"] = {"used": cores, "visible": visible, "job_share": share or None}
    ratio = json.loads(CPU_RATIO.read_text()) if CPU_RATIO.exists() else None
    src = str(CPU_RATIO.relative_to(ROOT))

    def scaled(d, leg):
        if ratio:
            r = ratio[leg]["port_over_reference"]
            d.update(port_measured=d["value"], value=d["value"] / r, port_over_reference=r, ratio_source=src)
        return d
    # (1) pure-Python restatement, 1 core: the reference's own per-step cost structure
    r = pyref.time_random_steps(seconds)
    out["python_1core"] = scaled({"value": r["value"], "sample": r["sample"]}, "random_step")
    # (2) the same loop on `cores` processes
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        parts = pool.map(_py_chunk, [(seconds, 0x2048 + i) for i in range(cores)])
    dt = time.perf_counter() - t0
    out["python_pool"] = scaled({"value": sum(p["steps"] for p in parts) / dt, "unit": "env-steps/s", "cores": cores,
                                 "sample": f"{cores} procs x pure-Python random-legal loop, {dt:.1f} s wall"},
                                "random_step")
    # (3) README train loop (rollout + advantage + minibatch-4 Muon/AdamW update), 1 process
    t = pyloop.time_train_loop(seconds)
    out["train_loop_cpu"] = scaled({"value": t["value"], "unit": "env-steps/s", "cores": 1, "sample": t["sample"]},
                                   "train_loop")
    # (4) C oracle, all cores (process pool over independent env shards)
    n_envs, steps = 4096, 8
    t0 = time.perf_counter()
    _c_chunk((0, n_envs, steps))
    one = time.perf_counter() - t0
    steps = max(1, int(steps * seconds / max(one * 4, 1e-3)))
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        total = sum(pool.map(_c_chunk, [(i, n_envs, steps) for i in range(cores)]))
    dt = time.perf_counter() - t0
    out["c_oracle"] = {"value": total / dt, "unit": "env-steps/s", "cores": cores,
                       "sample": f"{cores} procs x {n_envs} boards x {steps} random-legal steps, full info heuristics"}
    return out


def _py_chunk(args):
    from oracle import pyref
    seconds, seed = args
    return pyref.time_random_steps(seconds, seed)


def _c_chunk(args):
    from oracle import oracle as O
    i, n, steps = args
    b = O.reset(n, O.RNG_PHILOX, seed=0x2048, env_base=i * n)
    cnt, _ = O.random_rollout(b, steps, seed=0x2048, step0=1, env_base=i * n, full_info=True)
    return cnt


PMC_PROFILE = ROOT / "profiles" / "r06q"  # round 6, final env kernel (env_rollout.hip, scheduler bias 0): 65 536 boards x 1024 steps per launch
CPU_RATIO = ROOT / "profiles" / "r05b" / "cpu_ref_ratio.json"  # re-measured in round 5 (r02: 1.45 / 1.14)


def rollout_counters():
    """Committed rocprofv3 counters of env_rollout_kernel for this build (tools/profile.sh +
    tools/pmc_sq.sh -> tools/summarize_rollout_pmc.py): per env-step HBM bytes (2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 FETCH correction) and per wave-step SQ instruction counts."""
    f = PMC_PROFILE / "pmc_env_rollout.json"
    if not f.exists():
        return None
    return dict(json.loads(f.read_text()), source=str(f.relative_to(ROOT)))


def rollout_roofline(rb, avg_launch_s, pmc):
    """roofline / valu blocks of the headline kernel for one launch of `rb` lasting avg_launch_s."""
    steps = rb.n * rb.chunk  # env-steps per launch
    achieved = steps * STEP_BYTES / avg_launch_s / 1e9
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "traffic_unit": "B/launch",
            "kernel": "env_rollout_kernel", "avg_launch_us": avg_launch_s * 1e6,
            "bytes_per_step": STEP_BYTES, "algorithmic_bytes_per_launch": steps * STEP_BYTES,
            "bytes_written_per_launch": rb.bytes_per_launch(),
            "bytes_written_GBps": rb.bytes_per_launch() / avg_launch_s / 1e9}
    valu = None
    if pmc:
        roof["traffic"] = pmc["hbm_bytes_per_env_step"] * steps
        roof["traffic_source"] = pmc["source"] + f" ({pmc['envs']} boards x {pmc['chunk']} steps per launch, scaled per env-step)"
        waves = -(-rb.n // 64)
        vws = pmc["valu_per_wave_step"]
        rate = vws * waves * rb.chunk / avg_launch_s
        valu = {"valu_per_wave_step": vws, "lds_per_wave_step": pmc["lds_per_wave_step"],
                "lds_bank_conflict_cycles_per_lds_inst": pmc["lds_conflict_per_lds_inst"],
                "waves_per_simd": waves / 1024,
                "cycles_per_valu_per_wave": avg_launch_s * 2.4e9 * min(1.0, 1024 / waves) / (vws * rb.chunk),
                "achieved": rate, "peak": VALU_ISSUE_PEAK, "unit": "wave-instructions/s",
                "single_wave_peak": VALU_SINGLE_WAVE_PEAK, "frac_single_wave": rate / VALU_SINGLE_WAVE_PEAK,
                "frac": rate / VALU_ISSUE_PEAK, "source": pmc["source"]}
        if valu["frac"] > roof["frac"]:
            roof["bound"] = "valu"
        roof["bound_basis"] = "nearer peak of HBM (42 B/step) and VALU issue (SQ_INSTS_VALU, 1 024 SIMDs x 1.2 G/s)"
    return roof, valu


def run_sweep(args, rank, world, dev) -> dict:
    """env_rollout_kernel at the --sweep board counts (--sweep-chunk steps per launch, 5 timed launches)."""
    import torch
    sweep = {}
    for s in [int(x) for x in args.sweep.split(",") if x]:
        b = RolloutBench(s, args.sweep_chunk, rank, dev)
        b.capture(1)
        b.step()
        torch.cuda.synchronize()
        k = 5
        w, e = time_region(b.step, k, world)
        w = max_over_ranks(w, world)
        sweep[str(s)] = {"env_steps_per_s_per_gpu": s * args.sweep_chunk * k / w, "chunk": args.sweep_chunk,
                         "launches": k, "avg_launch_us": e / k * 1e6,
                         "achieved_GBps_42B": s * args.sweep_chunk * STEP_BYTES / (e / k) / 1e9,
                         "written_GBps": b.bytes_per_launch() / (e / k) / 1e9}
        del b
        torch.cuda.empty_cache()
    return sweep


def main():
    args = parse()
    hand_off_to_ranks(args)  # --gpus N > 1 without a launcher: N fresh ranks, before any GPU call
    import torch
    rank, world, local = setup_dist(args)
    dev = torch.device("cuda", local)
    from g2048 import _lib as L
    L.load()

    rb = RolloutBench(args.envs, args.chunk, rank, dev)
    rb.capture(args.launches_per_graph)
    # the warm-up and the timed steps each as ONE graph launch (K <= 256; capture launches nothing):
    # with 8-launch graphs and single launches for the remainder, the driver's K = 20 paid ~6 host
    # graph launches inside the timed region (194.6 vs 186.7 us per launch at K = 200, profiles/r06f)
    rb.capture_exact(args.warmup)
    rb.capture_exact(args.steps)
    # the sweep and single-step legs (same kernels, other sizes) run before the headline's warm-up and
    # timed steps, so the headline is not the first GPU work of the process (profiles/r06f/warmup.txt)
    sweep = run_sweep(args, rank, world, dev) if args.sweep else None
    single = bench_single_step(args.envs, args.single_steps, rank, dev, world) if args.single_steps > 0 else None
    rb.run(args.warmup)
    torch.cuda.synchronize()
    wall, ev = time_region(lambda: rb.run(args.steps), 1, world)
    wall = max_over_ranks(wall, world)
    ev_max = max_over_ranks(ev, world)
    env_steps = args.envs * args.chunk * args.steps * world
    value = env_steps / wall
    roof, valu = rollout_roofline(rb, ev / args.steps, rollout_counters())
    roof["event_ms_max_rank"] = ev_max * 1e3
    roof["frac_of_value"] = value / world * STEP_BYTES / 1e9 / HBM_PEAK_GBPS  # same basis from the wall clock
    result = {
        "metric": "env-steps/sec (whole node) at 65536 parallel 4x4 boards, 1/2/4/8 MI355X",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic: random-legal-action rollouts (Philox keyed 0x2048+rank), auto-reset",
        "config": {"workload": f"{args.envs} boards/GPU x {args.chunk} env steps per launch, random legal policy",
                   "boards_per_gpu": args.envs, "env_steps_per_step": args.envs * args.chunk,
                   "launches_per_graph": args.steps if args.steps in (getattr(rb, "graph_k", None) or {}) else rb.per_graph,
                   "parallelism": f"env-shard x{world} (no data-path collective)"},
        "roofline": roof,
    }
    if valu:
        result["valu"] = valu
    del rb
    torch.cuda.empty_cache()

    if sweep is not None:
        result["sweep"] = sweep
    if single is not None:
        result["single_step"] = single

    if args.train_iters > 0:
        from g2048 import benchloop
        result["train_loop"] = benchloop.bench_train(args, rank, world, dev)

    if args.urm_steps > 0:
        from g2048 import benchloop
        result["urm"] = benchloop.bench_urm(args, rank, world, dev)

    # the CPU baseline on rank 0's host cores after every GPU leg (at world > 1 the other ranks wait
    # at the barrier below, so the timed GPU regions never share the host with it)
    if rank == 0 and args.cpu_seconds > 0:
        cb = cpu_baselines(args.cpu_seconds)
        py = cb.get("python_1core")
        if py:
            result["cpu_baseline"] = dict(py, unit="env-steps/s", cores=1, kind="port")
        for k in ("c_oracle", "python_pool", "train_loop_cpu", "cores"):
            if k in cb:
                result[f"cpu_baseline_{k}"] = cb[k]
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        barrier(world)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
