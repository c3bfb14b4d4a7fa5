"""Vectorised trainer: rollout -> reward/RTG/advantage -> PPO update, all on the device
(the train() loop of train.py:1669-1908 for N envs per GPU, one process per GPU).

Two rollout modes:
  episodic (horizon = 0, the reference's semantics): every env plays exactly one full game per
      train step (play_game_for_episode / play_games_batched); finished envs go inactive
      (G2048_OPT_SKIP_DONE) and the step ends when every game is over or --max-steps is reached.
  fixed horizon (horizon = T > 0, throughput mode): T steps of every env per train step with
      auto-reset; returns are cut at episode ends and bootstrap 0 at the horizon, like --max-steps.
"""

from __future__ import annotations

import math
import time
import warnings
from dataclasses import dataclass, field
from pathlib import Path

import torch

from . import _lib as L
from . import fastmlp
from . import urm as urm_mod
from . import urmppo
from .advantage import RewardWeights, RTGTracker
from .dist import GradBucket, allreduce_min_, allreduce_sum_, broadcast_, equal_rows, world
from .dist import graph as graph_capture
from .optim import FusedMuonAdamW, MuonAdamW, ScheduledMuonAdamW, build_optimizer
from .ppo import PPOConfig, PPOUpdater
from .rollout import Rollout, make_policy


@dataclass
class TrainConfig:
    steps: int = 1000
    lr: float = 1e-3
    critic_lr: float = 1e-3
    gamma: float = 0.99
    entropy: float = 0.1
    critic: float = 1.0
    episodes: int = 1              # envs per rank (--episodes)
    batch_size: int = 1
    epochs: int = 1
    max_steps: int | None = None
    hidden: int = 64
    num_layers: int = 2
    dropout: float = 0.1
    model_type: str = "mlp"        # "mlp" (GameMLP) or "urm" (GameURM, g2048/urm.py rollout policy)
    num_heads: int = 4             # URM only
    num_loops: int = 4
    num_truncated_loops: int = 1
    decouple_critic: bool = False
    points: float = 0.0
    mono: float = 0.0
    emptiness: float = 0.0
    rtg_beta: float = 0.9
    warmup_steps: int = 200
    beta1: float = 0.9
    beta2: float = 0.999
    weight_decay: float = 0.01
    adaptive_beta: bool = False
    target_entropy: float = 0.7
    beta_min: float = 0.001
    beta_max: float = 1.0
    beta_lr: float = 0.01
    upsample_ratio: float = 0.0    # --upsample-ratio: D4 copies of int(ratio * samples) samples (device kernel)
    horizon: int = 0
    seed: int = 0x2048
    graph: bool = True
    graph_update: bool = True      # hipGraph-captured PPO minibatch step (graph-safe Muon+AdamW)
    fused_update: bool = True      # GameMLP forward/backward as explicit kernels (g2048/fastmlp.py)
    amp: bool = True
    episodic_cap: int = 4096       # step cap of an episodic rollout without --max-steps
    chunk: int = 32                # episodic: steps between "all games over?" checks
    unused_weights: dict = field(default_factory=dict)


class VecTrainer:
    def __init__(self, cfg: TrainConfig, device, model: torch.nn.Module | None = None):
        import agent
        self.cfg = cfg
        self.dev = torch.device(device)
        self.rank, self.world = world()
        if model is None:
            if cfg.model_type == "urm":
                model = agent.GameURM(agent.GameURMConfig(hidden_dim=cfg.hidden, num_layers=cfg.num_layers,
                                                          num_heads=cfg.num_heads, dropout=cfg.dropout,
                                                          num_loops=cfg.num_loops,
                                                          num_truncated_loops=cfg.num_truncated_loops))
            else:
                model = agent.GameMLP(agent.MLPConfig(hidden_dim=cfg.hidden, num_layers=cfg.num_layers,
                                                      dropout=cfg.dropout, decouple_critic=cfg.decouple_critic))
            with torch.no_grad():  # train.py:1559-1567
                model.action_head.weight.zero_()
                model.action_head.bias.zero_()
                model.value_head.weight.zero_()
                model.value_head.bias.zero_()
        self.model = model.to(self.dev)
        if self.world > 1:  # identical initial replicas
            for p in self.model.parameters():
                broadcast_(p.data, 0)
        if cfg.graph_update:
            opt = None
            if cfg.fused_update and self.dev.type == "cuda":
                opt = FusedMuonAdamW(self.model, cfg.lr, cfg.critic_lr, cfg.beta1, cfg.beta2, cfg.weight_decay)
                if not opt.supported:
                    opt = None
            if opt is None:
                opt = MuonAdamW(self.model, cfg.lr, cfg.critic_lr, cfg.beta1, cfg.beta2, cfg.weight_decay)
            self.opt = ScheduledMuonAdamW(opt, cfg.warmup_steps, cfg.steps)
            # grads of the AdamW groups contiguous in the bucket (2-D first, then each 1-D group)
            order = [p for p, _ in opt.muon] + [p for g in opt.adam_groups for p in g["params"]]
            self.grads = GradBucket(order)
        else:
            self.grads = GradBucket(self.model.parameters())
            self.opt = build_optimizer(self.model, cfg.lr, cfg.critic_lr, cfg.beta1, cfg.beta2, cfg.weight_decay,
                                       cfg.warmup_steps, cfg.steps)
        # GameURM: bf16 copies of the projection weights written by the fused optimizer step (no cast
        # kernels per use in the update; the rollout and KL re-forward read them too)
        self.bf16w = (urm_mod.attach_bf16_weights(self.model, self.opt)
                      if cfg.graph_update and cfg.amp and isinstance(self.model, agent.GameURM) and self.dev.type == "cuda"
                      else None)
        self.policy = make_policy(self.model, torch.bfloat16 if cfg.amp else torch.float32)
        n = cfg.episodes
        self.episodic = cfg.horizon <= 0
        T = cfg.horizon if not self.episodic else (cfg.max_steps or cfg.episodic_cap)
        if self.episodic:
            T = int(math.ceil(T / cfg.chunk) * cfg.chunk)
        self.rollout = Rollout(n, T, self.dev, seed=cfg.seed + 7919 * self.rank, env_base=self.rank * n,
                               episodic=self.episodic, obs_dtype=torch.bfloat16 if cfg.amp else torch.float32)
        self.weights = RewardWeights(cfg.gamma, cfg.points, cfg.mono, cfg.emptiness, cfg.rtg_beta)
        self.rtg = RTGTracker(n, self.dev, self.weights, allreduce=allreduce_sum_ if self.world > 1 else None)
        gen = torch.Generator(device=self.dev)
        gen.manual_seed(cfg.seed + 104729 * self.rank)
        self.trim_gen = torch.Generator(device=self.dev)  # equal_rows' random row subset
        self.trim_gen.manual_seed(cfg.seed + 15485863 * (self.rank + 1))
        pcfg = PPOConfig(batch_size=cfg.batch_size, epochs=cfg.epochs, critic=cfg.critic,
                         amp_dtype=torch.bfloat16 if cfg.amp else None)
        # GameMLP's update is captured in a hipGraph; so is a GameURM's whose every training op is a
        # device Function (urm.training_graph_ok), otherwise it runs eagerly
        graph_up = cfg.graph_update and not self.episodic and (
            isinstance(self.model, agent.GameMLP)
            or (isinstance(self.model, agent.GameURM) and cfg.amp and self.dev.type == "cuda"
                and urm_mod.training_graph_ok(self.model)))
        if cfg.fused_update and cfg.amp and self.dev.type == "cuda" and fastmlp.supports(self.model):
            self.ppo = fastmlp.FusedPPOUpdater(self.model, self.opt, pcfg, self.grads, gen, graph=graph_up,
                                               seed=cfg.seed * 31 + self.rank)
        elif (cfg.fused_update and cfg.amp and self.dev.type == "cuda" and urm_mod.training_graph_ok(self.model)
              and urmppo.supports(self.model, pcfg.amp_dtype)):
            # GameURM: the loss, its backward and the KL statistics on device kernels
            self.ppo = urmppo.URMPPOUpdater(self.model, self.opt, pcfg, self.grads, gen, graph=graph_up)
            self.ppo.weight_cache = self.bf16w
        else:
            self.ppo = PPOUpdater(self.model, self.opt, pcfg, self.grads, gen, graph=graph_up)
            self.ppo.weight_cache = self.bf16w
        self.beta = cfg.entropy
        self.obs_mb = None
        self.run_score = torch.zeros(n, dtype=torch.int64, device=self.dev)
        self.run_maxexp = torch.zeros(n, dtype=torch.int32, device=self.dev)
        self.highest = 0
        self.ema = {"avg_score": 0.0, "pct_512": 0.0, "pct_1024": 0.0, "pct_2048": 0.0, "explained_var": 0.0}
        self._started = False
        self._pool = None  # sample pool (real + D4 copies) when --upsample-ratio > 0
        self._chunk_graphs = {}
        self.profile = False
        self.timings: dict[str, float] = {}
        for msg in self.fallbacks:
            warnings.warn(f"g2048: {msg}", stacklevel=2)

    def _update_forward_path(self) -> str:
        """The update's forward / backward path as FusedPPOUpdater decided it in its buffer allocation
        (fastmlp.FusedPPOUpdater._alloc: fused_pass / fused_back), or the static prediction before the
        first update has run."""
        import agent
        up = self.ppo
        if not isinstance(up, fastmlp.FusedPPOUpdater):
            if isinstance(self.model, agent.GameURM):
                return "URM device Functions" if self._urm_device_functions() else "autograd (library GEMMs / SDPA)"
            return "autograd"
        if up.bs:  # decided by _alloc for the current minibatch size
            if up.fused_pass:
                return "fused train / KL passes + " + ("fused backward" if up.fused_back else "per-layer backward")
            return "mlp_fwd kernels" if all(up.mf_ok) else "hipBLASLt + ln_act_fwd"
        pred = L.mlp_pass_supported(self.model.config.hidden_dim, len(self.model.backbone))
        return ("fused train / KL passes + fused backward" if pred else
                "mlp_fwd kernels" if all(up.mf_ok) else "hipBLASLt + ln_act_fwd") + " (predicted: no update yet)"

    def _urm_device_functions(self) -> bool:
        """Every training op of this GameURM runs on a device Function (urm.training_graph_ok) and
        its projections / heads fit the MFMA projection kernel (no torch.mm fallback in urm._gemm)."""
        m = self.model
        c = m.config
        inter = m.layers[0].mlp.inter
        return (self.dev.type == "cuda" and self.cfg.amp and urm_mod.training_graph_ok(m)
                and urm_mod.gemm_supported(3 * c.hidden_dim, c.hidden_dim) and urm_mod.gemm_supported(c.hidden_dim, c.hidden_dim)
                and urm_mod.gemm_supported(c.hidden_dim, inter) and urm_mod.gemm_supported(8, c.hidden_dim))

    @property
    def paths(self) -> dict:
        return self._fast_paths()[0]

    @property
    def fallbacks(self) -> list[str]:
        return self._fast_paths()[1]

    def _fast_paths(self) -> tuple[dict, list[str]]:
        """Which kernel path each phase runs on, and a message per phase that fell back from its
        fused kernel (shapes the kernels do not cover, e.g. -l 3 or -h 256; a GameURM off the device
        Functions or the captured update): the CLI prints them and bench.py puts `paths` /
        `fallbacks` in its JSON line, so a fallback is never silent.  Re-evaluated on every read: the
        update paths come from the updater's own decision once it has allocated its buffers."""
        import agent
        pol, up = self.policy, self.ppo
        mlp = isinstance(self.model, agent.GameMLP)
        urm = isinstance(self.model, agent.GameURM)
        inner = getattr(self.opt, "opt", self.opt)
        paths = {"policy": type(pol).__name__,
                 "rollout": "policy_rollout_kernel" if getattr(pol, "fused_rollout", False) else "per-step kernels",
                 "update": type(up).__name__,
                 "update_forward": self._update_forward_path(),
                 "optimizer": "fused Muon/AdamW kernels" if getattr(inner, "supported", False) else type(inner).__name__,
                 "update_graph": bool(getattr(up, "graph", False))}
        if urm:
            paths["urm_rollout"] = ("one-launch g2048_urm_forward" if getattr(pol, "mega", False)
                                    else "per-op kernels" if getattr(pol, "fused", False) else "torch.mm + kernels")
        fb = []
        fused_up = isinstance(up, fastmlp.FusedPPOUpdater)
        if mlp and self.dev.type == "cuda":
            h, nl = self.model.config.hidden_dim, len(self.model.backbone)
            if not getattr(pol, "fused_rollout", False):
                fb.append(f"rollout: no fused policy_rollout_kernel for GameMLP h={h}, {nl} blocks "
                          f"({paths['policy']} per step)")
            if self.cfg.amp and self.cfg.fused_update and not fused_up:
                fb.append(f"update: FusedPPOUpdater does not cover h={h}; autograd PPOUpdater")
            elif fused_up and not all(up.mf_ok):
                fb.append(f"update forward: no MFMA layer kernel for h={h}; hipBLASLt GEMM + ln_act_fwd")
            if self.cfg.graph_update and self.cfg.fused_update and not getattr(inner, "supported", False):
                fb.append(f"optimizer: the fused Muon kernel does not cover h={h}; torch-op Newton-Schulz")
            if isinstance(up, fastmlp.FusedPPOUpdater) and up.bs and not (up.fused_pass and up.fused_back):
                fb.append(f"update: {paths['update_forward']} instead of the fused passes + fused backward")
        if urm and self.dev.type == "cuda":
            h = self.model.config.hidden_dim
            if not self._urm_device_functions():
                fb.append(f"update: GameURM h={h} is not covered by the device Functions; autograd with library "
                          f"GEMMs / SDPA where a Function does not apply")
            if self.cfg.graph_update and not self.episodic and not getattr(up, "graph", False):
                fb.append("update: GameURM minibatch step runs eagerly (not captured in a hipGraph)")
            if not getattr(pol, "mega", False):
                fb.append(f"rollout: GameURM h={h} off the one-launch forward ({paths['urm_rollout']})")
            if self.cfg.graph_update and self.cfg.fused_update and not getattr(inner, "supported", False):
                fb.append("optimizer: the fused Muon kernel does not cover this GameURM; torch-op Newton-Schulz")
        return paths, fb

    # ------------------------------------------------------------------ rollout ---------------
    def _encode(self, boards: torch.Tensor) -> torch.Tensor:
        if self.obs_mb is None or self.obs_mb.shape[0] != boards.shape[0]:
            self.obs_mb = torch.empty(boards.shape[0], 48, dtype=torch.float32, device=self.dev)
        L.obs_encode(boards.contiguous(), self.obs_mb)
        return self.obs_mb

    def _collect_episodic(self):
        """Play every env's game until all are over or the step cap (--max-steps, train.py:240:
        `step < max_steps`) is reached; returns the number of steps played (<= the cap).  Steps run
        in chunks of `chunk` captured in hipGraphs; the last chunk stops at the cap."""
        ro, b = self.rollout, self.rollout.buf
        ro.reset()
        self.run_score.zero_()
        self.run_maxexp.zero_()
        cap = min(ro.T, self.cfg.max_steps or self.cfg.episodic_cap)
        used = 0
        for c0 in range(0, cap, self.cfg.chunk):
            c1 = min(c0 + self.cfg.chunk, cap)
            if self.cfg.graph:
                g = self._chunk_graphs.get((c0, c1))
                if g is None:
                    g = self._capture_chunk(c0, c1)
                    self._chunk_graphs[(c0, c1)] = g
                g.replay()
            else:
                ro.steps(c0, c1, self.policy)
            used = c1
            if bool(((b.flags[used] & L.FLAG_LEGAL) == 0).all()):  # every game is over
                break
        ro.counter.add_(2 * ro.T)
        return used

    def _capture_chunk(self, c0, c1):
        ro = self.rollout
        b = ro.buf
        snap = (b.boards[c0].clone(), b.flags[c0].clone())
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ro.steps(c0, c1, self.policy)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            ro.steps(c0, c1, self.policy)
        b.boards[c0].copy_(snap[0])
        b.flags[c0].copy_(snap[1])
        return g

    # ------------------------------------------------------------------ train step ------------
    def _mark(self, name: str):
        if self.profile:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._events.append((name, e))

    def _collect_timings(self):
        if self.profile and self._events:
            torch.cuda.synchronize()
            for (n0, e0), (n1, e1) in zip(self._events[:-1], self._events[1:]):
                self.timings[n1] = self.timings.get(n1, 0.0) + e0.elapsed_time(e1)
        self._events = []

    def train_step(self, step: int) -> dict:
        cfg, ro, b = self.cfg, self.rollout, self.rollout.buf
        self._events = []
        self._mark("start")
        self.model.eval()
        self.policy.sync()
        if self.episodic:
            T = self._collect_episodic()
        else:
            if not self._started:
                ro.reset()
                self._started = True
            else:
                b.carry_over()
            ro.collect(self.policy, graph=cfg.graph)
            T = ro.T
        self._mark("rollout_ms")
        self._last_T = T
        sf = b.step_flags[:T]
        self.rtg.compute(b.points[:T], b.pot[:T], sf, b.value[:T], b.g_raw[:T], b.g_norm[:T], b.adv[:T])
        self._mark("rtg_ms")
        n = ro.n
        data = {"boards": b.boards[:T].reshape(T * n, 16), "actions": b.actions[:T].reshape(-1),
                "legal": b.flags[:T].reshape(-1), "logp": b.logp[:T].reshape(T * n, 4),
                "adv": b.adv[:T].reshape(-1), "ret": b.g_norm[:T].reshape(-1)}
        if self.episodic:
            valid = torch.nonzero(((sf & L.FLAG_INACTIVE) == 0).reshape(-1)).squeeze(1)
            data = {k: v.index_select(0, valid) for k, v in data.items()}
        n_aug = 0
        n_real = data["actions"].shape[0]
        if cfg.upsample_ratio > 0 and self.world > 1 and not self.episodic:
            # fixed horizon, several ranks: every rank has the same n_real real rows, so equal_rows is
            # "keep the smallest rank's copy count": the MIN all-reduce runs on the device count and
            # ONE host read serves both the copy count and the trim (no separate count read)
            data, n_aug = self._augment(data, step, min_over_ranks=True)
        else:
            if cfg.upsample_ratio > 0:
                data, n_aug = self._augment(data, step)
            if self.world > 1:  # every rank runs the same number of minibatches (one all-reduce each)
                data = equal_rows(data, n_real, self.trim_gen)
        self._mark("augment_ms")
        ustats = self.ppo.update(data, self.beta, self._encode)
        self.opt.scheduler_step()
        self._mark("update_ms")
        metrics = self._metrics(T, ustats)
        metrics["augmented_samples"] = n_aug
        self._mark("metrics_ms")
        self._collect_timings()
        if cfg.adaptive_beta:  # train.py:1740-1746
            err = cfg.target_entropy - metrics["entropy"]
            self.beta = max(cfg.beta_min, min(cfg.beta_max, self.beta * (1.0 + cfg.beta_lr * err)))
        metrics["current_beta"] = self.beta
        return metrics

    def _augment(self, data: dict, step: int, min_over_ranks: bool = False):
        """calculate_advantage's D4 up-sampling (train.py:774-881) on the device: the real samples are
        copied into a fixed pool (stable pointers for the captured update) and g2048_augment appends
        the mirror / rotation copies of int(n * ratio) distinct samples.  Returns (pool views over
        real + copies, number of copies); one host read of the copy count.  min_over_ranks: the
        count is first MIN-all-reduced on the device (dist.equal_rows for equal real-row counts: the
        copies past the smallest rank's count are dropped), so that read is the only sync."""
        n = data["actions"].shape[0]
        k = min(int(n * self.cfg.upsample_ratio), n)
        cap = n + 2 * k
        if self._pool is None or self._pool["actions"].shape[0] < cap:
            cap = cap if not self.episodic else int(cap * 1.25) + 1  # episodic sizes vary per step
            self._pool = {key: torch.empty((cap,) + tuple(v.shape[1:]), dtype=v.dtype, device=self.dev)
                          for key, v in data.items()}
            self._aug_ws = torch.empty(L.augment_workspace_bytes(max(k, 1) * 2), dtype=torch.uint8, device=self.dev)
            self._aug_count = torch.zeros(1, dtype=torch.int64, device=self.dev)
        pool = self._pool
        for key, v in data.items():
            pool[key][:n].copy_(v)
        if self._aug_ws.numel() < L.augment_workspace_bytes(k):
            self._aug_ws = torch.empty(L.augment_workspace_bytes(k), dtype=torch.uint8, device=self.dev)
        L.augment(pool["boards"], pool["actions"], pool["legal"], pool["logp"], pool["adv"], pool["ret"], n, k,
                  self.cfg.seed * 131 + self.rank, step, self._aug_ws, self._aug_count)
        if min_over_ranks:
            allreduce_min_(self._aug_count)
        c = int(self._aug_count.item())
        return {key: v[:c] for key, v in pool.items()}, c - n

    # ------------------------------------------------------------------ metrics ---------------
    def _rollout_stats(self, T) -> torch.Tensor:
        """The rollout half of the metrics as one device vector [23] (g2048_rollout_stats: reward /
        advantage / return summaries and the finished games of compute_batch_stats, train.py:1040-1120,
        in two launches, no host sync; fixed horizon carries each env's running score / max tile
        across rollouts in run_score / run_maxexp)."""
        b = self.rollout.buf
        need = L.rollout_stats_workspace_bytes(T, self.rollout.n)
        if getattr(self, "_rs_ws", None) is None or self._rs_ws.numel() < need:
            self._rs_ws = torch.zeros(need, dtype=torch.uint8, device=self.dev)  # the key counter starts at 0
            self._rs_out = torch.empty(L.ROLLOUT_STATS, dtype=torch.float32, device=self.dev)
        if self.episodic:
            L.rollout_stats(b.points[:T], b.pot[:T], b.step_flags[:T], b.value[:T], b.g_raw[:T], b.g_norm[:T],
                            b.adv[:T], b.boards[:T + 1], None, True, self.weights.cfg(), None, None, self._rs_ws,
                            self._rs_out)
        else:
            L.rollout_stats(b.points[:T], b.pot[:T], b.step_flags[:T], b.value[:T], b.g_raw[:T], b.g_norm[:T],
                            b.adv[:T], b.boards[:T], b.max_tile[:T], False, self.weights.cfg(), self.run_score,
                            self.run_maxexp, self._rs_ws, self._rs_out)
        return self._rs_out

    def _metrics(self, T, ustats) -> dict:
        """The train step's metrics: the rollout half from g2048_rollout_stats (which also drops the
        inactive steps of episodic mode itself: FLAG_INACTIVE), the update half from the updater, and
        the fused Muon's sticky timeout count (raised on, never silent)."""
        inner = getattr(self.opt, "opt", self.opt)
        err = inner.error_count() if hasattr(inner, "error_count") else None
        parts = [self._rollout_stats(T), torch.stack([ustats[k] for k in (
            "loss", "policy_loss", "entropy_loss", "value_loss", "grad_norm", "entropy", "kl_total", "kl_average",
            "kl_max")])]
        if err is not None:
            parts.append(err.float())
        vec = torch.cat(parts).tolist()  # the one host synchronisation of the train step
        if err is not None:
            inner.check_errors(vec.pop())
        (n, rm, rv, zr, am, av, al2, amin, amax, gnm, gns, gnmin, gnmax, grs, vs, g0m, avg_s, med_s, max_s, p512,
         p1024, p2048, n_eps, loss, pl, el, vl, gnorm, ent, klt, kla, klm) = vec
        if not math.isfinite(gnorm):
            # torch's clip_grad_norm_ lets a NaN norm through into the step (the fused optimizer now
            # does the same, optim.hip clip_coef); the trainer does not train on silently
            raise FloatingPointError(f"non-finite gradient norm ({gnorm}) in this train step's update: "
                                     f"{self.nonfinite_report()}")
        if n_eps > 0:
            self.highest = max(self.highest, int(max_s))
            d = 0.001
            for k, val in (("avg_score", avg_s), ("pct_512", p512), ("pct_1024", p1024), ("pct_2048", p2048)):
                self.ema[k] = (1 - d) * self.ema[k] + d * val
        explained = 1.0 - av / (gns ** 2) if gns > 0 else 0.0
        self.ema["explained_var"] = (1 - 0.001) * self.ema["explained_var"] + 0.001 * explained
        lrs = [g["lr"] for g in self.opt.optimizers[0].param_groups]
        if len(lrs) == 4:  # MuonAdamW groups: other 2-D, other 1-D, value 2-D, value 1-D
            lrs = [lrs[0], lrs[2]]
        return {
            "samples": int(n), "augmented_samples": 0, "actor_loss": 0, "critic_loss": 0, "total_loss": 0,
            "policy_loss": pl, "entropy_loss": el, "value_loss": vl, "actor_grad_norm": 0, "critic_grad_norm": 0,
            "grad_norm": gnorm, "entropy": ent, "peak_score": self.highest, "avg_score": avg_s,
            "ema_avg_score": self.ema["avg_score"], "median_score": med_s, "avg_episode_return": g0m,
            "pct_512": p512, "ema_pct_512": self.ema["pct_512"], "pct_1024": p1024, "ema_pct_1024": self.ema["pct_1024"],
            "pct_2048": p2048, "ema_pct_2048": self.ema["pct_2048"], "reward_var": rv, "reward_mean": rm,
            "zero_reward_pct": zr, "advantage_mean": am, "advantage_var": av, "advantage_l2": al2, "adv_min": amin,
            "adv_max": amax, "G_norm_mean": gnm, "G_norm_std": gns, "G_norm_min": gnmin, "G_norm_max": gnmax,
            "G_raw_std": grs, "V_std": vs, "A_std": math.sqrt(max(av, 0.0)),
            "var_reduction": (gns - math.sqrt(max(av, 0.0))) / gns * 100 if gns > 0 else 0.0,
            "explained_var": explained, "ema_explained_var": self.ema["explained_var"], "kl_total": klt,
            "kl_average": kla, "kl_max": klm, "actor_lr": lrs[0], "critic_lr": lrs[1] if len(lrs) > 1 else lrs[0],
            "loss": loss, "episodes_finished": int(n_eps), "env_steps": int(n),
        }

    # ------------------------------------------------------------------ reports ---------------
    def best_episode(self) -> dict:
        """EpisodeData of the env with the most points in the last rollout (the reference's "best game
        this batch", train.py:1800): episodic mode = its whole game, fixed horizon = its window of
        T steps.  Records carry the device info deltas, advantages and rewards of that env."""
        from types import SimpleNamespace
        from .episodes import to_episode_data
        ro, b = self.rollout, self.rollout.buf
        T = self._last_T
        sf = b.step_flags[:T]
        live = (sf & L.FLAG_INACTIVE) == 0
        e = int(torch.where(live, b.points[:T], 0).sum(0).argmax())
        col = lambda x, k: x[:k, e:e + 1].contiguous()  # noqa: E731
        sub = SimpleNamespace(boards=col(b.boards, T + 1), flags=col(b.flags, T + 1), actions=col(b.actions, T),
                              logp=col(b.logp, T), entropy=col(b.entropy, T), value=col(b.value, T),
                              points=col(b.points, T), max_tile=col(b.max_tile, T), pot=col(b.pot, T),
                              device=b.device)
        sub.step_flags = sub.flags[1:]
        n_moves = live[:, e].sum().reshape(1)
        ep = to_episode_data(SimpleNamespace(buf=sub, n=1), T, n_moves, T)[0]
        adv, ret = b.adv[:T, e].tolist(), b.g_norm[:T, e].tolist()
        for k, m in enumerate(ep["moves"]):
            m["advantage"], m["future_reward"] = adv[k], ret[k]
        return ep

    # ------------------------------------------------------------------ evaluation ------------
    @torch.no_grad()
    def evaluate(self, games: int = 100, max_steps: int | None = None) -> dict:
        """train.py:1840-1876: `games` episodic games, game i seeded like random.seed(i)."""
        from .episodes import play_games
        was = self.model.training
        self.model.eval()
        res = play_games(self.model, games, max_steps, self.dev, seeds=list(range(games)), record=False)
        self.model.train(was)
        scores = res["scores"]
        tiles = res["max_tiles"]
        k = len(scores)
        srt = sorted(scores)
        return {"eval/max_score": max(scores), "eval/avg_score": sum(scores) / k, "eval/median_score": srt[k // 2],
                "eval/pct_512": sum(1 for t in tiles if t >= 512) / k * 100,
                "eval/pct_1024": sum(1 for t in tiles if t >= 1024) / k * 100,
                "eval/pct_2048": sum(1 for t in tiles if t >= 2048) / k * 100}

    def close(self):
        """Release every captured hipGraph (the update's -- holding the captured RCCL all-reduces at
        world > 1 -- the rollout's and the episodic chunks') once the device is idle.  Call before
        torch.distributed.destroy_process_group() (bench.py, the CLI, the RCCL test)."""
        if self.dev.type != "cuda":
            return
        torch.cuda.synchronize(self.dev)
        if hasattr(self.ppo, "close"):
            self.ppo.close()
        self.rollout._graph = None
        self._chunk_graphs.clear()
        torch.cuda.synchronize(self.dev)
        if self.bf16w is not None:  # the weights may be reused with another optimizer / a loaded state
            self.bf16w.detach()
            self.bf16w = None
        inner = getattr(self.opt, "opt", self.opt)
        if hasattr(inner, "check_errors"):  # a Muon hand-off timeout after the last metrics read
            inner.check_errors()

    def nonfinite_report(self) -> str:
        """Which gradient-bucket segments and parameters hold non-finite values (names, counts), for the
        error raised on a non-finite gradient norm.  One host read of per-tensor counts."""
        names = {id(p): n for n, p in self.model.named_parameters()}
        rows = []
        for p in self.grads.params:
            bad_g = int((~torch.isfinite(p.grad)).sum()) if p.grad is not None else 0
            bad_p = int((~torch.isfinite(p.detach())).sum())
            if bad_g or bad_p:
                rows.append(f"{names.get(id(p), '?')}: grad {bad_g}/{p.numel()}, param {bad_p}/{p.numel()}")
        inner = getattr(self.opt, "opt", self.opt)
        part = getattr(inner, "norm_part", None)
        if part is not None:
            rows.append(f"norm partials non-finite: {int((~torch.isfinite(part)).sum())}/{part.numel()}")
        return "; ".join(rows) if rows else "gradient bucket and parameters finite now (the last minibatch's bucket)"

    def save_checkpoint(self, path, eval_avg_score: float, train_step: int):
        import agent
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        cfg = getattr(self.model, "config", None)
        if not isinstance(cfg, (agent.MLPConfig, agent.GameURMConfig)):
            cfg = agent.MLPConfig(hidden_dim=self.cfg.hidden, num_layers=self.cfg.num_layers,
                                  decouple_critic=self.cfg.decouple_critic)
        torch.save({"model_state_dict": self.model.state_dict(), "config": cfg.model_dump(),
                    "eval_avg_score": eval_avg_score, "train_step": train_step,
                    "optimizer": self.opt.state_dict(), "rtg_state": self.rtg.state.cpu()}, path)


def smoke_iteration(device) -> dict:
    """One tiny fixed-horizon train step (smoke test of the whole path)."""
    cfg = TrainConfig(steps=10, episodes=256, horizon=16, batch_size=1024, hidden=32, points=0.1, mono=1.0,
                      rtg_beta=0.99, gamma=0.99, entropy=0.02, critic=0.2, warmup_steps=0, graph=True)
    tr = VecTrainer(cfg, device)
    t0 = time.perf_counter()
    m = tr.train_step(0)
    m2 = tr.train_step(1)
    return {"loss": m2["loss"], "entropy": m2["entropy"], "grad_norm": m["grad_norm"],
            "samples": m2["samples"], "seconds": time.perf_counter() - t0}
