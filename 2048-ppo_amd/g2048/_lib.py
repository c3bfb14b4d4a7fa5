"""ctypes binding of libg2048.so (include/g2048.h) for torch tensors on a ROCm device.

This is the Python seam of the C ABI: every function takes torch tensors that already live on the
GPU, passes their data pointers and torch's current HIP stream, and raises on a non-zero status.
There is no CPU fallback: a missing library or a CPU tensor is an error (fail loudly).
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

LIB_PATH = Path(__file__).resolve().parent / "libg2048.so"

UP, DOWN, LEFT, RIGHT = 0, 1, 2, 3
RNG_PHILOX, RNG_MT19937, RNG_INJECT = 0, 1, 2
OPT_AUTO_RESET, OPT_SKIP_DONE = 0x1, 0x2
FLAG_LEGAL, FLAG_INVALID, FLAG_RESET, FLAG_INACTIVE, FLAG_DONE = 0x0F, 0x10, 0x20, 0x40, 0x80
DTYPE_F32, DTYPE_BF16 = 0, 1
RTG_STATE_DOUBLES = 8

EXPORTED = (
    "g2048_mt_state_words", "g2048_mt_seed", "g2048_env_reset", "g2048_env_step", "g2048_env_rollout_random",
    "g2048_env_rollout_random_adv",
    "g2048_preview_points", "g2048_legal_mask",
    "g2048_obs_encode", "g2048_info_deltas", "g2048_sample_actions", "g2048_rtg_prepare", "g2048_reward_rtg_workspace_bytes",
    "g2048_reward_rtg", "g2048_reward_rtg_ex", "g2048_rtg_finalize", "g2048_build_info", "g2048_episode_scan",
    "g2048_rollout_stats_workspace_bytes", "g2048_rollout_stats", "g2048_permutation",
    "g2048_augment_workspace_bytes", "g2048_augment",
    # include/g2048_ppo.h
    "g2048_obs_gather", "g2048_ln_act_fwd", "g2048_ln_act_bwd_partials", "g2048_ln_act_bwd",
    "g2048_ppo_head_partials", "g2048_ppo_head_loss", "g2048_ppo_head_kl", "g2048_dropout_mask", "g2048_colsum_batch",
    "g2048_colsum_batch_blocks", "g2048_colsum_batch_sq",
    "g2048_wgrad_partials", "g2048_wgrad", "g2048_wgrad_pair_partials", "g2048_wgrad_pair", "g2048_linear_dgrad_supported", "g2048_linear_dgrad",
    "g2048_grad_clip", "g2048_muon_supported", "g2048_muon_step", "g2048_adamw_step",
    "g2048_grad_sumsq", "g2048_muon_step_clip", "g2048_muon_workspace_bytes", "g2048_muon_error_offset", "g2048_lds_poison", "g2048_grad_sumsq_tick", "g2048_muon_adamw_step_clip", "g2048_mlp_fwd_kl", "g2048_urm_attention_bwd", "g2048_urm_attention_drop", "g2048_urm_attention_bwd_drop", "g2048_urm_attention_drop_at", "g2048_urm_attention_bwd_drop_at", "g2048_urm_stem_partials", "g2048_urm_stem_fwd", "g2048_urm_stem_bwd", "g2048_urm_stem_bwd3", "g2048_urm_rms_res_fwd2", "g2048_urm_rms_res_bwd2", "g2048_urm_rms_res_bwd3", "g2048_urm_add_cast", "g2048_urm_add_cast_bwd", "g2048_urm_add_cast_bwd_acc", "g2048_urm_forward_drop", "g2048_urm_rms_res_fwd",
    "g2048_urm_rms_res_bwd", "g2048_urm_swiglu_conv_partials", "g2048_urm_swiglu_conv_fwd", "g2048_urm_swiglu_conv_bwd",
    "g2048_mlp_fwd_lds_bytes", "g2048_mlp_fwd", "g2048_head_fwd", "g2048_ppo_stats",
    "g2048_policy_rollout_supported", "g2048_policy_rollout_lds_bytes", "g2048_policy_rollout",
    "g2048_head_split_bytes", "g2048_head_split", "g2048_mlp_pass_supported", "g2048_mlp_pass_partials",
    "g2048_ppo_forward_loss", "g2048_ppo_forward_kl", "g2048_ppo_forward_kl_stats", "g2048_mlp_back_partials", "g2048_ppo_backward",
    "g2048_mlp_wgrad_partials", "g2048_mlp_wgrad",
    # include/g2048_urm.h
    "g2048_urm_stem", "g2048_urm_attention", "g2048_urm_residual_rms", "g2048_urm_swiglu_conv",
    "g2048_urm_pool_heads", "g2048_urm_linear_supported", "g2048_urm_linear", "g2048_urm_linear_rms",
    "g2048_urm_linear_swiglu", "g2048_urm_linear_swiglu_train", "g2048_urm_linear_t", "g2048_urm_gate_up_swiglu_bwd_supported", "g2048_urm_gate_up_swiglu_bwd", "g2048_urm_gate_up_swiglu_bwd_acc", "g2048_urm_linear_res_rms", "g2048_urm_linear_bias", "g2048_urm_wgrad_supported", "g2048_urm_wgrad_partials", "g2048_urm_wgrad", "g2048_urm_wgrad_acc", "g2048_urm_linres_bwd_supported", "g2048_urm_linres_bwd_partials", "g2048_urm_linres_bwd", "g2048_urm_head_loss_partials", "g2048_urm_head_loss", "g2048_urm_head_loss_bwd", "g2048_urm_kl_stats", "g2048_urm_forward_supported", "g2048_urm_forward",
)


class G2048Error(RuntimeError):
    pass


class Rng(ctypes.Structure):
    """struct g2048_rng"""
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("env_base", ctypes.c_uint32),
        ("seed", ctypes.c_uint64),
        ("counter", ctypes.c_uint64),
        ("counter_dev", ctypes.c_void_p),
        ("mt_state", ctypes.c_void_p),
        ("inject", ctypes.c_void_p),
    ]


class UrmWeights(ctypes.Structure):
    """struct g2048_urm_weights"""
    _fields_ = [("hidden", ctypes.c_int32), ("heads", ctypes.c_int32), ("inter", ctypes.c_int32),
                ("num_layers", ctypes.c_int32), ("num_loops", ctypes.c_int32), ("eps", ctypes.c_float),
                ("stem_w", ctypes.c_void_p), ("ln_w", ctypes.c_void_p), ("ln_b", ctypes.c_void_p),
                ("init_hidden", ctypes.c_void_p), ("wa", ctypes.c_void_p), ("ba", ctypes.c_void_p),
                ("wv", ctypes.c_void_p), ("bv", ctypes.c_void_p), ("qkv", ctypes.c_void_p * 2),
                ("o", ctypes.c_void_p * 2), ("gate_up", ctypes.c_void_p * 2), ("down", ctypes.c_void_p * 2),
                ("conv_w", ctypes.c_void_p * 2), ("conv_b", ctypes.c_void_p * 2)]


class RewardCfg(ctypes.Structure):
    """struct g2048_reward_cfg"""
    _fields_ = [("gamma", ctypes.c_double), ("w_points", ctypes.c_double), ("w_mono", ctypes.c_double),
                ("w_empt", ctypes.c_double), ("beta", ctypes.c_double)]


class Dropout(ctypes.Structure):
    """struct g2048_dropout"""
    _fields_ = [("p", ctypes.c_float), ("layer", ctypes.c_uint32), ("pass_", ctypes.c_uint32),
                ("pad_", ctypes.c_uint32), ("seed", ctypes.c_uint64), ("counter", ctypes.c_uint64),
                ("counter_dev", ctypes.c_void_p)]


class PPOBatch(ctypes.Structure):
    """struct g2048_ppo_batch"""
    _fields_ = [("idx", ctypes.c_void_p), ("action", ctypes.c_void_p), ("legal", ctypes.c_void_p),
                ("old_logp", ctypes.c_void_p), ("adv", ctypes.c_void_p), ("ret", ctypes.c_void_p),
                ("rows", ctypes.c_void_p)]


DY_MAX_P = 4
COLSUM_SEGS = 5
COLSUM_MAX_JOBS = 16
COLSUM_SQ_MAX = 1024


class ColsumJob(ctypes.Structure):
    """struct g2048_colsum_job: a deferred fixed-order column sum"""
    _fields_ = [("part", ctypes.c_void_p), ("nb", ctypes.c_int32), ("cols", ctypes.c_int32),
                ("max_col", ctypes.c_int32), ("nseg", ctypes.c_int32), ("dst", ctypes.c_void_p * COLSUM_SEGS),
                ("len", ctypes.c_int32 * COLSUM_SEGS), ("pad_", ctypes.c_int32)]


class Dy(ctypes.Structure):
    """struct g2048_dy: the sources of a block's output gradient"""
    _fields_ = [("dres", ctypes.c_void_p), ("p", ctypes.c_void_p * DY_MAX_P), ("dz", ctypes.c_void_p),
                ("wa", ctypes.c_void_p), ("wv", ctypes.c_void_p)]


class MuonMatrix(ctypes.Structure):
    """struct g2048_muon_matrix"""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("momentum", ctypes.c_void_p),
                ("param_bf16", ctypes.c_void_p), ("head_frag", ctypes.c_void_p), ("rows", ctypes.c_int32),
                ("cols", ctypes.c_int32), ("lr_index", ctypes.c_int32), ("frag_row", ctypes.c_int32)]


class MuonCfg(ctypes.Structure):
    """struct g2048_muon_cfg (parts / workspace: the multi-CU Newton-Schulz of the h 196 / 192 squares)"""
    _fields_ = [("momentum", ctypes.c_float), ("weight_decay", ctypes.c_float), ("ns_a", ctypes.c_float),
                ("ns_b", ctypes.c_float), ("ns_c", ctypes.c_float), ("ns_eps", ctypes.c_float),
                ("ns_steps", ctypes.c_int32), ("nesterov", ctypes.c_int32), ("parts", ctypes.c_int32),
                ("npartials", ctypes.c_int32), ("workspace", ctypes.c_void_p)]


class AdamWGroup(ctypes.Structure):
    """struct g2048_adamw_group"""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_int64), ("lr_index", ctypes.c_int32),
                ("pad_", ctypes.c_int32)]


class MlpPassArgs(ctypes.Structure):
    """struct g2048_mlp_pass_args"""
    vp = ctypes.c_void_p
    _fields_ = [("boards", vp), ("batch", PPOBatch), ("m", ctypes.c_int64), ("hidden", ctypes.c_int32),
                ("decouple_critic", ctypes.c_int32), ("w_stem", vp), ("w_block", vp * 2), ("ln_gamma", vp * 3),
                ("ln_beta", vp * 3), ("head_frag", vp), ("ba", vp), ("bv", vp), ("drop", Dropout * 2),
                ("beta_dev", vp), ("critic", ctypes.c_float), ("clip_eps", ctypes.c_float), ("x0", vp), ("g", vp * 3),
                ("h", vp * 3), ("mean", vp * 3), ("rstd", vp * 3), ("masked", vp), ("dz", vp), ("dz_bf16", vp),
                ("partials", vp), ("keep", vp), ("idx_offset", vp)]


class MlpBackArgs(ctypes.Structure):
    """struct g2048_mlp_back_args"""
    vp = ctypes.c_void_p
    _fields_ = [("m", ctypes.c_int64), ("hidden", ctypes.c_int32), ("pad_", ctypes.c_int32), ("w_block", vp * 2),
                ("ln_gamma", vp * 3), ("ln_beta", vp * 3), ("wa", vp), ("wv", vp), ("dz", vp), ("g", vp * 3),
                ("mean", vp * 3), ("rstd", vp * 3), ("drop", Dropout * 2), ("dg", vp * 3), ("p_out", vp * 2), ("partials", vp),
                ("keep", vp)]


class MlpWgradArgs(ctypes.Structure):
    """struct g2048_mlp_wgrad_args"""
    vp = ctypes.c_void_p
    _fields_ = [("m", ctypes.c_int64), ("hidden", ctypes.c_int32), ("pad_", ctypes.c_int32), ("dz_bf16", vp),
                ("h2", vp), ("dg", vp * 3), ("x", vp * 3), ("partials", vp)]


class PPOStatsArgs(ctypes.Structure):
    """struct g2048_ppo_stats_args"""
    vp = ctypes.c_void_p
    _fields_ = [("sums", vp), ("grad_norm", vp), ("beta_dev", vp), ("rows", vp), ("stats", vp), ("counter", vp),
                ("sync", vp), ("critic", ctypes.c_float), ("pad_", ctypes.c_int32), ("m", ctypes.c_int64),
                ("idx_offset", vp), ("idx_step", ctypes.c_int64)]


class PolicyRolloutArgs(ctypes.Structure):
    """struct g2048_policy_rollout_args"""
    vp = ctypes.c_void_p
    _fields_ = [("boards", vp), ("flags", vp), ("actions", vp), ("logp", vp), ("entropy", vp), ("value", vp),
                ("points", vp), ("max_tile", vp), ("pot", vp), ("n", ctypes.c_int64), ("t0", ctypes.c_int64),
                ("t1", ctypes.c_int64), ("hidden", ctypes.c_int32), ("num_layers", ctypes.c_int32),
                ("opts", ctypes.c_uint32), ("env_base", ctypes.c_uint32), ("w_stem", vp), ("w_block", vp * 2),
                ("ln_gamma", vp * 3), ("ln_beta", vp * 3), ("head_bf16", vp), ("head_bias_action", vp),
                ("head_bias_value", vp), ("seed", ctypes.c_uint64), ("counter", ctypes.c_uint64),
                ("counter_dev", vp), ("debug", vp)]


_lib = None


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load libg2048.so (no GPU needed to load; every compute call needs one)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise G2048Error(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                         f"or `make -C 2048-ppo_amd/csrc`")
    L = ctypes.CDLL(str(p))
    vp, i64, i32, u32, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_size_t
    u64 = ctypes.c_uint64
    rp, cp = ctypes.POINTER(Rng), ctypes.POINTER(RewardCfg)
    dp, bp = ctypes.POINTER(Dropout), ctypes.POINTER(PPOBatch)
    jp = ctypes.POINTER(ColsumJob)
    sig = {
        "g2048_mt_state_words": (sz, []),
        "g2048_mt_seed": (ctypes.c_int, [vp, vp, vp, i64]),
        "g2048_env_reset": (ctypes.c_int, [vp, vp, vp, vp, i64, rp]),
        "g2048_env_step": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, rp, u32]),
        "g2048_env_rollout_random": (ctypes.c_int, [vp, vp, i64, i64, vp, vp, vp, vp, vp, rp]),
        "g2048_env_rollout_random_adv": (ctypes.c_int, [vp, vp, i64, i64, vp, vp, vp, vp, vp, rp, vp]),
        "g2048_preview_points": (ctypes.c_int, [vp, vp, vp, i64]),
        "g2048_legal_mask": (ctypes.c_int, [vp, vp, vp, i64]),
        "g2048_obs_encode": (ctypes.c_int, [vp, vp, vp, i32, i64]),
        "g2048_info_deltas": (ctypes.c_int, [vp, vp, vp, vp, vp, i64]),
        "g2048_sample_actions": (ctypes.c_int, [vp, vp, i64, vp, vp, vp, vp, i64, rp]),
        "g2048_rtg_prepare": (ctypes.c_int, [vp, vp, cp]),
        "g2048_reward_rtg_workspace_bytes": (sz, [i64]),
        "g2048_reward_rtg": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64, cp, vp, vp, vp, vp, vp, vp, sz]),
        "g2048_reward_rtg_ex": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64, cp, vp, vp, vp, vp, vp, vp, vp, sz]),
        "g2048_rtg_finalize": (ctypes.c_int, [vp, vp, vp, cp]),
        "g2048_build_info": (ctypes.c_char_p, []),
        "g2048_episode_scan": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i64, vp, vp, vp, vp]),
        "g2048_rollout_stats_workspace_bytes": (sz, [i64, i64]),
        "g2048_permutation": (ctypes.c_int, [vp, vp, i64, vp, u64, u64]),
        "g2048_rollout_stats": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i32, cp, vp, vp, vp,
                                               sz, vp]),
        "g2048_augment_workspace_bytes": (ctypes.c_size_t, [i64]),
        "g2048_augment": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, i64, u64, u64, vp, ctypes.c_size_t, vp]),
        "g2048_obs_gather": (ctypes.c_int, [vp, vp, vp, i64, vp]),
        "g2048_ln_act_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, dp]),
        "g2048_ln_act_bwd_partials": (sz, [i64, i32]),
        "g2048_ln_act_bwd": (ctypes.c_int, [vp, ctypes.POINTER(Dy), vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32,
                                            dp, jp]),
        "g2048_colsum_batch": (ctypes.c_int, [vp, jp, i32]),
        "g2048_colsum_batch_blocks": (ctypes.c_int, [jp, i32]),
        "g2048_colsum_batch_sq": (ctypes.c_int, [vp, jp, i32, vp, i32, vp]),
        "g2048_ppo_head_partials": (sz, [i64, i32]),
        "g2048_ppo_head_loss": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32, bp, vp, ctypes.c_float,
                                               ctypes.c_float, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, jp]),
        "g2048_ppo_head_kl": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, vp, vp, vp, vp, jp]),
        "g2048_dropout_mask": (ctypes.c_int, [vp, i64, i32, dp, vp]),
        "g2048_wgrad_partials": (sz, [i64, i32, i32]),
        "g2048_wgrad": (ctypes.c_int, [vp, vp, vp, i64, i32, i32, vp, vp, jp]),
        "g2048_wgrad_pair_partials": (sz, [i64, i32, i32]),
        "g2048_wgrad_pair": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32, i32, vp, vp, vp, vp, jp]),
        "g2048_grad_clip": (ctypes.c_int, [vp, vp, i64, ctypes.c_float, vp, vp, vp]),
        "g2048_mlp_fwd_lds_bytes": (sz, [i32, i32]),
        "g2048_mlp_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, i64, i32, i32, dp]),
        "g2048_head_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32, vp, i64, vp]),
        "g2048_ppo_stats": (ctypes.c_int, [vp, vp, vp, i32, vp, vp, ctypes.c_float, i64, vp, vp, vp]),
        "g2048_policy_rollout_supported": (ctypes.c_int, [i32, i32]),
        "g2048_policy_rollout_lds_bytes": (sz, [i32]),
        "g2048_policy_rollout": (ctypes.c_int, [vp, ctypes.POINTER(PolicyRolloutArgs)]),
        "g2048_head_split_bytes": (sz, [i32]),
        "g2048_head_split": (ctypes.c_int, [vp, vp, vp, i32, vp]),
        "g2048_mlp_pass_supported": (ctypes.c_int, [i32, i32]),
        "g2048_mlp_pass_partials": (sz, [i64, i32]),
        "g2048_ppo_forward_loss": (ctypes.c_int, [vp, ctypes.POINTER(MlpPassArgs), vp, vp, vp, jp]),
        "g2048_mlp_back_partials": (sz, [i64, i32]),
        "g2048_ppo_backward": (ctypes.c_int, [vp, ctypes.POINTER(MlpBackArgs), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                              jp]),
        "g2048_ppo_forward_kl": (ctypes.c_int, [vp, ctypes.POINTER(MlpPassArgs), vp, jp]),
        "g2048_ppo_forward_kl_stats": (ctypes.c_int, [vp, ctypes.POINTER(MlpPassArgs), ctypes.POINTER(PPOStatsArgs)]),
        "g2048_mlp_wgrad_partials": (sz, [i64, i32]),
        "g2048_mlp_wgrad": (ctypes.c_int, [vp, ctypes.POINTER(MlpWgradArgs), vp, ctypes.POINTER(vp), jp]),
        "g2048_linear_dgrad_supported": (ctypes.c_int, [i32, i32]),
        "g2048_linear_dgrad": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_stem": (ctypes.c_int, [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, i64, i32]),
        "g2048_urm_attention": (ctypes.c_int, [vp, vp, vp, i64, i32, i32]),
        "g2048_urm_residual_rms": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32, ctypes.c_float]),
        "g2048_urm_swiglu_conv": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32]),
        "g2048_urm_pool_heads": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, i64, i32]),
        "g2048_urm_linear_supported": (ctypes.c_int, [i32, i32, i32, i32]),
        "g2048_urm_forward_supported": (ctypes.c_int, [i32, i32, i32, i32, i32]),
        "g2048_urm_forward": (ctypes.c_int, [vp, ctypes.POINTER(UrmWeights), vp, i32, vp, vp, i64]),
        "g2048_urm_forward_drop": (ctypes.c_int, [vp, ctypes.POINTER(UrmWeights), vp, i32, vp, vp, i64, ctypes.c_float,
                                                  ctypes.c_uint64, vp]),
        "g2048_urm_linear": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_linear_rms": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32, i32, ctypes.c_float]),
        "g2048_urm_linear_bias": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_linear_res_rms": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, ctypes.c_float]),
        "g2048_urm_linear_swiglu": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_linear_swiglu_train": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_linear_t": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_gate_up_swiglu_bwd_supported": (ctypes.c_int, [i32, i32]),
        "g2048_urm_gate_up_swiglu_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_gate_up_swiglu_bwd_acc": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32, i32, i32]),
        "g2048_urm_wgrad_supported": (ctypes.c_int, [i32, i32]),
        "g2048_urm_wgrad_partials": (sz, [i64, i32, i32]),
        "g2048_urm_wgrad": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_wgrad_acc": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32, i32, i32]),
        "g2048_urm_linres_bwd_supported": (ctypes.c_int, [i32, i32]),
        "g2048_urm_linres_bwd_partials": (sz, [i64, i32]),
        "g2048_urm_linres_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, i32, i32]),
        "g2048_urm_head_loss_partials": (sz, [i64, i32]),
        "g2048_urm_head_loss": (ctypes.c_int, [vp, vp, i32, vp, vp, vp, vp, i64, i32, bp, vp, ctypes.c_float,
                                               ctypes.c_float, vp, vp, vp, vp, vp, vp]),
        "g2048_urm_head_loss_bwd": (ctypes.c_int, [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, i64,
                                                   i32]),
        "g2048_urm_kl_stats": (ctypes.c_int, [vp, vp, vp, i64, vp, vp, vp, ctypes.c_float, vp, vp, vp]),
        "g2048_muon_supported": (ctypes.c_int, [i32, i32]),
        "g2048_muon_step": (ctypes.c_int, [vp, ctypes.POINTER(MuonMatrix), i32, vp, vp, ctypes.POINTER(MuonCfg)]),
        "g2048_grad_sumsq": (ctypes.c_int, [vp, vp, i64, vp]),
        "g2048_muon_workspace_bytes": (sz, []),
        "g2048_muon_error_offset": (sz, []),
        "g2048_lds_poison": (ctypes.c_int, [vp, u32]),
        "g2048_muon_step_clip": (ctypes.c_int, [vp, ctypes.POINTER(MuonMatrix), i32, vp, vp, ctypes.c_float, vp, vp,
                                                ctypes.POINTER(MuonCfg)]),
        "g2048_adamw_step": (ctypes.c_int, [vp, ctypes.POINTER(AdamWGroup), i32, vp, vp, vp, ctypes.c_float,
                                            ctypes.c_float, ctypes.c_float, ctypes.c_float]),
        "g2048_grad_sumsq_tick": (ctypes.c_int, [vp, vp, i64, vp, vp]),
        "g2048_urm_attention_bwd": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32]),
        "g2048_urm_rms_res_fwd2": (ctypes.c_int, [vp, vp, vp, i32, vp, vp, vp, i64, i32, ctypes.c_float]),
        "g2048_urm_add_cast": (ctypes.c_int, [vp, vp, i64, vp, vp, vp, i64, i32]),
        "g2048_urm_add_cast_bwd": (ctypes.c_int, [vp, vp, vp, vp, i64, i32]),
        "g2048_urm_add_cast_bwd_acc": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64, i32]),
        "g2048_urm_rms_res_bwd3": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i64, i32]),
        "g2048_urm_rms_res_bwd2": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, i32, i64, i32]),
        "g2048_urm_stem_partials": (sz, [i64]),
        "g2048_urm_stem_fwd": (ctypes.c_int, [vp, vp, i32, vp, vp, vp, vp, i64, i32, ctypes.c_float]),
        "g2048_urm_stem_bwd": (ctypes.c_int, [vp, vp, i32, vp, vp, vp, vp, vp, vp, i64, i32, ctypes.c_float]),
        "g2048_urm_stem_bwd3": (ctypes.c_int, [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, i32, vp, i64, i32,
                                               ctypes.c_float]),
        "g2048_urm_attention_drop": (ctypes.c_int, [vp, vp, vp, i64, i32, i32, ctypes.c_float, ctypes.c_uint64, vp]),
        "g2048_urm_attention_bwd_drop": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32, ctypes.c_float, ctypes.c_uint64,
                                                        vp]),
        "g2048_urm_attention_drop_at": (ctypes.c_int, [vp, vp, vp, i64, i32, i32, ctypes.c_float, ctypes.c_uint64, vp,
                                                       ctypes.c_uint64]),
        "g2048_urm_attention_bwd_drop_at": (ctypes.c_int, [vp, vp, vp, vp, i64, i32, i32, ctypes.c_float,
                                                           ctypes.c_uint64, vp, ctypes.c_uint64]),
        "g2048_urm_rms_res_fwd": (ctypes.c_int, [vp, vp, vp, i32, vp, vp, i64, i32, ctypes.c_float]),
        "g2048_urm_rms_res_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i32, i64, i32]),
        "g2048_urm_swiglu_conv_partials": (sz, [i64, i32]),
        "g2048_urm_swiglu_conv_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32]),
        "g2048_urm_swiglu_conv_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i32]),
        "g2048_mlp_fwd_kl": (ctypes.c_int, [vp, vp, vp, vp, vp, i64, i32, i32, dp, vp, vp, vp, vp, vp, vp, jp]),
        "g2048_muon_adamw_step_clip": (ctypes.c_int, [vp, ctypes.POINTER(MuonMatrix), i32, ctypes.POINTER(AdamWGroup),
                                                      i32, vp, vp, vp, ctypes.c_float, vp, vp,
                                                      ctypes.POINTER(MuonCfg), ctypes.c_float, ctypes.c_float,
                                                      ctypes.c_float, ctypes.c_float]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if path is None:
                raise
            continue  # an older build loaded for an A/B timing: entry points it lacks stay unbound
        fn.restype, fn.argtypes = res, args
    if path is None:
        _lib = L
    return L


def _check(status: int, what: str):
    if status != 0:
        raise G2048Error(f"{what} failed with status {status}")


def _stream(t: torch.Tensor):
    if not t.is_cuda:
        raise G2048Error(f"tensor on {t.device}: libg2048 kernels need a ROCm device tensor (no CPU path)")
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _dev(t: torch.Tensor | None, dtype=None, name="tensor"):
    if t is None:
        return None
    if not t.is_cuda:
        raise G2048Error(f"{name} must be a ROCm device tensor (got {t.device}); there is no CPU path")
    if dtype is not None and t.dtype != dtype:
        raise G2048Error(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise G2048Error(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def make_rng(mode=RNG_PHILOX, seed=0, counter=0, env_base=0, counter_dev=None, mt_state=None, inject=None) -> Rng:
    return Rng(mode, env_base, seed & (2**64 - 1), counter, _dev(counter_dev, torch.int64, "counter_dev"),
               _dev(mt_state, torch.int32, "mt_state"), _dev(inject, torch.int32, "inject"))


# ------------------------------------------------------------------------------- wrappers ------
def mt_seed(mt_state: torch.Tensor, seeds: torch.Tensor):
    n = seeds.numel()
    _check(load().g2048_mt_seed(_stream(seeds), _dev(mt_state, torch.int32, "mt_state"),
                                _dev(seeds, torch.int64, "seeds"), n), "g2048_mt_seed")


def env_reset(boards: torch.Tensor, flags: torch.Tensor | None, rng: Rng, where: torch.Tensor | None = None):
    _check(load().g2048_env_reset(_stream(boards), _dev(boards, torch.int8, "boards"), _dev(flags, torch.uint8, "flags"),
                                  _dev(where, torch.uint8, "where"), boards.shape[0], ctypes.byref(rng)),
           "g2048_env_reset")


def env_step(boards_in, boards_out, actions_in, actions_out, points, max_tile, pot, flags, rng: Rng, options=0):
    n = boards_in.shape[0]
    _check(load().g2048_env_step(
        _stream(boards_in), _dev(boards_in, torch.int8, "boards_in"), _dev(boards_out, torch.int8, "boards_out"),
        _dev(actions_in, torch.uint8, "actions_in"), _dev(actions_out, torch.uint8, "actions_out"),
        _dev(points, torch.int32, "points"), _dev(max_tile, torch.int8, "max_tile"), _dev(pot, torch.int8, "pot"),
        _dev(flags, torch.uint8, "flags"), n, ctypes.byref(rng), options), "g2048_env_step")


def env_rollout_random(boards, steps, traj_boards, traj_actions, traj_points, traj_pot, traj_flags, rng: Rng,
                       ticket=None):
    """ticket (a zero-filled int32 device word): the launch also advances rng's device counter by `steps`
    (g2048_env_rollout_random_adv: no counter-bump kernel between consecutive launches)."""
    args = (_stream(boards), _dev(boards, torch.int8, "boards"), boards.shape[0], steps,
            _dev(traj_boards, torch.int8, "traj_boards"), _dev(traj_actions, torch.uint8, "traj_actions"),
            _dev(traj_points, torch.int32, "traj_points"), _dev(traj_pot, torch.int8, "traj_pot"),
            _dev(traj_flags, torch.uint8, "traj_flags"), ctypes.byref(rng))
    if ticket is None:
        _check(load().g2048_env_rollout_random(*args), "g2048_env_rollout_random")
    else:
        _check(load().g2048_env_rollout_random_adv(*args, _dev(ticket, torch.int32, "ticket")),
               "g2048_env_rollout_random_adv")


def preview_points(boards, points4):
    _check(load().g2048_preview_points(_stream(boards), _dev(boards, torch.int8, "boards"),
                                       _dev(points4, torch.int32, "points4"), boards.shape[0]), "g2048_preview_points")


def legal_mask(boards, flags):
    _check(load().g2048_legal_mask(_stream(boards), _dev(boards, torch.int8, "boards"), _dev(flags, torch.uint8, "flags"),
                                   boards.shape[0]), "g2048_legal_mask")


def obs_encode(boards, obs):
    dt = {torch.float32: DTYPE_F32, torch.bfloat16: DTYPE_BF16}.get(obs.dtype)
    if dt is None:
        raise G2048Error(f"obs dtype {obs.dtype} unsupported")
    _check(load().g2048_obs_encode(_stream(boards), _dev(boards, torch.int8, "boards"), _dev(obs, None, "obs"), dt,
                                   boards.shape[0]), "g2048_obs_encode")


def info_deltas(boards, actions, deltas, anchor=None):
    """boards int8 [n, 16], actions uint8 [n] -> deltas float64 [n, 5] (smoothness, corner, adjacency,
    chain, topological after - before the move), anchor int8 [n] (optional)."""
    n = boards.shape[0]
    _check(load().g2048_info_deltas(_stream(boards), _dev(boards, torch.int8, "boards"),
                                    _dev(actions, torch.uint8, "actions"), _dev(deltas, torch.float64, "deltas"),
                                    _dev(anchor, torch.int8, "anchor"), n), "g2048_info_deltas")


def sample_actions(logits, flags, actions, logp, entropy, rng: Rng):
    n = flags.shape[0]
    stride = 0
    lp = None
    if logits is not None:
        if logits.dtype != torch.float32 or not logits.is_cuda or logits.stride(-1) != 1:
            raise G2048Error("logits must be float32 on device with unit inner stride")
        stride = logits.stride(0)
        lp = ctypes.c_void_p(logits.data_ptr())
    _check(load().g2048_sample_actions(_stream(flags), lp, stride, _dev(flags, torch.uint8, "flags"),
                                       _dev(actions, torch.uint8, "actions"), _dev(logp, torch.float32, "logp"),
                                       _dev(entropy, torch.float32, "entropy"), n, ctypes.byref(rng)),
           "g2048_sample_actions")


def rtg_workspace_bytes(n: int) -> int:
    return int(load().g2048_reward_rtg_workspace_bytes(n))


def rtg_prepare(state, cfg: RewardCfg):
    _check(load().g2048_rtg_prepare(_stream(state), _dev(state, torch.float64, "state"), ctypes.byref(cfg)),
           "g2048_rtg_prepare")


def reward_rtg(points, pot, flags, value, state, g_raw, g_norm, adv, partials, workspace, cfg: RewardCfg,
               reward=None):
    """reward (optional) float64 [T, n]: the per-step reward the scan used."""
    T, n = points.shape[0], points.shape[1]
    _check(load().g2048_reward_rtg_ex(
        _stream(points), _dev(points, torch.int32, "points"), _dev(pot, torch.int8, "pot"),
        _dev(flags, torch.uint8, "flags"), _dev(value, torch.float32, "value"), T, n, ctypes.byref(cfg),
        _dev(state, torch.float64, "state"), _dev(g_raw, torch.float32, "g_raw"),
        _dev(g_norm, torch.float32, "g_norm"), _dev(adv, torch.float32, "adv"),
        _dev(reward, torch.float64, "reward") if reward is not None else None,
        _dev(partials, torch.float64, "partials"), _dev(workspace, torch.uint8, "workspace"), workspace.numel()),
        "g2048_reward_rtg_ex")


def episode_scan(points, boards, max_tile, step_flags, run_score, run_max, scores, tiles):
    """points/max_tile/step_flags [T, n], boards [T, n, 16]; run_score int64 / run_max int32 [n] carried."""
    T, n = points.shape[0], points.shape[1]
    _check(load().g2048_episode_scan(
        _stream(points), _dev(points, torch.int32, "points"), _dev(boards, torch.int8, "boards"),
        _dev(max_tile, torch.int8, "max_tile"), _dev(step_flags, torch.uint8, "step_flags"), T, n,
        _dev(run_score, torch.int64, "run_score"), _dev(run_max, torch.int32, "run_max"),
        _dev(scores, torch.int64, "scores"), _dev(tiles, torch.int32, "tiles")), "g2048_episode_scan")


def permutation(out, n: int, key=None, seed: int = 0, counter: int = 0):
    """out[:n] (int64, device) = a keyed random permutation of [0, n) (g2048_permutation); key: a
    device int64 [1] (e.g. drawn from the caller's generator: no host read) or None for (seed, counter)."""
    if out.numel() < n:
        raise G2048Error("permutation: out too small")
    _check(load().g2048_permutation(_stream(out), _dev(out, torch.int64, "out"), int(n),
                                    _dev(key, torch.int64, "key"), int(seed) & (2 ** 64 - 1),
                                    int(counter) & (2 ** 64 - 1)), "g2048_permutation")


ROLLOUT_STATS = 23  # g2048_rollout_stats' output vector


def rollout_stats_workspace_bytes(T: int, n: int) -> int:
    return int(load().g2048_rollout_stats_workspace_bytes(int(T), int(n)))


def rollout_stats(points, pot, step_flags, value, g_raw, g_norm, adv, boards, max_tile, episodic, cfg,
                  run_score, run_max, workspace, out):
    """The rollout metrics vector out [23] float32 (include/g2048.h g2048_rollout_stats).  points /
    step_flags / value / g_raw / g_norm / adv [T, n], pot [T, n, 4]; fixed horizon: boards [T, n, 16],
    max_tile [T, n], run_score / run_max [n] carried; episodic: boards [T + 1, n, 16] (the final board
    read), max_tile / run_* may be None.  cfg: RewardCfg.  workspace: a zero-filled uint8 tensor of
    rollout_stats_workspace_bytes(T, n) bytes, left zeroed."""
    T, n = points.shape[0], points.shape[1]
    _check(load().g2048_rollout_stats(
        _stream(points), _dev(points, torch.int32, "points"), _dev(pot, torch.int8, "pot"),
        _dev(step_flags, torch.uint8, "step_flags"), _dev(value, torch.float32, "value"),
        _dev(g_raw, torch.float32, "g_raw"), _dev(g_norm, torch.float32, "g_norm"), _dev(adv, torch.float32, "adv"),
        _dev(boards, torch.int8, "boards"), _dev(max_tile, torch.int8, "max_tile"), T, n, 1 if episodic else 0,
        ctypes.byref(cfg), _dev(run_score, torch.int64, "run_score"), _dev(run_max, torch.int32, "run_max"),
        _dev(workspace, torch.uint8, "workspace"), workspace.numel(), _dev(out, torch.float32, "out")),
        "g2048_rollout_stats")


def augment_workspace_bytes(k: int) -> int:
    return int(load().g2048_augment_workspace_bytes(int(k)))


def augment(boards, actions, legal, logp, adv, ret, n: int, k: int, seed: int, counter: int, workspace, count):
    """D4 up-sampling (train.py:774-881): appends the copies of k sampled rows of the pool after its
    n real rows; count (int64 [1], device) = n + copies.  Pool capacity >= n + 2k."""
    cap = boards.shape[0]
    for t, nm in ((actions, "actions"), (legal, "legal"), (logp, "logp"), (adv, "adv"), (ret, "ret")):
        if t.shape[0] != cap:
            raise G2048Error(f"augment: {nm} has {t.shape[0]} rows, boards {cap}")
    if k > 0 and cap < n + 2 * k:
        raise G2048Error(f"augment: pool capacity {cap} < n + 2k = {n + 2 * k}")
    _check(load().g2048_augment(
        _stream(boards), _dev(boards, torch.int8, "boards"), _dev(actions, torch.uint8, "actions"),
        _dev(legal, torch.uint8, "legal"), _dev(logp, torch.float32, "logp"), _dev(adv, torch.float32, "adv"),
        _dev(ret, torch.float32, "ret"), int(n), int(k), int(seed) & (2**64 - 1), int(counter) & (2**64 - 1),
        _dev(workspace, None, "workspace"), workspace.numel() * workspace.element_size(),
        _dev(count, torch.int64, "count")), "g2048_augment")


def rtg_finalize(state, partials, cfg: RewardCfg):
    _check(load().g2048_rtg_finalize(_stream(state), _dev(state, torch.float64, "state"),
                                     _dev(partials, torch.float64, "partials"), ctypes.byref(cfg)),
           "g2048_rtg_finalize")


# ------------------------------------------------------------- PPO update (g2048_ppo.h) -------
def make_dropout(p=0.0, layer=0, pass_=0, seed=0, counter=0, counter_dev=None) -> Dropout:
    return Dropout(float(p), layer, pass_, 0, seed & (2**64 - 1), counter,
                   _dev(counter_dev, torch.int64, "counter_dev"))


def obs_gather(boards, idx, obs):
    _check(load().g2048_obs_gather(_stream(idx), _dev(boards, torch.int8, "boards"), _dev(idx, torch.int64, "idx"),
                                   idx.shape[0], _dev(obs, torch.bfloat16, "obs")), "g2048_obs_gather")


def ln_act_fwd(g, gamma, beta, res, y, mean, rstd, drop: Dropout | None = None):
    m, h = g.shape
    _check(load().g2048_ln_act_fwd(
        _stream(g), _dev(g, torch.bfloat16, "g"), _dev(gamma, torch.float32, "gamma"),
        _dev(beta, torch.float32, "beta"), _dev(res, torch.bfloat16, "res"), _dev(y, torch.bfloat16, "y"),
        _dev(mean, torch.float32, "mean"), _dev(rstd, torch.float32, "rstd"), m, h,
        ctypes.byref(drop) if drop is not None else None), "g2048_ln_act_fwd")


def ln_act_bwd_partials(m: int, h: int) -> int:
    return int(load().g2048_ln_act_bwd_partials(m, h))


def make_dy(dres=None, ps=(), head=None) -> Dy:
    """dy = dres + sum(ps) + heads; head = (dz, wa, wv) with wv None for a decoupled critic."""
    ps = [p for p in ps if p is not None]
    if len(ps) > DY_MAX_P:
        raise G2048Error(f"at most {DY_MAX_P} matmul gradients per LayerNorm backward")
    d = Dy()
    d.dres = _dev(dres, torch.float32, "dres")
    for i, p in enumerate(ps):
        d.p[i] = _dev(p, torch.bfloat16, f"p[{i}]")
    if head is not None:
        dz, wa, wv = head
        d.dz, d.wa, d.wv = _dev(dz, torch.float32, "dz"), _dev(wa, torch.float32, "wa"), _dev(wv, torch.float32, "wv")
    return d


def _defer(job):
    return ctypes.byref(job) if job is not None else None


def ln_act_bwd(dres_in, p_in, g, mean, rstd, gamma, beta, dg, dres_out, partials, dgamma, dbeta,
               drop: Dropout | None = None, head=None, dy: Dy | None = None, defer: ColsumJob | None = None):
    """LayerNorm/ReLU/dropout backward; the output gradient is `dy` (a Dy) or dres_in + p_in (+ head)."""
    m, h = g.shape
    if dy is None:
        dy = make_dy(dres_in, [p_in], head)
    _check(load().g2048_ln_act_bwd(
        _stream(g), ctypes.byref(dy), _dev(g, torch.bfloat16, "g"), _dev(mean, torch.float32, "mean"),
        _dev(rstd, torch.float32, "rstd"), _dev(gamma, torch.float32, "gamma"), _dev(beta, torch.float32, "beta"),
        _dev(dg, torch.bfloat16, "dg"), _dev(dres_out, torch.float32, "dres_out"),
        _dev(partials, torch.float32, "partials"), _dev(dgamma, torch.float32, "dgamma"),
        _dev(dbeta, torch.float32, "dbeta"), m, h, ctypes.byref(drop) if drop is not None else None, _defer(defer)),
        "g2048_ln_act_bwd")


def ppo_head_partials(m: int, h: int) -> int:
    return int(load().g2048_ppo_head_partials(m, h))


def make_ppo_batch(idx, action, legal, old_logp, adv, ret, rows=None) -> PPOBatch:
    """rows (optional int64 device scalar): valid rows of a padded ragged minibatch."""
    return PPOBatch(_dev(idx, torch.int64, "idx"), _dev(action, torch.uint8, "action"),
                    _dev(legal, torch.uint8, "legal"), _dev(old_logp, torch.float32, "old_logp"),
                    _dev(adv, torch.float32, "adv"), _dev(ret, torch.float32, "ret"), _dev(rows, torch.int64, "rows"))


def ppo_head_loss(x, wa, ba, wv, bv, batch: PPOBatch, beta_dev, critic, clip_eps, decouple, masked, dx, partials,
                  dwa, dba, dwv, dbv, sums, dz=None, defer: ColsumJob | None = None):
    m, h = x.shape
    _check(load().g2048_ppo_head_loss(
        _stream(x), _dev(x, torch.bfloat16, "x"), _dev(wa, torch.float32, "wa"), _dev(ba, torch.float32, "ba"),
        _dev(wv, torch.float32, "wv"), _dev(bv, torch.float32, "bv"), m, h, ctypes.byref(batch),
        _dev(beta_dev, torch.float32, "beta"), float(critic), float(clip_eps), int(bool(decouple)),
        _dev(masked, torch.float32, "masked"), _dev(dx, torch.float32, "dx"), _dev(dz, torch.float32, "dz"),
        _dev(partials, torch.float32, "partials"), _dev(dwa, torch.float32, "dwa"), _dev(dba, torch.float32, "dba"),
        _dev(dwv, torch.float32, "dwv"), _dev(dbv, torch.float32, "dbv"), _dev(sums, torch.float32, "sums"),
        _defer(defer)), "g2048_ppo_head_loss")


def mlp_fwd_kl_supported(n: int, k: int) -> bool:
    return n == 196 and k == 196


def mlp_fwd_kl(x, w, gamma, beta, drop, wa, ba, old_masked, partials, out, defer: ColsumJob | None = None, rows=None):
    """The KL re-forward's last ResidualBlock fused with the action head and the KL reduction."""
    m, k = x.shape
    _check(load().g2048_mlp_fwd_kl(
        _stream(x), _dev(x, torch.bfloat16, "x"), _dev(w, torch.bfloat16, "w"), _dev(gamma, torch.float32, "gamma"),
        _dev(beta, torch.float32, "beta"), m, w.shape[0], k, ctypes.byref(drop) if drop is not None else None,
        _dev(wa, torch.float32, "wa"), _dev(ba, torch.float32, "ba"), _dev(old_masked, torch.float32, "old_masked"),
        _dev(rows, torch.int64, "rows"), _dev(partials, torch.float32, "partials"), _dev(out, torch.float32, "out"),
        _defer(defer)), "g2048_mlp_fwd_kl")


def ppo_head_kl(x, wa, ba, old_masked, partials, out, defer: ColsumJob | None = None, rows=None):
    m, h = x.shape
    _check(load().g2048_ppo_head_kl(
        _stream(x), _dev(x, torch.bfloat16, "x"), _dev(wa, torch.float32, "wa"), _dev(ba, torch.float32, "ba"), m, h,
        _dev(old_masked, torch.float32, "old_masked"), _dev(rows, torch.int64, "rows"),
        _dev(partials, torch.float32, "partials"),
        _dev(out, torch.float32, "out"), _defer(defer)), "g2048_ppo_head_kl")


def mlp_pass_supported(hidden: int, num_layers: int) -> bool:
    """The fused train / KL passes (g2048_ppo_forward_loss / _kl) cover this GameMLP shape."""
    return bool(load().g2048_mlp_pass_supported(int(hidden), int(num_layers)))


def mlp_pass_partials(m: int, train: bool) -> int:
    return int(load().g2048_mlp_pass_partials(int(m), int(bool(train))))


def head_split_bytes(hidden: int) -> int:
    return int(load().g2048_head_split_bytes(int(hidden)))


def head_split(wa, wv, frag):
    """frag (uint8 device buffer of head_split_bytes(h)) <- the 3-term bf16 split of [wa; wv]."""
    h = wa.shape[1]
    _check(load().g2048_head_split(_stream(wa), _dev(wa, torch.float32, "wa"), _dev(wv, torch.float32, "wv"), h,
                                   _dev(frag, None, "frag")), "g2048_head_split")


def make_mlp_pass(boards, batch: PPOBatch, m: int, w_stem, w_blocks, gammas, betas, head_frag, ba, bv=None,
                  drops=(None, None), beta_dev=None, critic=0.0, clip_eps=0.2, decouple=False, x0=None,
                  g=(None, None, None), h=(None, None, None), mean=(None, None, None), rstd=(None, None, None),
                  masked=None, dz=None, dz_bf16=None, partials=None, keep=None, idx_offset=None) -> MlpPassArgs:
    """struct g2048_mlp_pass_args for g2048_ppo_forward_loss / g2048_ppo_forward_kl (GameMLP, 2 blocks).
    keep (train pass, optional): int64 [2, m, 4] out, the blocks' dropout keep bits for the backward."""
    a = MlpPassArgs()
    a.boards = _dev(boards, torch.int8, "boards")
    a.batch = batch
    a.m = int(m)
    a.hidden = int(w_stem.shape[0])
    a.decouple_critic = int(bool(decouple))
    a.w_stem = _dev(w_stem, torch.bfloat16, "w_stem")
    for i, w in enumerate(w_blocks):
        a.w_block[i] = _dev(w, torch.bfloat16, f"w_block[{i}]")
    for i, (gm, bt) in enumerate(zip(gammas, betas)):
        a.ln_gamma[i], a.ln_beta[i] = _dev(gm, torch.float32, "gamma"), _dev(bt, torch.float32, "beta")
    a.head_frag = _dev(head_frag, None, "head_frag")
    a.ba, a.bv = _dev(ba, torch.float32, "ba"), _dev(bv, torch.float32, "bv")
    for i, d in enumerate(drops):
        if d is not None:
            a.drop[i] = d
    a.beta_dev = _dev(beta_dev, torch.float32, "beta_dev")
    a.critic, a.clip_eps = float(critic), float(clip_eps)
    a.x0 = _dev(x0, torch.bfloat16, "x0")
    for i in range(3):
        a.g[i] = _dev(g[i], torch.bfloat16, f"g[{i}]")
        a.h[i] = _dev(h[i], torch.bfloat16, f"h[{i}]")
        a.mean[i] = _dev(mean[i], torch.float32, f"mean[{i}]")
        a.rstd[i] = _dev(rstd[i], torch.float32, f"rstd[{i}]")
    a.masked = _dev(masked, torch.float32, "masked")
    a.dz = _dev(dz, torch.float32, "dz")
    a.dz_bf16 = _dev(dz_bf16, torch.bfloat16, "dz_bf16")
    a.partials = _dev(partials, torch.float32, "partials")
    a.keep = _dev(keep, torch.int64, "keep")
    a.idx_offset = _dev(idx_offset, torch.int64, "idx_offset")
    return a


def ppo_forward_loss(args: MlpPassArgs, dba, dbv, sums, defer: ColsumJob | None = None, like=None):
    """The fused train pass (obs -> GameMLP -> heads -> PPO loss / dz) of one minibatch."""
    _check(load().g2048_ppo_forward_loss(_stream(like if like is not None else dba), ctypes.byref(args),
                                         _dev(dba, torch.float32, "dba"), _dev(dbv, torch.float32, "dbv"),
                                         _dev(sums, torch.float32, "sums"), _defer(defer)), "g2048_ppo_forward_loss")


def ppo_forward_kl(args: MlpPassArgs, out, defer: ColsumJob | None = None):
    """The fused KL re-forward of one minibatch: out[2] = {sum KL, max KL}."""
    _check(load().g2048_ppo_forward_kl(_stream(out), ctypes.byref(args), _dev(out, torch.float32, "out"),
                                       _defer(defer)), "g2048_ppo_forward_kl")


def ppo_forward_kl_stats(args: MlpPassArgs, sums, grad_norm, beta_dev, critic: float, m: int, stats, sync,
                         counter=None, rows=None, idx_offset=None, idx_step: int = 0):
    """The fused KL re-forward whose last block also accumulates the minibatch statistics
    (g2048_ppo_stats folded in); sync: a zeroed int32 device word kept across calls."""
    st = PPOStatsArgs(_dev(sums, torch.float32, "sums"), _dev(grad_norm, torch.float32, "grad_norm"),
                      _dev(beta_dev, torch.float32, "beta_dev"), _dev(rows, torch.int64, "rows"),
                      _dev(stats, torch.float32, "stats"), _dev(counter, torch.int64, "counter"),
                      _dev(sync, torch.int32, "sync"), float(critic), 0, int(m),
                      _dev(idx_offset, torch.int64, "idx_offset"), int(idx_step))
    _check(load().g2048_ppo_forward_kl_stats(_stream(stats), ctypes.byref(args), ctypes.byref(st)),
           "g2048_ppo_forward_kl_stats")


def mlp_back_partials(m: int, h: int) -> int:
    return int(load().g2048_mlp_back_partials(int(m), int(h)))


def make_mlp_back(m: int, w_blocks, gammas, betas, wa, wv, dz, g, mean, rstd, drops=(None, None), dg=(None,) * 3,
                  partials=None, p_out=(None, None), keep=None) -> MlpBackArgs:
    """struct g2048_mlp_back_args for g2048_ppo_backward (GameMLP, 2 blocks).  keep: the train pass's
    keep bits (make_mlp_pass(keep=...)) for the same drops, read instead of re-drawing the masks."""
    a = MlpBackArgs()
    a.m = int(m)
    a.hidden = int(w_blocks[0].shape[0])
    for i, w in enumerate(w_blocks):
        a.w_block[i] = _dev(w, torch.bfloat16, f"w_block[{i}]")
    for i, (gm, bt) in enumerate(zip(gammas, betas)):
        a.ln_gamma[i], a.ln_beta[i] = _dev(gm, torch.float32, "gamma"), _dev(bt, torch.float32, "beta")
    a.wa, a.wv = _dev(wa, torch.float32, "wa"), _dev(wv, torch.float32, "wv")
    a.dz = _dev(dz, torch.float32, "dz")
    for i in range(3):
        a.g[i] = _dev(g[i], torch.bfloat16, f"g[{i}]")
        a.mean[i] = _dev(mean[i], torch.float32, f"mean[{i}]")
        a.rstd[i] = _dev(rstd[i], torch.float32, f"rstd[{i}]")
        a.dg[i] = _dev(dg[i], torch.bfloat16, f"dg[{i}]")
    for i in range(2):
        a.p_out[i] = _dev(p_out[i], torch.bfloat16, f"p_out[{i}]")
    for i, d in enumerate(drops):
        if d is not None:
            a.drop[i] = d
    a.partials = _dev(partials, torch.float32, "partials")
    a.keep = _dev(keep, torch.int64, "keep")
    return a


def mlp_wgrad_partials(m: int, h: int) -> int:
    return int(load().g2048_mlp_wgrad_partials(int(m), int(h)))


def mlp_wgrad(m: int, dz_bf16, h2, dg, x, partials, out_head, out_w, defer=None):
    """The four weight gradients of the GameMLP minibatch in one launch (g2048_mlp_wgrad):
    out_head [16, h] = dz_bf16^T h2, out_w[0] [h, 48] = dg[0]^T x[0], out_w[l] [h, h] = dg[l]^T x[l];
    defer: a list of four ColsumJob (head, stem, block 1, block 2) filled instead of summing."""
    a = MlpWgradArgs()
    a.m = int(m)
    a.hidden = int(h2.shape[1])
    a.dz_bf16 = _dev(dz_bf16, torch.bfloat16, "dz_bf16")
    a.h2 = _dev(h2, torch.bfloat16, "h2")
    for i in range(3):
        a.dg[i] = _dev(dg[i], torch.bfloat16, f"dg[{i}]")
        a.x[i] = _dev(x[i], torch.bfloat16, f"x[{i}]")
    a.partials = _dev(partials, torch.float32, "partials")
    vp = ctypes.c_void_p
    outs = (vp * 3)(*[_dev(t, torch.float32, "out_w") for t in out_w])
    jobs = (ColsumJob * 4)() if defer is not None else None
    _check(load().g2048_mlp_wgrad(_stream(out_head), ctypes.byref(a), _dev(out_head, torch.float32, "out_head"), outs,
                                  jobs), "g2048_mlp_wgrad")
    if defer is not None:
        for i in range(4):
            defer[i] = jobs[i]


def ppo_backward(args: MlpBackArgs, dgamma, dbeta, defer=None, like=None):
    """The fused MLP backward of one minibatch (three dG, the LayerNorm affine gradients); defer: a
    list of three ColsumJob filled instead of summing at once."""
    vp = ctypes.c_void_p
    dgp = (vp * 3)(*[_dev(t, torch.float32, "dgamma") for t in dgamma])
    dbp = (vp * 3)(*[_dev(t, torch.float32, "dbeta") for t in dbeta])
    jobs = None
    if defer is not None:
        jobs = (ColsumJob * 3)()
    _check(load().g2048_ppo_backward(_stream(like if like is not None else dgamma[0]), ctypes.byref(args), dgp, dbp,
                                     jobs), "g2048_ppo_backward")
    if defer is not None:
        for i in range(3):
            defer[i] = jobs[i]


def dropout_mask(m: int, h: int, drop: Dropout, mask):
    _check(load().g2048_dropout_mask(_stream(mask), m, h, ctypes.byref(drop), _dev(mask, torch.uint8, "mask")),
           "g2048_dropout_mask")


def wgrad_partials(m: int, n1: int, n2: int) -> int:
    """Scratch floats of wgrad (0 = shape not supported by the MFMA kernel)."""
    return int(load().g2048_wgrad_partials(m, n1, n2))


def wgrad(a, b, partials, out, defer: ColsumJob | None = None):
    """out[n1, n2] = a^T b for bf16 a [m, n1], b [m, n2]; fp32 out."""
    m, n1 = a.shape
    n2 = b.shape[1]
    if b.shape[0] != m or tuple(out.shape) != (n1, n2):
        raise G2048Error(f"wgrad shapes: a {tuple(a.shape)} b {tuple(b.shape)} out {tuple(out.shape)}")
    _check(load().g2048_wgrad(_stream(a), _dev(a, torch.bfloat16, "a"), _dev(b, torch.bfloat16, "b"), m, n1, n2,
                              _dev(partials, torch.float32, "partials"), _dev(out, torch.float32, "out"),
                              _defer(defer)), "g2048_wgrad")


def wgrad_pair_partials(m: int, n1: int, n2: int) -> int:
    return int(load().g2048_wgrad_pair_partials(m, n1, n2))


def wgrad_pair(a0, b0, a1, b1, partials0, partials1, out0, out1, defer=None):
    """out0 = a0^T b0 and out1 = a1^T b1 (same shapes) in one launch; defer: a list of two ColsumJob."""
    m, n1 = a0.shape
    n2 = b0.shape[1]
    for a, b, o in ((a0, b0, out0), (a1, b1, out1)):
        if a.shape != (m, n1) or b.shape != (m, n2) or tuple(o.shape) != (n1, n2):
            raise G2048Error("wgrad_pair shapes")
    jobs = (ColsumJob * 2)() if defer is not None else None
    _check(load().g2048_wgrad_pair(_stream(a0), *[_dev(t, torch.bfloat16, "a/b") for t in (a0, b0, a1, b1)], m, n1, n2,
                                   _dev(partials0, torch.float32, "partials0"), _dev(partials1, torch.float32, "partials1"),
                                   _dev(out0, torch.float32, "out0"), _dev(out1, torch.float32, "out1"), jobs),
           "g2048_wgrad_pair")
    if defer is not None:
        defer[0], defer[1] = jobs[0], jobs[1]


def colsum_batch(jobs):
    """Performs deferred column sums (ColsumJob list, at most COLSUM_MAX_JOBS) in one launch; `jobs`
    may also be a ctypes array built once (graph-captured callers)."""
    n = len(jobs)
    if n > COLSUM_MAX_JOBS:
        raise G2048Error(f"at most {COLSUM_MAX_JOBS} column-sum jobs per launch")
    if not isinstance(jobs, ctypes.Array):
        jobs = (ColsumJob * max(1, n))(*jobs)
    stream = torch.cuda.current_stream().cuda_stream
    _check(load().g2048_colsum_batch(ctypes.c_void_p(stream), jobs, n), "g2048_colsum_batch")


def colsum_batch_sq(jobs, sq, tick=None):
    """colsum_batch + the gradient norm's partials: sq (fp32, COLSUM_SQ_MAX) <- per-block sums of
    squares of the segments marked in each job's pad_ (bit k = segment k is gradient), *tick += 1."""
    n = len(jobs)
    if n > COLSUM_MAX_JOBS:
        raise G2048Error(f"at most {COLSUM_MAX_JOBS} column-sum jobs per launch")
    if not isinstance(jobs, ctypes.Array):
        jobs = (ColsumJob * max(1, n))(*jobs)
    stream = torch.cuda.current_stream().cuda_stream
    _check(load().g2048_colsum_batch_sq(ctypes.c_void_p(stream), jobs, n, _dev(sq, torch.float32, "sq"), sq.numel(),
                                        _dev(tick, torch.float32, "tick")), "g2048_colsum_batch_sq")


def colsum_batch_blocks(jobs) -> int:
    if not isinstance(jobs, ctypes.Array):
        jobs = (ColsumJob * max(1, len(jobs)))(*jobs)
    return int(load().g2048_colsum_batch_blocks(jobs, len(jobs)))


# ------------------------------------------------------------- optimizer step -------------------
def grad_clip(grad, max_norm: float, norm_out, coef_out, partials):
    """partials: >= 64 float32 of scratch."""
    _check(load().g2048_grad_clip(_stream(grad), _dev(grad, torch.float32, "grad"), grad.numel(), float(max_norm),
                                  _dev(norm_out, torch.float32, "norm_out"), _dev(coef_out, torch.float32, "coef_out"),
                                  _dev(partials, torch.float32, "partials")), "g2048_grad_clip")


def muon_supported(rows: int, cols: int) -> bool:
    return bool(load().g2048_muon_supported(rows, cols))


def muon_step(mats, lr_dev, clip_coef_dev, cfg: MuonCfg, stream_tensor):
    """mats: a ctypes array of MuonMatrix (built once; device pointers stay valid)."""
    _check(load().g2048_muon_step(_stream(stream_tensor), mats, len(mats), _dev(lr_dev, torch.float32, "lr"),
                                  _dev(clip_coef_dev, torch.float32, "clip"), ctypes.byref(cfg)), "g2048_muon_step")


def grad_sumsq(grad, partials):
    _check(load().g2048_grad_sumsq(_stream(grad), _dev(grad, torch.float32, "grad"), grad.numel(),
                                   _dev(partials, torch.float32, "partials")), "g2048_grad_sumsq")


def muon_step_clip(mats, lr_dev, partials, max_norm: float, norm_out, coef_out, cfg: MuonCfg):
    """Muon with the gradient clip folded in (partials from grad_sumsq; norm / coef published)."""
    _check(load().g2048_muon_step_clip(_stream(lr_dev), mats, len(mats), _dev(lr_dev, torch.float32, "lr"),
                                       _dev(partials, torch.float32, "partials"), float(max_norm),
                                       _dev(norm_out, torch.float32, "norm_out"), _dev(coef_out, torch.float32, "coef_out"),
                                       ctypes.byref(cfg)), "g2048_muon_step_clip")


def grad_sumsq_tick(grad, partials, step_dev):
    """grad_sumsq + the optimizer's device step count += 1 (one launch)."""
    _check(load().g2048_grad_sumsq_tick(_stream(grad), _dev(grad, torch.float32, "grad"), grad.numel(),
                                        _dev(partials, torch.float32, "partials"), _dev(step_dev, torch.float32, "step")),
           "g2048_grad_sumsq_tick")


def muon_adamw_step_clip(mats, groups, lr_dev, step_dev, partials, max_norm: float, norm_out, coef_out, cfg: MuonCfg,
                         beta1, beta2, eps, adam_weight_decay):
    """muon_step_clip with the AdamW update of the 1-D groups in the same launch."""
    _check(load().g2048_muon_adamw_step_clip(
        _stream(lr_dev), mats, len(mats), groups, len(groups) if groups is not None else 0,
        _dev(lr_dev, torch.float32, "lr"), _dev(step_dev, torch.float32, "step"),
        _dev(partials, torch.float32, "partials"), float(max_norm), _dev(norm_out, torch.float32, "norm_out"),
        _dev(coef_out, torch.float32, "coef_out"), ctypes.byref(cfg), float(beta1), float(beta2), float(eps),
        float(adam_weight_decay)), "g2048_muon_adamw_step_clip")


def adamw_step(groups, lr_dev, step_dev, clip_coef_dev, beta1, beta2, eps, weight_decay):
    _check(load().g2048_adamw_step(_stream(lr_dev), groups, len(groups), _dev(lr_dev, torch.float32, "lr"),
                                   _dev(step_dev, torch.float32, "step"), _dev(clip_coef_dev, torch.float32, "clip"),
                                   float(beta1), float(beta2), float(eps), float(weight_decay)), "g2048_adamw_step")


def mlp_fwd_supported(n: int, k: int) -> bool:
    return int(load().g2048_mlp_fwd_lds_bytes(n, k)) > 0


def mlp_fwd(x, w, gamma, beta, residual: bool, g, y, mean, rstd, drop: Dropout | None = None):
    """g = x w^T; y = [x +] Dropout(ReLU(LayerNorm(g))) in one MFMA kernel (bf16 x [m,k], w [n,k])."""
    m, k = x.shape
    n = w.shape[0]
    _check(load().g2048_mlp_fwd(
        _stream(x), _dev(x, torch.bfloat16, "x"), _dev(w, torch.bfloat16, "w"), _dev(gamma, torch.float32, "gamma"),
        _dev(beta, torch.float32, "beta"), int(bool(residual)), _dev(g, torch.bfloat16, "g"),
        _dev(y, torch.bfloat16, "y"), _dev(mean, torch.float32, "mean"), _dev(rstd, torch.float32, "rstd"), m, n, k,
        ctypes.byref(drop) if drop is not None else None), "g2048_mlp_fwd")


def head_fwd(x, wa, ba, wv, bv, logits, value):
    """logits [m, >=4] (row stride may exceed 4) and value [m] of the GameMLP heads on MFMA."""
    m, h = x.shape
    if logits.stride(-1) != 1 or logits.dtype != torch.float32 or not logits.is_cuda:
        raise G2048Error("logits must be a float32 device tensor with unit inner stride")
    _check(load().g2048_head_fwd(
        _stream(x), _dev(x, torch.bfloat16, "x"), _dev(wa, torch.float32, "wa"), _dev(ba, torch.float32, "ba"),
        _dev(wv, torch.float32, "wv"), _dev(bv, torch.float32, "bv"), m, h, ctypes.c_void_p(logits.data_ptr()),
        logits.stride(0), _dev(value, torch.float32, "value")), "g2048_head_fwd")


def linear_dgrad_supported(n: int, k: int) -> bool:
    return bool(load().g2048_linear_dgrad_supported(int(n), int(k)))


def linear_dgrad(dg, w, out):
    """out = dg @ w on bf16 MFMA (dg [m, n], w [n, k] the Linear weight, out [m, k], all bf16)."""
    m, n = dg.shape
    k = w.shape[1]
    if w.shape[0] != n or out.shape != (m, k):
        raise G2048Error("linear_dgrad: shape mismatch")
    _check(load().g2048_linear_dgrad(_stream(dg), _dev(dg, torch.bfloat16, "dg"), _dev(w, torch.bfloat16, "w"),
                                     _dev(out, torch.bfloat16, "out"), m, n, k), "g2048_linear_dgrad")


def policy_rollout_supported(hidden: int, num_layers: int) -> bool:
    return bool(load().g2048_policy_rollout_supported(int(hidden), int(num_layers)))


def policy_rollout(buf, t0: int, t1: int, w_stem, w_block, ln_gamma, ln_beta, head_bf16, ba, bv, seed: int,
                   env_base: int, counter_dev, opts: int, counter: int = 0, debug=None):
    """Steps t0 .. t1-1 of a rollout buffer (g2048/rollout.RolloutBuffers) in one fused launch:
    GameMLP (bf16 weights w_stem [h,48], w_block[2] [h,h]; fp32 LayerNorm affines; bf16 heads
    head_bf16 [5, 32*ceil(h/32)]) + sampler + env step, records bitwise the per-step path's."""
    n = buf.boards.shape[1]
    h = w_stem.shape[0]
    T = buf.actions.shape[0]
    if not (0 <= t0 <= t1 <= T) or len(w_block) != 2 or len(ln_gamma) != 3 or len(ln_beta) != 3:
        raise G2048Error("policy_rollout: bad step range or layer count")
    a = PolicyRolloutArgs()
    a.boards = _dev(buf.boards, torch.int8, "boards")
    a.flags = _dev(buf.flags, torch.uint8, "flags")
    a.actions = _dev(buf.actions, torch.uint8, "actions")
    a.logp = _dev(buf.logp, torch.float32, "logp")
    a.entropy = _dev(buf.entropy, torch.float32, "entropy")
    a.value = _dev(buf.value, torch.float32, "value")
    a.points = _dev(buf.points, torch.int32, "points")
    a.max_tile = _dev(buf.max_tile, torch.int8, "max_tile")
    a.pot = _dev(buf.pot, torch.int8, "pot")
    a.n, a.t0, a.t1, a.hidden, a.num_layers = n, t0, t1, h, len(w_block)
    a.opts, a.env_base = opts, env_base
    a.w_stem = _dev(w_stem, torch.bfloat16, "w_stem")
    for i, w in enumerate(w_block):
        a.w_block[i] = _dev(w, torch.bfloat16, "w_block")
    for i in range(3):
        a.ln_gamma[i] = _dev(ln_gamma[i], torch.float32, "ln_gamma")
        a.ln_beta[i] = _dev(ln_beta[i], torch.float32, "ln_beta")
    a.head_bf16 = _dev(head_bf16, torch.bfloat16, "head_bf16")
    a.head_bias_action = _dev(ba, torch.float32, "ba")
    a.head_bias_value = _dev(bv, torch.float32, "bv")
    a.seed, a.counter = seed & (2**64 - 1), counter
    a.counter_dev = _dev(counter_dev, torch.int64, "counter_dev")
    a.debug = _dev(debug, torch.float32, "debug")
    _check(load().g2048_policy_rollout(_stream(buf.boards), ctypes.byref(a)), "g2048_policy_rollout")


def ppo_stats(sums, kl, grad_norm, beta_dev, critic: float, m: int, stats, counter=None, kl_rows: int = 0, rows=None):
    """kl: final {sum, max}, or (kl_rows > 0) the partial rows of a deferred ppo_head_kl."""
    _check(load().g2048_ppo_stats(_stream(stats), _dev(sums, torch.float32, "sums"), _dev(kl, torch.float32, "kl"),
                                  int(kl_rows),
                                  _dev(grad_norm, torch.float32, "grad_norm"), _dev(beta_dev, torch.float32, "beta"),
                                  float(critic), int(m), _dev(rows, torch.int64, "rows"),
                                  _dev(stats, torch.float32, "stats"),
                                  _dev(counter, torch.int64, "counter")), "g2048_ppo_stats")


# ---------------------------------------------------------------- GameURM (include/g2048_urm.h) ----
def urm_stem(obs, w, ln_w, ln_b, init_hidden, emb, x, xb):
    """emb = SiLU(LayerNorm(obs-cell features W^T)); x = init_hidden + emb; xb = bf16(x)."""
    n = obs.shape[0]
    h = w.shape[0]
    if obs.dtype not in (torch.float32, torch.bfloat16):
        raise G2048Error("obs must be float32 or bfloat16")
    _check(load().g2048_urm_stem(_stream(obs), _dev(obs, None, "obs"), int(obs.dtype == torch.bfloat16),
                                 _dev(w, torch.float32, "w"), _dev(ln_w, torch.float32, "ln_w"),
                                 _dev(ln_b, torch.float32, "ln_b"), _dev(init_hidden, torch.float32, "init_hidden"),
                                 _dev(emb, torch.float32, "emb"), _dev(x, torch.float32, "x"),
                                 _dev(xb, torch.bfloat16, "xb"), n, h), "g2048_urm_stem")


def urm_attention(qkv, out, heads: int, p: float = 0.0, seed: int = 0, counter=None, offset: int = 0):
    """counter: device int64 [1] call counter of the dropout mask (required when p > 0); the mask is
    keyed by *counter + offset."""
    rows, h3 = qkv.shape
    if p > 0.0:
        _check(load().g2048_urm_attention_drop_at(_stream(qkv), _dev(qkv, torch.bfloat16, "qkv"),
                                                  _dev(out, torch.bfloat16, "out"), rows // 16, h3 // 3, int(heads),
                                                  float(p), int(seed) & (2 ** 64 - 1),
                                                  _dev(counter, torch.int64, "counter"), int(offset)),
               "g2048_urm_attention_drop_at")
        return
    _check(load().g2048_urm_attention(_stream(qkv), _dev(qkv, torch.bfloat16, "qkv"), _dev(out, torch.bfloat16, "out"),
                                      rows // 16, h3 // 3, int(heads)), "g2048_urm_attention")


def urm_attention_bwd(qkv, dout, dqkv, heads: int, p: float = 0.0, seed: int = 0, counter=None, offset: int = 0):
    rows, h3 = qkv.shape
    if p > 0.0:
        _check(load().g2048_urm_attention_bwd_drop_at(_stream(qkv), _dev(qkv, torch.bfloat16, "qkv"),
                                                      _dev(dout, torch.bfloat16, "dout"),
                                                      _dev(dqkv, torch.bfloat16, "dqkv"), rows // 16, h3 // 3, int(heads),
                                                      float(p), int(seed) & (2 ** 64 - 1),
                                                      _dev(counter, torch.int64, "counter"), int(offset)),
               "g2048_urm_attention_bwd_drop_at")
        return
    _check(load().g2048_urm_attention_bwd(_stream(qkv), _dev(qkv, torch.bfloat16, "qkv"),
                                          _dev(dout, torch.bfloat16, "dout"), _dev(dqkv, torch.bfloat16, "dqkv"),
                                          rows // 16, h3 // 3, int(heads)), "g2048_urm_attention_bwd")


def urm_stem_partials(n: int) -> int:
    return int(load().g2048_urm_stem_partials(n))


def _obs_dtype(obs) -> int:
    if obs.dtype not in (torch.float32, torch.bfloat16):
        raise G2048Error(f"obs must be float32 or bfloat16, got {obs.dtype}")
    return 1 if obs.dtype == torch.bfloat16 else 0


def urm_stem_fwd(obs, w, ln_w, ln_b, emb, eps: float):
    rows, h = emb.shape
    _check(load().g2048_urm_stem_fwd(_stream(obs), _dev(obs, None, "obs"), _obs_dtype(obs), _dev(w, torch.float32, "w"),
                                     _dev(ln_w, torch.float32, "ln_w"), _dev(ln_b, torch.float32, "ln_b"),
                                     _dev(emb, torch.float32, "emb"), rows // 16, h, float(eps)), "g2048_urm_stem_fwd")


def urm_stem_bwd(obs, w, ln_w, ln_b, demb, grads, partials, eps: float):
    rows, h = demb.shape
    _check(load().g2048_urm_stem_bwd(_stream(obs), _dev(obs, None, "obs"), _obs_dtype(obs), _dev(w, torch.float32, "w"),
                                     _dev(ln_w, torch.float32, "ln_w"), _dev(ln_b, torch.float32, "ln_b"),
                                     _dev(demb, torch.float32, "demb"), _dev(grads, torch.float32, "grads"),
                                     _dev(partials, torch.float32, "partials"), rows // 16, h, float(eps)),
           "g2048_urm_stem_bwd")


def urm_stem_bwd3(obs, w, ln_w, ln_b, demb, dw, dln_w, dln_b, partials, eps: float, accumulate: bool = False):
    """g2048_urm_stem_bwd3: the three stem gradients at their own addresses (accumulate: added to)."""
    rows, h = demb.shape
    _check(load().g2048_urm_stem_bwd3(_stream(obs), _dev(obs, None, "obs"), _obs_dtype(obs), _dev(w, torch.float32, "w"),
                                      _dev(ln_w, torch.float32, "ln_w"), _dev(ln_b, torch.float32, "ln_b"),
                                      _dev(demb, torch.float32, "demb"), _dev(dw, torch.float32, "dw"),
                                      _dev(dln_w, torch.float32, "dln_w"), _dev(dln_b, torch.float32, "dln_b"),
                                      int(bool(accumulate)), _dev(partials, torch.float32, "partials"), rows // 16, h,
                                      float(eps)), "g2048_urm_stem_bwd3")


def urm_rms_res_fwd(h, a, out, rstd, eps: float, outb=None):
    """outb: optional bf16 [rows, 64] copy of out (g2048_urm_rms_res_fwd2)."""
    rows, hid = h.shape
    abf = a.dtype == torch.bfloat16
    _check(load().g2048_urm_rms_res_fwd2(_stream(h), _dev(h, torch.float32, "h"),
                                         _dev(a, torch.bfloat16 if abf else torch.float32, "a"), int(abf),
                                         _dev(out, torch.float32, "out"), _dev(outb, torch.bfloat16, "outb"),
                                         _dev(rstd, torch.float32, "rstd"), rows, hid, float(eps)),
           "g2048_urm_rms_res_fwd2")


def urm_add_cast(a, a_rows: int, e, out, outb):
    """out = a + e, outb = bf16(out) (g2048_urm_add_cast); a broadcast over groups of a_rows rows
    when a_rows > 0."""
    rows, hid = e.shape
    _check(load().g2048_urm_add_cast(_stream(e), _dev(a, torch.float32, "a"), int(a_rows), _dev(e, torch.float32, "e"),
                                     _dev(out, torch.float32, "out"), _dev(outb, torch.bfloat16, "outb"), rows, hid),
           "g2048_urm_add_cast")


def urm_add_cast_bwd(dout, doutb, dx, acc_in=None, acc_out=None):
    """dx = dout + float(doutb) (either may be None); acc_out = acc_in + dx when given, dx may then be
    None (g2048_urm_add_cast_bwd_acc)."""
    ref = dx if dx is not None else acc_out
    rows, hid = ref.shape
    _check(load().g2048_urm_add_cast_bwd_acc(_stream(ref), _dev(dout, torch.float32, "dout"),
                                             _dev(doutb, torch.bfloat16, "doutb"), _dev(dx, torch.float32, "dx"),
                                             _dev(acc_in, torch.float32, "acc_in"), _dev(acc_out, torch.float32, "acc_out"),
                                             rows, hid), "g2048_urm_add_cast_bwd_acc")


def urm_rms_res_bwd(dout, out, rstd, dh, da, doutb=None, dpool=None):
    """dout fp32 and / or doutb bf16 (the bf16 copy's gradient); either may be None.  dpool (instead of
    dout): fp32 [rows / 16, 64] broadcast over each board's 16 token rows (the mean-pool backward)."""
    rows, hid = out.shape
    abf = da.dtype == torch.bfloat16
    _check(load().g2048_urm_rms_res_bwd3(_stream(out), _dev(dout, torch.float32, "dout"), _dev(dpool, torch.float32, "dpool"),
                                         _dev(doutb, torch.bfloat16, "doutb"), _dev(out, torch.float32, "out"),
                                         _dev(rstd, torch.float32, "rstd"), _dev(dh, torch.float32, "dh"),
                                         _dev(da, torch.bfloat16 if abf else torch.float32, "da"), int(abf), rows, hid),
           "g2048_urm_rms_res_bwd3")


def urm_swiglu_conv_partials(n: int, inter: int) -> int:
    return int(load().g2048_urm_swiglu_conv_partials(n, inter))


def urm_gate_up_swiglu_bwd_supported(h: int, inter: int) -> bool:
    return bool(load().g2048_urm_gate_up_swiglu_bwd_supported(h, inter))


def urm_gate_up_swiglu_bwd(x, w, conv_w, conv_b, dact, dgu, dw, db, partials, accumulate: bool = False):
    """dgu, dw, db of the SwiGLU-conv with gu = bf16(x w^T) recomputed on MFMA
    (g2048_urm_gate_up_swiglu_bwd_acc; accumulate: dw / db += the sums)."""
    rows, h = x.shape
    inter = w.shape[0] // 2
    _check(load().g2048_urm_gate_up_swiglu_bwd_acc(_stream(x), _dev(x, torch.bfloat16, "x"), _dev(w, torch.bfloat16, "w"),
                                                   _dev(conv_w, torch.float32, "conv_w"),
                                                   _dev(conv_b, torch.float32, "conv_b"),
                                                   _dev(dact, torch.bfloat16, "dact"), _dev(dgu, torch.bfloat16, "dgu"),
                                                   _dev(dw, torch.float32, "dw"), _dev(db, torch.float32, "db"),
                                                   _dev(partials, torch.float32, "partials"), rows // 16, h, inter,
                                                   int(bool(accumulate))), "g2048_urm_gate_up_swiglu_bwd_acc")


def urm_swiglu_conv_fwd(gu, w, b, act):
    rows, inter = act.shape
    _check(load().g2048_urm_swiglu_conv_fwd(_stream(gu), _dev(gu, torch.bfloat16, "gu"), _dev(w, torch.float32, "w"),
                                            _dev(b, torch.float32, "b"), _dev(act, torch.bfloat16, "act"), rows // 16,
                                            inter), "g2048_urm_swiglu_conv_fwd")


def urm_swiglu_conv_bwd(gu, w, b, dact, dgu, dw, db, partials):
    rows, inter = dact.shape
    _check(load().g2048_urm_swiglu_conv_bwd(_stream(gu), _dev(gu, torch.bfloat16, "gu"), _dev(w, torch.float32, "w"),
                                            _dev(b, torch.float32, "b"), _dev(dact, torch.bfloat16, "dact"),
                                            _dev(dgu, torch.bfloat16, "dgu"), _dev(dw, torch.float32, "dw"),
                                            _dev(db, torch.float32, "db"), _dev(partials, torch.float32, "partials"),
                                            rows // 16, inter), "g2048_urm_swiglu_conv_bwd")


def urm_residual_rms(x, y, emb, xb, eps: float):
    rows, h = x.shape
    _check(load().g2048_urm_residual_rms(_stream(x), _dev(x, torch.float32, "x"), _dev(y, torch.bfloat16, "y"),
                                         _dev(emb, torch.float32, "emb"), _dev(xb, torch.bfloat16, "xb"), rows, h,
                                         float(eps)), "g2048_urm_residual_rms")


def urm_swiglu_conv(gu, w, b, out):
    rows, inter2 = gu.shape
    _check(load().g2048_urm_swiglu_conv(_stream(gu), _dev(gu, torch.bfloat16, "gu"), _dev(w, torch.float32, "w"),
                                        _dev(b, torch.float32, "b"), _dev(out, torch.bfloat16, "out"), rows // 16,
                                        inter2 // 2), "g2048_urm_swiglu_conv")


def urm_pool_heads(x, wa, ba, wv, bv, logits, value):
    rows, h = x.shape
    _check(load().g2048_urm_pool_heads(_stream(x), _dev(x, torch.float32, "x"), _dev(wa, torch.float32, "wa"),
                                       _dev(ba, torch.float32, "ba"), _dev(wv, torch.float32, "wv"),
                                       _dev(bv, torch.float32, "bv"), _dev(logits, torch.float32, "logits"),
                                       _dev(value, torch.float32, "value"), rows // 16, h), "g2048_urm_pool_heads")


def urm_linear_supported(epilogue: int, k: int, n: int, inter: int = 0) -> bool:
    return bool(load().g2048_urm_linear_supported(int(epilogue), int(k), int(n), int(inter)))


def urm_linear(inp, w, out):
    """out = inp w^T (bf16, fp32 accumulate) on the fused-projection kernel (qkv_proj)."""
    rows, k = inp.shape
    _check(load().g2048_urm_linear(_stream(inp), _dev(inp, torch.bfloat16, "in"), _dev(w, torch.bfloat16, "w"),
                                   _dev(out, torch.bfloat16, "out"), rows, k, w.shape[0]), "g2048_urm_linear")


def urm_linear_t(inp, w, out):
    """out = inp w for w [k, n] (bf16): dX = dY W without a transposed copy (g2048_urm_linear_t)."""
    rows, k = inp.shape
    _check(load().g2048_urm_linear_t(_stream(inp), _dev(inp, torch.bfloat16, "in"), _dev(w, torch.bfloat16, "w"),
                                     _dev(out, torch.bfloat16, "out"), rows, k, w.shape[1]), "g2048_urm_linear_t")


def urm_linear_bias(inp, w, bias, out):
    """out = bf16(inp w^T + bias) with one rounding (autocast's biased Linear; g2048_urm_linear_bias)."""
    rows, k = inp.shape
    _check(load().g2048_urm_linear_bias(_stream(inp), _dev(inp, torch.bfloat16, "in"), _dev(w, torch.bfloat16, "w"),
                                        _dev(bias, torch.float32, "bias"), _dev(out, torch.bfloat16, "out"), rows, k,
                                        w.shape[0]), "g2048_urm_linear_bias")


def urm_linear_res_rms(inp, w, h, out, outb, rstd, eps: float):
    """out = rms_norm(h + bf16(inp w^T)), outb = bf16(out) (optional), rstd (g2048_urm_linear_res_rms)."""
    rows, k = inp.shape
    _check(load().g2048_urm_linear_res_rms(_stream(inp), _dev(inp, torch.bfloat16, "in"), _dev(w, torch.bfloat16, "w"),
                                           _dev(h, torch.float32, "h"), _dev(out, torch.float32, "out"),
                                           _dev(outb, torch.bfloat16, "outb"), _dev(rstd, torch.float32, "rstd"), rows,
                                           k, w.shape[0], float(eps)), "g2048_urm_linear_res_rms")


def urm_linear_rms(inp, w, x, emb, xb, eps: float):
    """x = rms_norm(x + inp w^T) [+ emb]; xb = bf16(x)  (o_proj / down_proj with the post-norm)."""
    rows, k = inp.shape
    _check(load().g2048_urm_linear_rms(_stream(inp), _dev(inp, torch.bfloat16, "in"), _dev(w, torch.bfloat16, "w"),
                                       _dev(x, torch.float32, "x"), _dev(emb, torch.float32, "emb"),
                                       _dev(xb, torch.bfloat16, "xb"), rows, k, w.shape[0], float(eps)),
           "g2048_urm_linear_rms")


def urm_wgrad_supported(n: int, k: int) -> bool:
    """g2048_urm_wgrad covers dw [n, k] (the projection shapes of the URM training Functions)."""
    return bool(load().g2048_urm_wgrad_supported(n, k))


def urm_wgrad_partials(m: int, n: int, k: int) -> int:
    return int(load().g2048_urm_wgrad_partials(m, n, k))


def lds_poison(word: int, device=None):
    """Test hook: every CU's LDS filled with the 32-bit `word` (g2048_lds_poison)."""
    dev = device or torch.device("cuda", torch.cuda.current_device())
    _check(load().g2048_lds_poison(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream), int(word) & 0xFFFFFFFF),
           "g2048_lds_poison")


def urm_head_loss_partials(m: int, h: int) -> int:
    return int(load().g2048_urm_head_loss_partials(m, h))


def _pooled_dtype(t) -> int:
    if t.dtype not in (torch.float32, torch.bfloat16):
        raise G2048Error("pooled must be float32 or bfloat16")
    return int(t.dtype == torch.bfloat16)


def urm_head_loss(pooled, wa, ba, wv, bv, batch: PPOBatch, beta_dev, critic, clip_eps, dz, masked, partials, sync,
                  sums, loss):
    """GameURM's heads + PPO loss + dz / masked / sums / loss (g2048_urm_head_loss)."""
    m, h = pooled.shape
    _check(load().g2048_urm_head_loss(
        _stream(pooled), _dev(pooled, None, "pooled"), _pooled_dtype(pooled), _dev(wa, torch.float32, "wa"),
        _dev(ba, torch.float32, "ba"), _dev(wv, torch.float32, "wv"), _dev(bv, torch.float32, "bv"), m, h,
        ctypes.byref(batch), _dev(beta_dev, torch.float32, "beta"), float(critic), float(clip_eps),
        _dev(dz, torch.float32, "dz"), _dev(masked, torch.float32, "masked"), _dev(partials, torch.float32, "partials"),
        _dev(sync, torch.int32, "sync"), _dev(sums, torch.float32, "sums"), _dev(loss, torch.float32, "loss")),
        "g2048_urm_head_loss")


def urm_head_loss_bwd(pooled, wa, wv, dz, grad_out, dpooled, partials, sync, dwa, dba, dwv, dbv,
                      accumulate: bool = False):
    """dpooled and the head gradients of g2048_urm_head_loss (g2048_urm_head_loss_bwd)."""
    m, h = pooled.shape
    _check(load().g2048_urm_head_loss_bwd(
        _stream(pooled), _dev(pooled, None, "pooled"), _pooled_dtype(pooled), _dev(wa, torch.float32, "wa"),
        _dev(wv, torch.float32, "wv"), _dev(dz, torch.float32, "dz"), _dev(grad_out, torch.float32, "grad_out"),
        _dev(dpooled, pooled.dtype, "dpooled"), _dev(partials, torch.float32, "partials"), _dev(sync, torch.int32, "sync"),
        _dev(dwa, torch.float32, "dwa"), _dev(dba, torch.float32, "dba"), _dev(dwv, torch.float32, "dwv"),
        _dev(dbv, torch.float32, "dbv"), int(bool(accumulate)), m, h), "g2048_urm_head_loss_bwd")


def urm_kl_stats(old_masked, logits, sums, gn, beta_dev, critic, stats, partials, sync):
    """KL(old || new) + the minibatch statistics update (g2048_urm_kl_stats)."""
    _check(load().g2048_urm_kl_stats(
        _stream(logits), _dev(old_masked, torch.float32, "old_masked"), _dev(logits, torch.float32, "logits"),
        logits.shape[0], _dev(sums, torch.float32, "sums"), _dev(gn, torch.float32, "gn"),
        _dev(beta_dev, torch.float32, "beta"), float(critic), _dev(stats, torch.float32, "stats"),
        _dev(partials, torch.float32, "partials"), _dev(sync, torch.int32, "sync")), "g2048_urm_kl_stats")


def urm_wgrad(dy, x, dw, partials, accumulate: bool = False):
    """dw fp32 [n, k] = dy^T x (g2048_urm_wgrad_acc; accumulate: dw += dy^T x); dy bf16 [m, n], x bf16 [m, k]."""
    m, n = dy.shape
    _check(load().g2048_urm_wgrad_acc(_stream(dy), _dev(dy, torch.bfloat16, "dy"), _dev(x, torch.bfloat16, "x"),
                                      _dev(dw, torch.float32, "dw"), _dev(partials, torch.float32, "partials"), m, n,
                                      x.shape[1], int(bool(accumulate))), "g2048_urm_wgrad_acc")


def urm_linres_bwd_supported(hidden: int, k: int) -> bool:
    return bool(load().g2048_urm_linres_bwd_supported(hidden, k))


def urm_linres_bwd_partials(rows: int, k: int) -> int:
    return int(load().g2048_urm_linres_bwd_partials(rows, k))


def urm_linres_bwd(out, rstd, w, x, dh, dw, partials, dout=None, dpool=None, doutb=None, dx=None,
                   accumulate: bool = False):
    """The residual-RMSNorm projection's backward in one pass (g2048_urm_linres_bwd): dh fp32 [rows, 64],
    dx bf16 [rows, k] (None: skipped), dw fp32 [64, k] (+= with accumulate) from dout fp32 [rows, 64] /
    dpool fp32 [rows / 16, 64] / doutb bf16 [rows, 64] (each may be None), out fp32, rstd fp32 [rows],
    w bf16 [64, k], x bf16 [rows, k]."""
    rows, hid = out.shape
    k = x.shape[1]
    _check(load().g2048_urm_linres_bwd(_stream(out), _dev(dout, torch.float32, "dout"), _dev(dpool, torch.float32, "dpool"),
                                       _dev(doutb, torch.bfloat16, "doutb"), _dev(out, torch.float32, "out"),
                                       _dev(rstd, torch.float32, "rstd"), _dev(w, torch.bfloat16, "w"),
                                       _dev(x, torch.bfloat16, "x"), _dev(dh, torch.float32, "dh"),
                                       _dev(dx, torch.bfloat16, "dx"), _dev(dw, torch.float32, "dw"),
                                       _dev(partials, torch.float32, "partials"), int(bool(accumulate)), rows, hid, k),
           "g2048_urm_linres_bwd")


def urm_linear_swiglu_train(inp, w, conv_w, conv_b, gu, act):
    rows, h = inp.shape
    _check(load().g2048_urm_linear_swiglu_train(_stream(inp), _dev(inp, torch.bfloat16, "in"),
                                                _dev(w, torch.bfloat16, "w"), _dev(conv_w, torch.float32, "conv_w"),
                                                _dev(conv_b, torch.float32, "conv_b"), _dev(gu, torch.bfloat16, "gu"),
                                                _dev(act, torch.bfloat16, "act"), rows, h, act.shape[1]),
           "g2048_urm_linear_swiglu_train")


def urm_linear_swiglu(inp, w, conv_w, conv_b, out):
    """out = SiLU(dwconv(SiLU(gate) * up)) with [gate | up] = inp w^T (gate_up_proj + ConvSwiGLU)."""
    rows, h = inp.shape
    _check(load().g2048_urm_linear_swiglu(_stream(inp), _dev(inp, torch.bfloat16, "in"), _dev(w, torch.bfloat16, "w"),
                                          _dev(conv_w, torch.float32, "conv_w"), _dev(conv_b, torch.float32, "conv_b"),
                                          _dev(out, torch.bfloat16, "out"), rows, h, w.shape[0] // 2),
           "g2048_urm_linear_swiglu")


def urm_forward_supported(hidden: int, heads: int, inter: int, num_layers: int, conv_kernel: int) -> bool:
    return bool(load().g2048_urm_forward_supported(int(hidden), int(heads), int(inter), int(num_layers),
                                                   int(conv_kernel)))


def urm_forward_drop(weights: UrmWeights, obs, logits, value, p: float, seed: int, counter):
    """g2048_urm_forward in training mode (attention dropout p, mask counter *counter + block app)."""
    if obs.dtype not in (torch.float32, torch.bfloat16):
        raise G2048Error("obs must be float32 or bfloat16")
    _check(load().g2048_urm_forward_drop(_stream(obs), ctypes.byref(weights), _dev(obs, None, "obs"),
                                         int(obs.dtype == torch.bfloat16), _dev(logits, torch.float32, "logits"),
                                         _dev(value, torch.float32, "value"), obs.shape[0], float(p),
                                         int(seed) & (2 ** 64 - 1), _dev(counter, torch.int64, "counter")),
           "g2048_urm_forward_drop")


def urm_forward(weights: UrmWeights, obs, logits, value):
    """The whole GameURM forward in one launch (g2048_urm_forward); `weights` holds device pointers."""
    if obs.dtype not in (torch.float32, torch.bfloat16):
        raise G2048Error("obs must be float32 or bfloat16")
    _check(load().g2048_urm_forward(_stream(obs), ctypes.byref(weights), _dev(obs, None, "obs"),
                                    int(obs.dtype == torch.bfloat16), _dev(logits, torch.float32, "logits"),
                                    _dev(value, torch.float32, "value"), obs.shape[0]), "g2048_urm_forward")
