"""CPU-side checks of the C ABI: the library loads and exports every symbol include/*.h declares,
and the Python seam refuses CPU tensors (no silent CPU fallback)."""

import ctypes
import re

import pytest
import torch

from conftest import ROOT


def declared_functions():
    text = "\n".join(p.read_text() for p in sorted((ROOT / "include").glob("*.h")))
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(g2048_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("g2048_env_step", "g2048_env_reset", "g2048_legal_mask", "g2048_obs_encode",
                     "g2048_sample_actions", "g2048_reward_rtg", "g2048_rtg_prepare", "g2048_rtg_finalize",
                     "g2048_mt_seed", "g2048_obs_gather", "g2048_ln_act_fwd", "g2048_ln_act_bwd",
                     "g2048_ppo_head_loss", "g2048_ppo_head_kl"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from g2048 import _lib
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(_lib.EXPORTED) == set(declared_functions())
    assert b"gfx950" in lib.g2048_build_info()
    assert lib.g2048_mt_state_words() == 625


def test_library_is_gfx950_code_object():
    from g2048 import _lib
    data = _lib.LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_cpu_tensors_are_rejected():
    from g2048 import _lib
    b = torch.zeros(4, 16, dtype=torch.int8)
    f = torch.zeros(4, dtype=torch.uint8)
    with pytest.raises(_lib.G2048Error):
        _lib.legal_mask(b, f)


def test_struct_layouts_match_header():
    from g2048 import _lib
    assert ctypes.sizeof(_lib.Rng) == 48
    assert _lib.Rng.counter_dev.offset == 24
    assert ctypes.sizeof(_lib.RewardCfg) == 40
    assert ctypes.sizeof(_lib.Dropout) == 40
    assert _lib.Dropout.counter_dev.offset == 32
    assert ctypes.sizeof(_lib.PPOBatch) == 56 and _lib.PPOBatch.rows.offset == 48
    assert ctypes.sizeof(_lib.Dy) == 64 and _lib.Dy.dz.offset == 40 and _lib.DY_MAX_P == 4
    assert ctypes.sizeof(_lib.ColsumJob) == 88 and _lib.ColsumJob.len.offset == 64
    assert ctypes.sizeof(_lib.MlpPassArgs) == 424 and _lib.MlpPassArgs.drop.offset == 176
    assert _lib.MlpPassArgs.keep.offset == 408 and _lib.MlpPassArgs.idx_offset.offset == 416
    assert ctypes.sizeof(_lib.PPOStatsArgs) == 88 and _lib.PPOStatsArgs.idx_offset.offset == 72
    assert ctypes.sizeof(_lib.MlpBackArgs) == 312 and _lib.MlpBackArgs.keep.offset == 304
    assert ctypes.sizeof(_lib.MuonCfg) == 48 and _lib.MuonCfg.workspace.offset == 40
    assert ctypes.sizeof(_lib.MuonMatrix) == 56 and _lib.MuonMatrix.head_frag.offset == 32
    assert _lib.MlpPassArgs.partials.offset == 400


def test_urm_wgrad_supported_shapes():
    """The URM training Functions pick g2048_urm_wgrad only for shapes it accepts (<= 64 output
    tiles): hidden 64 (default) qkv / o / gate_up / down yes; hidden 80 qkv (240 x 80 = 75 tiles) and
    hidden 192 o_proj (144 tiles) fall back to autocast's nn.Linear."""
    from g2048 import _lib
    for n, k in ((192, 64), (64, 64), (240, 64), (64, 120)):
        assert _lib.urm_wgrad_supported(n, k), (n, k)
    for n, k in ((240, 80), (192, 192), (256, 256), (8, 64), (64, 60)):
        assert not _lib.urm_wgrad_supported(n, k), (n, k)
