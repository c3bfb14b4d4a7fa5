"""In-memory loader for the read-only reference at /root/reference (fixture generation only).

The reference targets Python 3.12 (`/root/reference/.python-version`); this container runs
3.10.12.  Two 3.12-only constructs stop a plain import:

* `game.py:3`   ``type Grid = list[list[int]]``  (PEP 695)        -> SyntaxError on 3.10
* `train.py:15` ``from typing import NotRequired``                  -> ImportError on 3.10

and `train.py:30` imports `batched_rollout`, a module missing from the snapshot.

This shim reads the reference files as text, rewrites only the PEP-695 line into a plain
assignment, and `exec`s the sources into fresh module objects.  Nothing under /root/reference is
written (bytecode writing is disabled) and nothing is fetched.  It is used exclusively by
`tools/gen_golden.py`, which runs in the build container; the reference never travels to the GPU
box and no test, smoke() or bench.py code path imports this module.
"""

from __future__ import annotations

import sys
import types
import typing
from pathlib import Path

REF = Path("/root/reference")


def _exec_module(name: str, path: Path, patch=None) -> types.ModuleType:
    src = path.read_text()
    if patch is not None:
        src = patch(src)
    mod = types.ModuleType(name)
    mod.__file__ = str(path)
    sys.modules[name] = mod
    exec(compile(src, str(path), "exec"), mod.__dict__)
    return mod


def load_reference():
    """Return (game, train) reference modules loaded in memory."""
    if not REF.exists():
        raise FileNotFoundError("reference not mounted at /root/reference")
    sys.dont_write_bytecode = True
    import typing_extensions

    if not hasattr(typing, "NotRequired"):
        typing.NotRequired = typing_extensions.NotRequired  # 3.11+ name used at train.py:15

    game = _exec_module(
        "game",
        REF / "game.py",
        patch=lambda s: s.replace("type Grid = list[list[int]]", "Grid = list[list[int]]", 1),
    )
    _exec_module("logger", REF / "logger.py")

    stub = types.ModuleType("batched_rollout")

    def play_games_batched(*args, **kwargs):  # the missing module of train.py:30
        raise RuntimeError("batched_rollout is not part of the reference snapshot")

    stub.play_games_batched = play_games_batched
    sys.modules["batched_rollout"] = stub
    train = _exec_module("train", REF / "train.py")
    return game, train
