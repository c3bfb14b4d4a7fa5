"""Metric logging with the reference's output formats (logger.py:11-168).

stdout: "--- Step N ---" then "  key: value" lines (floats as .2f, or .2e when |v| < 0.01 or >= 1e4);
JSONL: one {"step", "timestamp", **metrics} object per line in "<log_dir>/<name>_<YYYYMMDD>_<NNN>.jsonl";
wandb only when importable (it is not in this image) -- the reference degrades the same way.
"""

from __future__ import annotations

import json
from datetime import datetime
from pathlib import Path
from typing import Any


class MetricLogger:
    def __init__(self, log_dir=None, experiment_name: str = "train", use_wandb: bool = False, wandb_project=None,
                 wandb_run_name=None, wandb_config=None, quiet: bool = False):
        self.quiet = quiet
        self.log_file = None
        self._fh = None
        self.use_wandb = False
        self._wandb = None
        if log_dir is not None:
            d = Path(log_dir)
            d.mkdir(parents=True, exist_ok=True)
            stamp = datetime.now().strftime("%Y%m%d")
            k = 1
            while (d / f"{experiment_name}_{stamp}_{k:03d}.jsonl").exists():
                k += 1
            self.log_file = d / f"{experiment_name}_{stamp}_{k:03d}.jsonl"
            self._fh = open(self.log_file, "a")
            self.print(f"Logging to: {self.log_file}")
        if use_wandb:
            try:
                import wandb  # noqa: F401
                self._wandb = wandb
                self._wandb.init(project=wandb_project, name=wandb_run_name, config=wandb_config, reinit=True)
                self.use_wandb = True
            except ImportError:
                self.print("Warning: wandb not installed. Install with 'pip install wandb'")

    @staticmethod
    def _fmt(v: Any) -> str:
        if isinstance(v, float):
            return f"{v:.2e}" if (abs(v) < 0.01 or abs(v) >= 10000) else f"{v:.2f}"
        return str(v)

    def log(self, metrics: dict, step=None, header=None, verbose: bool = True):
        if verbose and not self.quiet:
            if header is not None:
                print(header)
            elif step is not None:
                print(f"--- Step {step} ---")
            for k, v in metrics.items():
                print(f"  {k}: {self._fmt(v)}")
        if self._fh is not None:
            entry = {"step": step, "timestamp": datetime.now().isoformat()}
            entry.update(metrics)
            self._fh.write(json.dumps(entry) + "\n")
            self._fh.flush()
        if self.use_wandb:
            self._wandb.log(metrics, step=step)

    def print(self, msg: str = ""):
        if not self.quiet:
            print(msg, flush=True)

    def close(self):
        if self._fh is not None:
            self._fh.close()
            self._fh = None
        if self.use_wandb:
            self._wandb.finish()
            self.use_wandb = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
