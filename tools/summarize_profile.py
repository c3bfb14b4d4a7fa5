"""Condense a tools/profile.sh output directory into the committed profile summary.

    python tools/summarize_profile.py gpurun_out/prof_<tag> profiles/<tag>

Writes kernel_stats.csv (rocprofv3 --stats of the trace pass, copied), domain_stats.csv when
present, pmc_summary.json: per kernel the average FETCH_SIZE / WRITE_SIZE per dispatch (KB =
1024 B, as rocprofv3 reports) and the HBM traffic per dispatch = 2 x FETCH_SIZE + WRITE_SIZE
(gfx950 counts a wide coalesced streaming read at half its bytes in FETCH_SIZE:
/opt/skills/guides/MI355X_MICROARCH.md, HBM section), pmc_sq.json: per kernel the average of
every SQ/GRBM counter of the sqa/sqb passes, and pmc_env_rollout.json: the headline kernel's
counters normalised per env-step / per wave-step for bench.py (PMC_ENVS / PMC_CHUNK = the
rollout configuration of the PMC passes, default 65536 x 256).
"""

from __future__ import annotations

import collections
import csv
import json
import os
import shutil
import sys
from pathlib import Path


def counters(path: Path, name: str) -> dict:
    out = collections.defaultdict(list)
    for f in path.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                out[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return out


def main(src: str, dst: str):
    src_p, dst_p = Path(src), Path(dst)
    dst_p.mkdir(parents=True, exist_ok=True)
    for pattern, name in (("*kernel_stats.csv", "kernel_stats.csv"), ("*domain_stats.csv", "domain_stats.csv")):
        found = sorted(src_p.rglob(pattern))
        if found:
            shutil.copy(found[0], dst_p / name)
    fetch = counters(src_p / "fetch", "FETCH_SIZE")
    write = counters(src_p / "write", "WRITE_SIZE")
    summary = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        e = {}
        if f:
            e["FETCH_SIZE"] = {"dispatches": len(f), "avg_KB": sum(f) / len(f)}
        if w:
            e["WRITE_SIZE"] = {"dispatches": len(w), "avg_KB": sum(w) / len(w)}
        if f and w:
            e["hbm_bytes_per_dispatch"] = (2 * sum(f) / len(f) + sum(w) / len(w)) * 1024
        summary[k] = e
    (dst_p / "pmc_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
    sq = collections.defaultdict(dict)
    for sub in ("sqa", "sqb", "sqc"):
        for f in (src_p / sub).rglob("*counter_collection.csv") if (src_p / sub).exists() else []:
            acc = collections.defaultdict(list)
            for r in csv.DictReader(open(f)):
                acc[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
            for (k, c), v in acc.items():
                sq[k][c] = sum(v) / len(v)
    if sq:
        (dst_p / "pmc_sq.json").write_text(json.dumps(sq, indent=1, sort_keys=True) + "\n")
    roll = next((k for k in summary if k.startswith("env_rollout_kernel")), None)
    sqr = next((v for k, v in sq.items() if k.startswith("env_rollout_kernel")), None)
    if roll and sqr and "hbm_bytes_per_dispatch" in summary[roll]:
        envs, chunk = int(os.environ.get("PMC_ENVS", 65536)), int(os.environ.get("PMC_CHUNK", 256))
        steps = envs * chunk
        ws = sqr["SQ_WAVES"] * chunk
        out = {"envs": envs, "chunk": chunk, "hbm_bytes_per_dispatch": summary[roll]["hbm_bytes_per_dispatch"],
               "hbm_bytes_per_env_step": summary[roll]["hbm_bytes_per_dispatch"] / steps,
               "valu_per_wave_step": sqr["SQ_INSTS_VALU"] / ws, "lds_per_wave_step": sqr["SQ_INSTS_LDS"] / ws,
               "salu_per_wave_step": sqr.get("SQ_INSTS_SALU", 0.0) / ws,
               "lds_conflict_per_lds_inst": sqr.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(sqr["SQ_INSTS_LDS"], 1.0),
               "counters": sqr}
        (dst_p / "pmc_env_rollout.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps({k: v.get("hbm_bytes_per_dispatch") for k, v in summary.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
