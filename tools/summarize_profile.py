"""Condense a tools/profile.sh output directory into the committed profile summary.

    python tools/summarize_profile.py gpurun_out/prof_<tag> profiles/<tag>

Writes kernel_stats.csv (rocprofv3 --stats of the trace pass, copied), domain_stats.csv when
present, and pmc_summary.json: per kernel the average FETCH_SIZE / WRITE_SIZE per dispatch (KB =
1024 B, as rocprofv3 reports) and the HBM traffic per dispatch = 2 x FETCH_SIZE + WRITE_SIZE
(gfx950 counts a wide coalesced streaming read at half its bytes in FETCH_SIZE:
/opt/skills/guides/MI355X_MICROARCH.md, HBM section).
"""

from __future__ import annotations

import collections
import csv
import json
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
    print(json.dumps({k: v.get("hbm_bytes_per_dispatch") for k, v in summary.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
