"""Sum the HBM traffic of the GameURM update between tools/urm_update_pmc.py's two marker dispatches.

    python3 tools/urm_update_hbm.py gpurun_out/purmhbm_<tag> profiles/<tag>/urm_update_hbm.json

Inputs: <src>/fetch and <src>/write (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the
program; KB = 1024 B as rocprofv3 reports) and <src>/fetch.log (its URM_UPDATE_PMC line).  HBM bytes
per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 counts a wide coalesced streaming read at half
its bytes in FETCH_SIZE: MI355X_MICROARCH.md, HBM section), summed over every dispatch between the
last two lds_poison_kernel dispatches (the update: its graph replays, the eager kernels, the
optimizer and the KL re-forward), with a per-kernel breakdown."""

from __future__ import annotations

import collections
import csv
import json
import sys
from pathlib import Path


def between_markers(path: Path, counter: str):
    rows = []
    for f in path.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    marks = [i for i, (_, k, _) in enumerate(rows) if k.startswith("lds_poison_kernel")]
    if len(marks) < 2:
        raise SystemExit(f"{path}: {len(marks)} marker dispatches (need 2)")
    a, b = marks[-2], marks[-1]
    per = collections.defaultdict(lambda: [0, 0.0])
    for _, k, v in rows[a + 1:b]:
        name = k.split("(")[0].split("<")[0].strip()
        per[name][0] += 1
        per[name][1] += v
    return per


def main(src: str, dst: str):
    s = Path(src)
    fetch, write = between_markers(s / "fetch", "FETCH_SIZE"), between_markers(s / "write", "WRITE_SIZE")
    info = {}
    for line in (s / "fetch.log").read_text().splitlines():
        if line.startswith("URM_UPDATE_PMC "):
            info = json.loads(line[len("URM_UPDATE_PMC "):])
    kernels = {}
    total = 0.0
    for k in sorted(set(fetch) | set(write)):
        n = max(fetch.get(k, [0])[0], write.get(k, [0])[0])
        b = (2 * fetch.get(k, [0, 0.0])[1] + write.get(k, [0, 0.0])[1]) * 1024
        kernels[k] = {"dispatches": n, "hbm_bytes": b}
        total += b
    top = dict(sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes"]))
    out = {"bytes_per_update": total, "dispatches": sum(v["dispatches"] for v in kernels.values()), **info,
           "kernels": top,
           "basis": "HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE per dispatch (gfx950 FETCH correction), summed over "
                    "every dispatch of one GameURM update (between tools/urm_update_pmc.py's markers)",
           "source": f"{src} (tools/gpu/check.sh urmhbm)"}
    Path(dst).parent.mkdir(parents=True, exist_ok=True)
    Path(dst).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps({"bytes_per_update": total, **info}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
