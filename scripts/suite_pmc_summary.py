#!/usr/bin/env python3
"""Per-kernel HBM traffic per suite config from scripts/suite_pmc.sh (gpurun_out/spmc):
mean FETCH_SIZE and WRITE_SIZE per dispatch (KB, each from its own pass) and the corrected
traffic 2 x FETCH + WRITE in bytes (MI355X_MICROARCH.md: FETCH_SIZE counts half of a wide
coalesced read stream on gfx950)."""
import collections
import csv
import glob
import json
import os
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/spmc"
for cfg in sorted(os.listdir(root)):
    d = os.path.join(root, cfg)
    if not os.path.isdir(d):
        continue
    per = collections.defaultdict(dict)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for f in glob.glob(os.path.join(d, c, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                m = re.search(r"(k_\w+)", r["Kernel_Name"])
                name = m.group(1) if m else r["Kernel_Name"][:40]
                if "ListSource" in r["Kernel_Name"]:
                    name += "<List>"
                elif "StridedSource" in r["Kernel_Name"]:
                    name += "<Strided>"
                acc[name][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for name, disp in acc.items():
            v = list(disp.values())
            per[name][c] = (len(v), sum(v) / len(v))
    rows = []
    for name, cs in per.items():
        n, fk = cs.get("FETCH_SIZE", (0, 0.0))
        _, wk = cs.get("WRITE_SIZE", (0, 0.0))
        rows.append({"config": cfg, "kernel": name, "dispatches": n, "fetch_kb": round(fk, 1), "write_kb": round(wk, 1),
                     "traffic_bytes": int(2 * fk * 1024 + wk * 1024)})
    for r in sorted(rows, key=lambda x: -x["traffic_bytes"])[:6]:
        print(json.dumps(r))
