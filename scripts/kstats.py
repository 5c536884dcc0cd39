#!/usr/bin/env python3
"""Short per-kernel table of a rocprofv3 --stats run: kstats.py DIR [top]."""
import csv
import glob
import re
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for r in rows[:top]:
    name = r["Name"].replace("(anonymous namespace)::", "").replace("hf3fs_crc::", "").replace("void ", "", 1)
    name = re.sub(r"\(.*", "", name)
    print(f'{name[:70]:70s} calls {int(r["Calls"]):6d} avg_us {float(r["AverageNs"]) / 1e3:9.1f} pct {float(r["Percentage"]):5.1f}')
