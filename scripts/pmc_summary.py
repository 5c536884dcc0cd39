"""Mean per-dispatch PMC values per kernel from rocprofv3 counter_collection.csv files under a directory."""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(f) as fh:
        for r in csv.DictReader(fh):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            name = m.group(1) if m else r["Kernel_Name"][:40]
            acc[name][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print("==", f)
    for name, d in acc.items():
        per = collections.defaultdict(list)
        for (disp, c), vals in d.items():
            per[c].append(sum(vals))
        print(f"  {name}: " + " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(per.items())))
