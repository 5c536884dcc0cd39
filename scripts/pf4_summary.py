"""Per-kernel mean durations of the f4 profiles under gpurun_out/pf4 (rocprofv3 SQLite output)."""
import glob
import sqlite3
import sys

for d in sorted(glob.glob("gpurun_out/pf4/*/")):
    dbs = glob.glob(d + "**/*.db", recursive=True)
    if not dbs:
        continue
    con = sqlite3.connect(dbs[0])
    rows = con.execute("select name, count(*), avg(end-start)/1000.0 from kernels where name like '%frame%' "
                       "or name like '%k_crc_ranges%' group by name").fetchall()
    out = []
    for name, cnt, us in rows:
        import re
        short = re.search(r"(k_\w+)", name).group(1)
        out.append(f"{short}={us:.1f}")
    print(d.split("/")[-2], " ".join(out))
