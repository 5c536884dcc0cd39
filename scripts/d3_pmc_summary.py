"""Per-batch HBM traffic of the d3 DELTA leg (tests/bench_suite.py d3) from rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE passes, against the algorithmic bytes of the same seeded
plan.  FETCH_SIZE is doubled per the gfx950 correction (MI355X_MICROARCH.md, HBM).
usage: python scripts/d3_pmc_summary.py FETCH_DIR WRITE_DIR [TRACE_DIR] > profiles/r03_d3_pmc.json"""
import collections
import csv
import glob
import json
import re
import sys

import numpy as np


def plan(n=4096, chunk=4 << 20, batches=8):
    rng = np.random.default_rng(3)  # the same draws as tests/bench_suite.py::_d3_run
    sizes = rng.integers(2 << 20, chunk + 1, n).astype(np.int64)
    out = []
    for _ in range(batches):
        lens = rng.integers(64 << 10, (1 << 20) + 1, n)
        offs = np.array([rng.integers(0, chunk - ln + 1) for ln in lens])
        r = rng.random(n)
        app = (r < 0.10) & (sizes + lens <= chunk)
        offs[app] = sizes[app]
        gap = (r >= 0.10) & (r < 0.15) & (sizes + lens + 4096 <= chunk)
        offs[gap] = sizes[gap] + rng.integers(1, 4097, gap.sum())
        old = np.clip(np.minimum(offs + lens, sizes) - offs, 0, None)
        gapb = np.clip(offs - sizes, 0, None)
        out.append({"payload": int(lens.sum()), "old": int(old.sum()), "gap": int(gapb.sum())})
        sizes = np.maximum(sizes, offs + lens)
    return out


def per_dispatch(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        k = m.group(1) if m else "other"
        key = (int(r["Dispatch_Id"]), k)
        acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"]) * 1024  # KB -> bytes
    return sorted(acc.items())


def batches_of(rows):
    """(pre hash, apply) per update batch: the k_crc_ranges dispatch right before each apply."""
    out, prev = [], None
    for (d, k), v in rows:
        if k == "k_update_apply" and prev is not None:
            out.append((prev, v))
        prev = v if k == "k_crc_ranges" else prev
    return out


def main():
    fetch, write = per_dispatch(sys.argv[1]), per_dispatch(sys.argv[2])
    bf, bw = batches_of(fetch), batches_of(write)
    p = plan()  # batch 0 is the untimed warm-up; all 8 are profiled
    rows = []
    for i, ((hf, af), (hw, aw)) in enumerate(zip(bf, bw)):
        a = p[i]
        pre_alg = a["payload"] + a["old"]
        app_alg_r, app_alg_w = a["payload"], a["payload"] + a["gap"]
        rows.append({"batch": i, "pre_hash": {"fetch": 2 * hf, "write": hw, "algorithmic_read": pre_alg,
                                              "read_ratio": round(2 * hf / pre_alg, 4)},
                     "apply": {"fetch": 2 * af, "write": aw, "algorithmic_read": app_alg_r,
                               "algorithmic_write": app_alg_w, "read_ratio": round(2 * af / app_alg_r, 4),
                               "write_ratio": round(aw / app_alg_w, 4)}})
    res = {"round": "r03", "config": "d3 DELTA, tests/bench_suite.py d3 (D3_MODES=delta D3_AB=0)",
           "note": "FETCH_SIZE x2 (gfx950 correction), separate --pmc passes; algorithmic bytes from the seeded plan",
           "batches": rows,
           "mean": {f"{s}_{k}": round(float(np.mean([r[s][k] for r in rows])), 4) for s, k in
                    [("pre_hash", "read_ratio"), ("apply", "read_ratio"), ("apply", "write_ratio")]}}
    if len(sys.argv) > 3:
        tr = glob.glob(f"{sys.argv[3]}/**/*kernel_trace.csv", recursive=True)[0]
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(tr)):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            if m:
                dur[m.group(1)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        ap = [d for _, d in sorted(dur["k_update_apply"])]
        res["apply_us"] = [round(x / 1e3, 1) for x in ap]
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
