#!/usr/bin/env python3
"""Summarise a gpu_profile.sh run (gpurun_out/prof) into profiles/<round>_*.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads
exactly half of a wide coalesced stream on gfx950, so traffic =
2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024, each from its own --pmc pass.
Usage: python scripts/parse_prof.py r01 [kernel-substring]
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "gpurun_out", "prof")


def counter(name, kernel):
    path = os.path.join(PROF, name, "run_counter_collection.csv")
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    return vals


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    # the bulk launch: whole-buffer (DIRECT) tasks over the strided 4096 x 4 MiB batch
    kernel = sys.argv[2] if len(sys.argv) > 2 else "k_crc_ranges<2197175160u, true, true, hf3fs_crc::StridedSource>"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20  # bench.py's timed launches (the last ones)
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    stats_src = os.path.join(PROF, "trace", "run_kernel_stats.csv")
    shutil.copy(stats_src, os.path.join(REPO, "profiles", f"{rnd}_bulk_kernel_stats.csv"))
    rows = [r for r in csv.DictReader(open(os.path.join(PROF, "trace", "run_kernel_trace.csv")))
            if kernel in r["Kernel_Name"]]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    timed = durs[-steps:]
    fetch = counter("fetch", kernel)
    write = counter("write", kernel)
    fetch_b = 2 * statistics.mean(fetch) * 1024
    write_b = statistics.mean(write) * 1024
    algo = 4096 * (4 << 20)
    out = {
        "round": rnd,
        "kernel": rows[0]["Kernel_Name"] if rows else kernel,
        "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py (defaults: --steps 20 --warmup 3); "
                   "PMC: separate --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --steps 3 --warmup 1",
        "launches": len(durs),
        "kernel_ms_mean": round(statistics.mean(durs), 4),
        "kernel_ms_min": round(min(durs), 4),
        "kernel_ms_median": round(statistics.median(durs), 4),
        "kernel_ms_mean_timed": round(statistics.mean(timed), 4),
        "timed_launches": len(timed),
        "fetch_size_kb_per_launch": statistics.mean(fetch),
        "write_size_kb_per_launch": statistics.mean(write),
        "hbm_read_bytes_per_launch": int(fetch_b),
        "hbm_write_bytes_per_launch": int(write_b),
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": round((fetch_b + write_b) / algo, 5),
        "achieved_gbs_at_profiled_mean": round(algo / (statistics.mean(durs) / 1e3) / 1e9, 1),
        "achieved_gbs_at_profiled_timed_mean": round(algo / (statistics.mean(timed) / 1e3) / 1e9, 1),
        "frac_at_profiled_timed_mean": round(algo / (statistics.mean(timed) / 1e3) / 1e9 / 8000.0, 4),
        "note": "FETCH_SIZE doubled per the gfx950 correction (MI355X_MICROARCH.md §HBM); separate --pmc passes",
    }
    # the bench line the profiled run itself printed (same process as the trace)
    line = None
    for ln in open(os.path.join(PROF, "trace.log"), errors="replace"):
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    if line:
        rf = line["roofline"]
        out["profiled_run_line"] = {"value": line["value"], "ms_per_step": line["ms_per_step"],
                                    "launch_ms_mean_hip_events": rf["launch_ms_mean"], "frac": rf["frac"],
                                    "bit_exact": line["bit_exact"]}
        out["trace_timed_mean_le_ms_per_step"] = out["kernel_ms_mean_timed"] <= line["ms_per_step"]
    with open(os.path.join(REPO, "profiles", f"{rnd}_bulk_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    with open(os.path.join(REPO, "profiles", "pmc_bulk_4096x4MiB.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
