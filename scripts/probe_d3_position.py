#!/usr/bin/env python3
"""d3 DELTA run three times in one process (probe, not product code): is the first run of a
process slower than the later ones (the suite runs the default pipeline first)?"""
import os, sys, json
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import bench_suite as B
import torch
s = torch.cuda.current_stream()
for i in range(3):
    r = B._d3_run(4096, 4 << 20, 8, B.hf.MODE_DELTA, "delta", s)
    print(json.dumps({"run": i, "ms_per_batch": r["ms_per_batch"], "bit_exact": r["bit_exact"]}), flush=True)
