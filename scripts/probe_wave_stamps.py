#!/usr/bin/env python3
"""Where the bulk kernel's fixed cost goes (probe, not product code).  Needs a diagnostic build:
  scripts/build_variant.sh stamps WT -DHF3FS_CRC_WAVE_STAMPS
  HF3FS_CRC_LIB=$PWD/3fs_amd/lib/ab/stamps.so python scripts/probe_wave_stamps.py
Runs create_strided over n x 4 MiB (bench.py's kernel path; WS_CASES=n:seg_kib,... with
option seg_kib forcing segment tasks) and reads every wave's wall clock
at entry, after the LDS tables and at exit; prints, relative to the first wave's entry, the
launch ramp (last entry), the table fill, and the spread of the exits, with the event time."""
import importlib
import json
import os
import statistics
import sys
import ctypes

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
hf = importlib.import_module("3fs_amd")
L = hf._lib
lib = L.load()
from bench_suite import warm_gpu  # noqa: E402

fn = lib.hf3fs_crc_debug_wave_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int)]
dev = torch.device("cuda:0")
s = torch.cuda.current_stream()
CH = 4 << 20
buf = torch.empty(4096 * CH, dtype=torch.uint8, device=dev)
L.fill_synth(buf, CH, CH, 4096, 0x3F5C3C00, 0, stream=s)
out = torch.zeros(4096, dtype=torch.int32, device=dev)
nw = torch.cuda.get_device_properties(0).multi_processor_count * 16
host = np.zeros(4 * nw, dtype=np.uint64)
khz = ctypes.c_int(0)
for n, seg in [(int(x), int(y)) for x, y in (c.split(":") for c in os.environ.get("WS_CASES", "4096:0,1024:0").split(","))]:
    L.set_option("seg_kib", str(seg))  # 0: whole-buffer tasks (the default plan for 4 MiB chunks)
    for rep in range(4):
        warm_gpu(0.05)
        L.create_strided(hf.CRC32C, buf, CH, CH, n, out, stream=s)  # back to back: the second is stamped
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        L.create_strided(hf.CRC32C, buf, CH, CH, n, out, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        assert fn(host.ctypes.data, 4 * nw, ctypes.byref(khz)) == 0
        st = host.reshape(nw, 4).astype(np.int64)
        busy = np.arange(nw) < n * max(1, (CH >> 10) // seg if seg else 1)  # waves with a first task
        t0 = st[:, 0].min()
        us = lambda v: round(float(v - t0) * 1e3 / khz.value, 1)  # noqa: E731
        ends = np.sort(st[busy, 2])
        fill = (st[:, 1] - st[:, 0]) * 1e3 / khz.value
        print(json.dumps({"probe": "wave_stamps", "chunks": n, "seg_kib": seg, "rep": rep, "event_ms": round(a.elapsed_time(b), 4),
                          "waves": int(nw), "busy_waves": int(busy.sum()), "last_entry_us": us(st[:, 0].max()),
                          "table_fill_us_p50": round(float(np.median(fill)), 2),
                          "table_fill_us_max": round(float(fill.max()), 2),
                          "first_exit_us": us(ends[0]), "p10_exit_us": us(ends[len(ends) // 10]),
                          "p50_exit_us": us(ends[len(ends) // 2]), "p90_exit_us": us(ends[len(ends) * 9 // 10]),
                          "p99_exit_us": us(ends[len(ends) * 99 // 100]), "last_exit_us": us(ends[-1])}), flush=True)
        if rep == 0:  # exits by XCD (workgroups are dealt to the 8 XCDs round robin) and by wave slot
            wg = np.arange(nw) // 16
            ex = (st[:, 2] - t0) * 1e3 / khz.value
            print(json.dumps({"probe": "wave_stamps_xcd", "chunks": n, "seg_kib": seg,
                              "xcd_mean_exit_us": [round(float(ex[busy & (wg % 8 == x)].mean()), 1) for x in range(8)],
                              "xcd_max_exit_us": [round(float(ex[busy & (wg % 8 == x)].max()), 1) for x in range(8)],
                              "slot_mean_exit_us": [round(float(ex[busy & (np.arange(nw) % 16 == k)].mean()), 1)
                                                    for k in range(16)]}), flush=True)
            np.save(f"gpurun_out/wave_stamps_{n}_{seg}.npy", st)
