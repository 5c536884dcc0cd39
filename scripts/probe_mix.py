#!/usr/bin/env python3
"""HBM read/write mix probe (scripts/probe_mix.hip): the d3 DELTA byte volumes scheduled
two ways, without hashing --
  now:  pass 1 reads payload + old bytes (3.96 GB, pure reads), pass 2 copies the payload
        (2.29 GB read + 2.29 GB written);
  alt:  pass 1 reads the payload (2.29 GB), pass 2 copies it and reads the old bytes along
        (3.96 GB read + 2.29 GB written).
Prints one JSON line per measurement (median of interleaved rounds, HIP events)."""
import ctypes
import json
import os
import statistics
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "..", "3fs_amd", "lib", "ab", "probe_mix.so")
if not os.path.exists(SO):
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                           os.path.join(HERE, "probe_mix.hip"), "-o", SO])
lib = ctypes.CDLL(SO)
V, U64, U32, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
lib.probe_read.argtypes = [V, U64, V, U32, V]
lib.probe_copy.argtypes = [V, V, U64, U32, I, V]
lib.probe_copy_r.argtypes = [V, V, U64, V, U64, V, U32, I, V]

PAY, OLD = 2_285_386_082 & ~15, 1_673_985_060 & ~15  # the d3 batch's payload / old bytes
dev = torch.device("cuda:0")
A = torch.randint(0, 255, (PAY,), dtype=torch.uint8, device=dev)
B = torch.randint(0, 255, (OLD,), dtype=torch.uint8, device=dev)
C = torch.empty(PAY, dtype=torch.uint8, device=dev)
sink = torch.zeros(4, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
sp = s.cuda_stream
grid = int(os.environ.get("PROBE_GRID", 4096))
nts = int(os.environ.get("PROBE_NTS", 1))

legs = {
    "read_pay": lambda: lib.probe_read(A.data_ptr(), PAY, sink.data_ptr(), grid, sp),
    "read_old": lambda: lib.probe_read(B.data_ptr(), OLD, sink.data_ptr(), grid, sp),
    "copy_pay": lambda: lib.probe_copy(A.data_ptr(), C.data_ptr(), PAY, grid, nts, sp),
    "copy_pay_read_old": lambda: lib.probe_copy_r(A.data_ptr(), C.data_ptr(), PAY, B.data_ptr(), OLD,
                                                  sink.data_ptr(), grid, nts, sp),
}
vol = {"read_pay": PAY, "read_old": OLD, "copy_pay": 2 * PAY, "copy_pay_read_old": 2 * PAY + OLD}
res = {k: [] for k in legs}
for rnd in range(8):
    for k, f in (legs.items() if rnd % 2 == 0 else reversed(list(legs.items()))):
        f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            assert f() == 0
        e1.record(s)
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 3)
med = {k: statistics.median(v) for k, v in res.items()}
for k in legs:
    print(json.dumps({"probe": "mix", "leg": k, "grid": grid, "nts": nts, "ms": round(med[k], 4),
                      "tbs": round(vol[k] / med[k] / 1e9, 3)}))
now = med["read_pay"] + med["read_old"] + med["copy_pay"]
alt = med["read_pay"] + med["copy_pay_read_old"]
print(json.dumps({"probe": "mix", "schedule_now_ms": round(now, 4), "schedule_alt_ms": round(alt, 4),
                  "alt_over_now": round(alt / now, 4)}))
sys.stdout.flush()
