#!/usr/bin/env python3
"""Device-to-device copy ceiling of this box (probe, not product code): hipMemcpyAsync
(runtime blit) and torch copy_ of 0.6-2.3 GB, read + write bytes / time (the d3 apply
moves 2.29 GB read + 2.29 GB write per batch at ~5.0 TB/s)."""
import json

import torch

dev = torch.device("cuda:0")
for gb in (0.6, 1.2, 2.29):
    n = int(gb * 1e9) // 16 * 16
    a = torch.empty(n, dtype=torch.uint8, device=dev).fill_(7)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    for name in ("torch_copy", "float4_copy"):
        def run():
            if name == "torch_copy":
                b.copy_(a)
            else:
                b.view(torch.float32).copy_(a.view(torch.float32))
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(json.dumps({"probe": "d2d", "copy": name, "gb": gb, "ms": round(ms, 4),
                          "tbs_read_plus_write": round(2 * n / ms / 1e9, 3)}), flush=True)
    del a, b
    torch.cuda.empty_cache()
