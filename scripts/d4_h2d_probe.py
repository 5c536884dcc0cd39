#!/usr/bin/env python3
"""d4 streamed-H2D probe: why did the suite's pinned-host leg fall
50 -> 39 GB/s while bench.py's ring gives 52?  Same process, same pinned buffer; each
line is one variant of the ring (pieces of 64 MiB copied H2D on `slots` streams, each
piece hashed on its stream after its copy):

  copy_only      the copies alone (PCIe + DMA engine ceiling of this ring)
  ring           copy + hf3fs_crc_create_strided of the piece (the suite's / bench's ring)
  ring_after_big the same after a 64 GiB HBM buffer was allocated, used and freed in this
                 process (the suite runs d4's HBM leg first)
  zero_copy      the kernel reads the mapped pinned pages (no DMA)
Prints one JSON line per variant.  Not product code."""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
hf = importlib.import_module("3fs_amd")
L = hf._lib
SEED = 0x3F5C3C00
CHUNK = 64 << 20


def ring(host, nchunks, slots, hash_it, steps=2):
    dev = torch.device("cuda:0")
    bufs = [torch.empty(CHUNK, dtype=torch.uint8, device=dev) for _ in range(slots)]
    streams = [torch.cuda.Stream() for _ in range(slots)]
    out = torch.zeros(nchunks, dtype=torch.int32, device=dev)

    def one():
        for i in range(nchunks):
            k = i % slots
            with torch.cuda.stream(streams[k]):
                bufs[k].copy_(host[i * CHUNK:(i + 1) * CHUNK], non_blocking=True)
                if hash_it:
                    L.create_strided(hf.CRC32C, bufs[k], CHUNK, CHUNK, 1, out[i:i + 1], stream=streams[k])

    one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    return nchunks * CHUNK * steps / (time.perf_counter() - t0) / 1e9, out


def main():
    L.load()
    dev = torch.device("cuda:0")
    nchunks = int(os.environ.get("H2D_CHUNKS", "32"))
    host = torch.empty(nchunks * CHUNK, dtype=torch.uint8, pin_memory=True)
    src = torch.empty(nchunks * CHUNK, dtype=torch.uint8, device=dev)
    L.fill_synth(src, CHUNK, CHUNK, nchunks, SEED, 0, stream=torch.cuda.current_stream())
    host.copy_(src)
    del src
    torch.cuda.synchronize()
    golden = np.fromfile(os.path.join(REPO, "tests", "golden", "bulk_64MiB_digests.bin"), dtype="<u4")[:nchunks]

    def emit(name, gbs, out=None, **kw):
        ok = None if out is None else bool(np.array_equal(out.cpu().numpy().astype(np.uint32), golden))
        print(json.dumps({"variant": name, "gbs": round(gbs, 2), "chunks": nchunks, "bit_exact": ok, **kw}), flush=True)

    for slots in (4, 2, 8):
        g, _ = ring(host, nchunks, slots, False)
        emit("copy_only", g, slots=slots)
        g, out = ring(host, nchunks, slots, True)
        emit("ring", g, out, slots=slots)
    big = torch.empty(1024 * CHUNK, dtype=torch.uint8, device=dev)  # 64 GiB, as the suite's HBM leg
    L.fill_synth(big, CHUNK, CHUNK, 1024, SEED, 0, stream=torch.cuda.current_stream())
    o = torch.zeros(1024, dtype=torch.int32, device=dev)
    L.create_strided(hf.CRC32C, big, CHUNK, CHUNK, 1024, o, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    del big, o
    torch.cuda.empty_cache()
    g, out = ring(host, nchunks, 4, True)
    emit("ring_after_big", g, out, slots=4)
    hip = ctypes.CDLL("libamdhip64.so")
    dptr = ctypes.c_void_p()
    if hip.hipHostGetDevicePointer(ctypes.byref(dptr), ctypes.c_void_p(host.data_ptr()), 0) == 0:
        zc = torch.zeros(nchunks, dtype=torch.int32, device=dev)
        s = torch.cuda.current_stream()
        L.create_strided(hf.CRC32C, dptr.value, CHUNK, CHUNK, nchunks, zc, stream=s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            L.create_strided(hf.CRC32C, dptr.value, CHUNK, CHUNK, nchunks, zc, stream=s)
        torch.cuda.synchronize()
        emit("zero_copy", nchunks * CHUNK * 2 / (time.perf_counter() - t0) / 1e9, zc)


if __name__ == "__main__":
    main()
