"""Generate the full-size golden digest tables of the bulk configs.

BASELINE configs[1] ("bulk write path", the default): 4 MiB chunks of the
splitmix64 synthetic stream (seed 0x3F5C3C00), chunk ids
0 .. 32767 -- 4096 chunks for each of up to 8 GPUs, rank r owning ids
[4096 r, 4096 (r+1)).
BASELINE configs[3] ("node scale", --chunk-mib 64 --chunks 1024 --per-gpu 128):
64 MiB chunks, ids 0 .. 1023 -- the node's 64 GiB, 128 chunks per GPU of 8.
Every digest is ChecksumInfo::create(CRC32C, chunk, chunk size).value (folly raw
register, start ~0) from the C oracle's SSE4.2 restatement; every 64th chunk is
re-hashed with the oracle's independent slicing-by-8 table form.

Outputs (data only; the GPU tests and bench.py read them, nothing here runs on
the GPU box):
  bulk_<M>MiB_digests.bin   N x uint32 little-endian
  bulk_<M>MiB_digests.json  seed, sizes, sha256 of the .bin, and two
                          size-independent pins of the first per-GPU chunks:
                          raw CRC32C of the digest table's bytes, and the raw
                          CRC32C of those chunks as ONE buffer
                          (ChecksumInfo::combine fold, Common.h:179-198).
Run:  python tests/golden/make_bulk_golden.py   (about 30 s on 8 cores)
      python tests/golden/make_bulk_golden.py --chunk-mib 64 --chunks 1024 --per-gpu 128   (about 30 s)
"""
import argparse
import hashlib
import json
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402  (test infrastructure)

SEED = 0x3F5C3C00
CHUNK = 4 << 20
PER_GPU = 4096
N = 8 * PER_GPU


def _init(chunk):
    global CHUNK
    CHUNK = chunk


def digest(i):
    d = oracle.fill_synth(CHUNK, SEED, i)
    v = oracle.crc32c_raw(d)
    if i % 64 == 0:
        assert oracle.crc32c_raw(d, kind="sw") == v, i
    return v


def main():
    global CHUNK, PER_GPU, N
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk-mib", type=int, default=4)
    ap.add_argument("--chunks", type=int, default=N)
    ap.add_argument("--per-gpu", type=int, default=PER_GPU)
    a = ap.parse_args()
    CHUNK, N, PER_GPU = a.chunk_mib << 20, a.chunks, a.per_gpu
    with Pool(min(8, os.cpu_count() or 1), initializer=_init, initargs=(CHUNK,)) as p:
        vals = np.array(p.map(digest, range(N), chunksize=max(1, min(64, N // 64))), dtype="<u4")
    raw = vals.tobytes()
    acc = (oracle.CRC32C, int(vals[0]))
    for i in range(1, PER_GPU):
        rc, acc = oracle.combine(acc, (oracle.CRC32C, int(vals[i])), CHUNK)
        assert rc == 0
    meta = {
        "seed": SEED,
        "chunk_bytes": CHUNK,
        "chunks": N,
        "chunks_per_gpu": PER_GPU,
        "sha256": hashlib.sha256(raw).hexdigest(),
        f"table_crc32c_raw_first_{PER_GPU}": oracle.crc32c_raw(np.frombuffer(raw[:4 * PER_GPU], dtype=np.uint8)),
        f"whole_batch_crc32c_raw_first_{PER_GPU}": acc[1],
        "generator": "tests/golden/make_bulk_golden.py (oracle/crc_oracle.c, SSE4.2 + slicing-by-8 cross-check)",
    }
    name = f"bulk_{a.chunk_mib}MiB_digests"
    with open(os.path.join(HERE, name + ".bin"), "wb") as f:
        f.write(raw)
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
