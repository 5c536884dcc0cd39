"""Generate tests/golden/golden.json -- parity vectors for the CRC32C/CRC32 path.

Independent of both the C oracle and the HIP library: a byte-table CRC built
bit by bit in pure Python, a pure-Python splitmix64 generator, and zero-byte
feeding for combine (no GF(2) multiplication), so the oracle and the product
are each checked against code that shares nothing with them.

Pins from the reference (no folly/Rust build exists here):
  * tests/common/utils/TestFolly.cc:11-18  combine(crc(hello,0), crc(world,0), 5)
                                            == crc32c(world, 5, crc(hello,0))
  * tests/common/utils/TestFolly.cc:20-21  CRC-32C(1 MiB zeros) = 0x14298C12,
                                            CRC-32C(one zero byte) = 0x527D5351
  * RFC 3720 check value CRC-32C("123456789") = 0xE3069283
  * zlib.crc32 (IEEE) for ChecksumType::CRC32: folly::crc32(d, n, ~0) == ~zlib.crc32(d)
Run:  python tests/golden/make_golden.py   (about 10 s)
"""
import hashlib
import json
import os
import zlib

POLY_C = 0x82F63B78
POLY_I = 0xEDB88320
M32 = 0xFFFFFFFF
SEED = 0x3F5C3C00


def table(poly):
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        t.append(c)
    return t


TC, TI = table(POLY_C), table(POLY_I)


def crc_raw(data, start, t):
    c = start
    for b in data:
        c = (c >> 8) ^ t[(c ^ b) & 0xFF]
    return c


def splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def synth(n, seed, chunk_id, byte_off=0):
    """splitmix64(seed ^ (chunk_id << 32) ^ word_index), little-endian words."""
    key = seed ^ (chunk_id << 32)
    first_w, last_w = byte_off // 8, (byte_off + n + 7) // 8
    raw = b"".join(splitmix64(key ^ w).to_bytes(8, "little") for w in range(first_w, last_w))
    s = byte_off - first_w * 8
    return raw[s:s + n]


LENGTHS = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 63, 64, 65, 255, 256, 257, 1000, 1023, 1024, 1025, 2047, 2048,
           3072, 4095, 4096, 4097, 8191, 12345, 65535, 65536, 65537, 131075, 524288]


def main():
    out = {"seed": SEED, "poly_crc32c": POLY_C, "poly_crc32": POLY_I, "kat": {}, "synth": [], "combine": [],
           "strings": []}
    kat = out["kat"]
    kat["crc32c_123456789_fin"] = (~crc_raw(b"123456789", M32, TC)) & M32
    kat["crc32c_1MiB_zeros_fin"] = (~crc_raw(bytes(1 << 20), M32, TC)) & M32
    kat["crc32c_one_zero_fin"] = (~crc_raw(bytes(1), M32, TC)) & M32
    kat["crc32_123456789_fin"] = (~crc_raw(b"123456789", M32, TI)) & M32
    assert kat["crc32c_123456789_fin"] == 0xE3069283
    assert kat["crc32c_1MiB_zeros_fin"] == 0x14298C12
    assert kat["crc32c_one_zero_fin"] == 0x527D5351
    assert kat["crc32_123456789_fin"] == zlib.crc32(b"123456789")
    h0 = crc_raw(b"hello", 0, TC)
    w0 = crc_raw(b"world", 0, TC)
    kat["hello_world"] = {"crc_hello_0": h0, "crc_world_0": w0, "continued": crc_raw(b"world", h0, TC)}

    for s in [b"", b"a", b"abc", b"123456789", b"hello world", b"etc", b"zzz", b"etczzz", bytes(range(256))]:
        out["strings"].append({"hex": s.hex(), "crc32c_raw": crc_raw(s, M32, TC), "crc32_raw": crc_raw(s, M32, TI),
                               "crc32c_raw_start0": crc_raw(s, 0, TC)})

    for k, n in enumerate(LENGTHS):
        for off in ([0, 3] if n < 70000 else [0]):
            d = synth(n, SEED, k, off)
            assert (~crc_raw(d, M32, TI)) & M32 == zlib.crc32(d)
            out["synth"].append({
                "chunk_id": k, "byte_off": off, "len": n, "sha256": hashlib.sha256(d).hexdigest(),
                "crc32c_raw": crc_raw(d, M32, TC), "crc32c_raw_start0": crc_raw(d, 0, TC),
                "crc32c_raw_start_custom": crc_raw(d, 0x12345678, TC), "crc32_raw": crc_raw(d, M32, TI)})

    # combine(c1, c2, len2) = crc of c1 fed len2 zero bytes, xor c2 -- computed by feeding zeros
    for k, (c1, c2, n) in enumerate([(0x12345678, 0x9ABCDEF0, 0), (0x12345678, 0x9ABCDEF0, 1), (M32, 0, 3),
                                     (0xDEADBEEF, 0x0BADF00D, 4), (1, 2, 5), (0x80000000, 0, 1023),
                                     (0xCAFEBABE, 0x11111111, 1024), (0x55555555, 0xAAAAAAAA, 4096 + 17),
                                     (0x13579BDF, 0x2468ACE0, 65536 + 5), (0xFFFF0000, 0x0000FFFF, 100003)]):
        z = bytes(n)
        out["combine"].append({"c1": c1, "c2": c2, "len2": n,
                               "crc32c": crc_raw(z, c1, TC) ^ c2, "crc32": crc_raw(z, c1, TI) ^ c2})

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(path, len(out["synth"]), "synth vectors")


if __name__ == "__main__":
    main()
