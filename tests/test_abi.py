"""C-ABI checks that need no GPU: the HIP library loads, exports every symbol
include/hf3fs_crc.h declares, and its host-side scalar algebra (combine/shift,
ChecksumInfo::combine) agrees with the oracle and the golden vectors."""
import ctypes
import os
import subprocess

import pytest

M32 = 0xFFFFFFFF


def test_library_exports_header(hf):
    lib = hf._lib.load()
    declared = hf._lib.header_symbols()
    assert len(declared) >= 17
    out = subprocess.check_output(["nm", "-D", "--defined-only", hf._lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    for s in declared:
        assert hasattr(lib, s)
        assert s in hf._lib.SIGNATURES, f"no ctypes signature for {s}"


def test_update_io_layout(hf):
    assert ctypes.sizeof(hf.UpdateIO) == 56
    assert hf.UpdateIO.status.offset == 52
    assert hf.UpdateIO.out_checksum.offset == 44


def test_version(hf):
    assert b"gfx950" in hf._lib.load().hf3fs_crc_version()


def test_scalar_combine_golden(hf, golden):
    for v in golden["combine"]:
        assert hf._lib.crc32c_combine(v["c1"], v["c2"], v["len2"]) == v["crc32c"]
        assert hf._lib.crc32_combine(v["c1"], v["c2"], v["len2"]) == v["crc32"]
    kat = golden["kat"]["hello_world"]
    assert hf._lib.crc32c_combine(kat["crc_hello_0"], kat["crc_world_0"], 5) == kat["continued"]


def test_shift_matches_oracle(hf, orc):
    for n in [0, 1, 3, 4, 1000, 1 << 20, (1 << 26) + 5, (1 << 33) + 7]:
        for c in [1, 0x80000000, 0xDEADBEEF]:
            assert hf._lib.shift(1, c, n) == orc.shift(c, n, orc.POLY_CRC32C)
            assert hf._lib.shift(2, c, n) == orc.shift(c, n, orc.POLY_CRC32)


@pytest.mark.parametrize("a,b,length", [((1, 5), (2, 6), 10), ((0, 0), (1, 7), 0), ((1, 9), (1, 7), 0),
                                        ((0, 0), (1, 7), 3), ((1, 0x1234), (1, 0x9876), 77777),
                                        ((2, 0x1234), (2, 0x9876), 5)])
def test_checksum_combine_semantics(hf, orc, a, b, length):
    assert hf._lib.checksum_combine(a, b, length) == orc.combine(a, b, length)


def test_python_checksuminfo_formatter(hf):
    ci = hf.ChecksumInfo(hf.ChecksumType.CRC32C, 0x1CF96D7C)
    assert str(ci) == "CRC32C#E3069283"  # formatter prints ~value (Common.h:768-773)
    o = hf.ChecksumInfo(hf.ChecksumType.CRC32, 1)
    assert ci.combine(o, 5) == 4080
    assert ci.combine(o, 0) == 4080  # type check happens before the length check


def test_build_is_incremental():
    import importlib
    b = importlib.import_module("3fs_amd.build")
    assert b.build() == b.LIB  # up to date: no rebuild needed


def test_checksuminfo_serde_form(hf):
    """TestCommonStruct.cc:46-55: serialize({CRC32, 0xff}) is 1 + 1 + 4 bytes and
    deserializes to an equal value.  The byte order restates serde's binary Out
    (Serde.h:282-290, 422-432): the table's varint length, then type, then value LE."""
    ser = hf.ChecksumInfo(hf.ChecksumType.CRC32, 0xFF)
    out = ser.serialize()
    assert len(out) == 1 + 1 + 4
    assert out == bytes([5, 2, 0xFF, 0, 0, 0])
    rc, des = hf.ChecksumInfo.deserialize(out)
    assert rc == 0 and des == ser
    for t, v in [(0, 0), (1, 0x1CF96D7C), (2, 0xFFFFFFFF), (1, 0)]:
        rc, des = hf.ChecksumInfo.deserialize(hf.ChecksumInfo(hf.ChecksumType(t), v).serialize())
        assert rc == 0 and (int(des.type), des.value) == (t, v)


def test_checksuminfo_serde_edges(hf):
    L = hf._lib
    assert L.checksum_deserialize(b"") == (L.SERDE_INSUFFICIENT_LENGTH, (0, 0), 0)  # no length varint
    assert L.checksum_deserialize(bytes([5, 1, 2, 3]))[0] == L.SERDE_INSUFFICIENT_LENGTH  # table cut short
    assert L.checksum_deserialize(bytes([3, 1, 2, 3]))[0] == L.SERDE_INSUFFICIENT_LENGTH  # value field cut short
    assert L.checksum_deserialize(bytes([0])) == (0, (0, 0), 1)  # every field missing: defaults
    assert L.checksum_deserialize(bytes([1, 2])) == (0, (2, 0), 2)  # value missing at the end: default
    # fields added by a newer writer are skipped; trailing bytes after the table are not consumed
    assert L.checksum_deserialize(bytes([7, 1, 4, 3, 2, 1, 9, 9, 0xAA])) == (0, (1, 0x01020304), 8)
    assert L.checksum_deserialize(bytes([0x85, 0x00, 1, 4, 3, 2, 1])) == (0, (1, 0x01020304), 7)  # 2-byte varint


def test_fin_helpers(hf, orc):
    import numpy as np
    d = np.random.default_rng(4).integers(0, 256, 5000, dtype=np.uint8)
    a, b = d[:1234].tobytes(), d[1234:].tobytes()
    # crc32c crate (finalized) combine == finalized CRC of the concatenation (chunk.rs:229)
    assert hf._lib.crc32c_combine_fin(orc.rs_crc32c(a), orc.rs_crc32c(b), len(b)) == orc.rs_crc32c(a + b)


def test_no_hip_memset_in_library_sources():
    """Round-1 incident guard: the library zeroes accumulators, ticket counters and
    device length bounds with its own kernel (launch_zero_words), never hipMemset*: a small
    memset node replayed a stale pattern in a hipGraph, and round 1's update path memset the
    XOR-accumulated hash outputs and tickets.  Comments may name the call; code may not."""
    import re
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3fs_amd", "csrc")
    bad = []
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".hip", ".h", ".cc", ".cpp")):
            continue
        text = open(os.path.join(csrc, name)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"\bhipMemset\w*\s*\(", text):
            bad.append(f"{name}:{text[:m.start()].count(chr(10)) + 1}")
    assert not bad, f"hipMemset* in library code: {bad}"


def test_options_set_get_and_reject(hf):
    """Tuning / test switches (hf3fs_crc_set_option): read once from the
    environment, overridden only through the ABI; unknown names and values are kInvalidArg
    (a typo must not silently select another pipeline)."""
    L = hf._lib
    assert L.get_option("update_pipeline") == "mode"
    for v in ("fused", "unfused", "mode"):
        L.set_option("update_pipeline", v)
        assert L.get_option("update_pipeline") == v
    for name, value in [("update_pipeline", "single"), ("update_pipeline", "Fused"), ("nt", "2"), ("pipe", "x"),
                        ("apply_pieces", "0"), ("apply_pieces", "65"), ("apply_grid", "3"), ("apply_grid", "-2"),
                        ("apply_piece_kib", "2"), ("apply_piece_kib", "32"), ("no_such_switch", "1")]:
        with pytest.raises(hf.Hf3fsCrcError) as e:
            L.set_option(name, value)
        assert e.value.code == hf.INVALID_ARG
    with L.option("poison", 0xDEADBEEF):
        assert L.get_option("poison") == str(0xDEADBEEF)
    assert L.get_option("poison") == "0" and L.get_option("audit") == "1"
    assert L.get_option("apply_grid") == "-1" and L.get_option("apply_piece_kib") == "8"


def test_options_environment_read_once():
    """The environment is read at the first call only: a later change of HF3FS_CRC_* has no
    effect, and an invalid value or a retired switch is reported on stderr, not applied."""
    code = r'''
import importlib, os, sys
sys.path.insert(0, os.environ["REPO"])
L = importlib.import_module("3fs_amd")._lib
print(L.get_option("update_pipeline"), L.get_option("nt"), L.get_option("apply_pieces"))
os.environ["HF3FS_CRC_NT"] = "1"
print(L.get_option("nt"))
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, REPO=repo, HF3FS_CRC_UPDATE_PIPELINE="fused", HF3FS_CRC_NT="0",
               HF3FS_CRC_APPLY_PIECES="banana", HF3FS_CRC_UPDATE_UNFUSED="1")
    r = subprocess.run(["python3", "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split("\n")[:2] == ["fused 0 8", "0"]
    assert "ignoring HF3FS_CRC_APPLY_PIECES=banana" in r.stderr
    assert "HF3FS_CRC_UPDATE_UNFUSED is no longer read" in r.stderr


def test_no_getenv_outside_options():
    """Library code reads the environment in options.cc only (no per-call switches)."""
    import re
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "3fs_amd", "csrc")
    bad = []
    for name in sorted(os.listdir(csrc)):
        if not name.endswith((".hip", ".h", ".cc", ".cpp")) or name == "options.cc":
            continue
        text = re.sub(r"//[^\n]*", "", open(os.path.join(csrc, name)).read())
        if re.search(r"\bgetenv\s*\(", text):
            bad.append(name)
    assert not bad, bad


def _py_xpow8(nbytes, poly):
    """x^(8 nbytes) mod P with Python's unbounded exponent (reflected register form, bit 31 =
    x^0): an independent check of the 64-bit-overflow-free shift."""
    def mul(a, b):
        p = 0
        for i in range(32):
            if a & (1 << (31 - i)):
                p ^= b
            b = (b >> 1) ^ poly if b & 1 else b >> 1
        return p
    result, base, e = 1 << 31, 1 << 30, 8 * nbytes
    while e:
        if e & 1:
            result = mul(result, base)
        base = mul(base, base)
        e >>= 1
    return result, mul


@pytest.mark.parametrize("len2", [(1 << 61) - 1, 1 << 61, (1 << 61) + 12345, 1 << 62, (1 << 63) + 7, (1 << 64) - 1])
def test_combine_lengths_past_2_61(hf, orc, len2):
    """combine / shift for byte counts whose bit count overflows 64 bits: the library's host
    algebra and the oracle against an unbounded-exponent Python product, both polynomials."""
    for poly, lib_combine in ((orc.POLY_CRC32C, hf._lib.crc32c_combine), (orc.POLY_CRC32, hf._lib.crc32_combine)):
        x, mul = _py_xpow8(len2, poly)
        c1, c2 = 0x12345678, 0x9ABCDEF0
        want = mul(c1, x) ^ c2
        assert lib_combine(c1, c2, len2) == want, (hex(poly), len2)
        assert orc.shift(c1, len2, poly) ^ c2 == want, (hex(poly), len2)
