"""ctypes view of the CPU parity oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package (3fs_amd/).
See crc_oracle.h for what it restates and the reference file:line it follows.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

POLY_CRC32C = 0x82F63B78
POLY_CRC32 = 0xEDB88320
NONE, CRC32C, CRC32 = 0, 1, 2
OK, INVALID_ARG, CHUNK_READ_FAILED, CHECKSUM_MISMATCH = 0, 3, 4010, 4080


class Checksum(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint8), ("value", ctypes.c_uint32)]

    def tup(self):
        return (int(self.type), int(self.value))


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p, u32, u64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
        sig = {
            "orc_crc32c_sw": (u32, [u32, u8p, sz]),
            "orc_crc32c_hw": (u32, [u32, u8p, sz]),
            "orc_crc32_sw": (u32, [u32, u8p, sz]),
            "orc_crc_bitwise": (u32, [u32, u8p, sz, u32]),
            "orc_have_sse42": (ctypes.c_int, []),
            "orc_crc32c_clmul": (u32, [u32, u8p, sz]),
            "orc_crc32c_pclmul128": (u32, [u32, u8p, sz]),
            "orc_have_clmul": (ctypes.c_int, []),
            "orc_have_vpclmul": (ctypes.c_int, []),
            "orc_gf2_mulmod": (u32, [u32, u32, u32]),
            "orc_x8n": (u32, [u64, u32]),
            "orc_shift": (u32, [u32, u64, u32]),
            "orc_crc32c_combine": (u32, [u32, u32, u64]),
            "orc_crc32_combine": (u32, [u32, u32, u64]),
            "orc_rs_crc32c": (u32, [u8p, sz]),
            "orc_rs_crc32c_append": (u32, [u32, u8p, sz]),
            "orc_rs_crc32c_combine": (u32, [u32, u32, sz]),
            "orc_checksum_create": (Checksum, [ctypes.c_uint8, u8p, sz, u32]),
            "orc_checksum_combine": (ctypes.c_int, [ctypes.POINTER(Checksum), Checksum, sz]),
            "orc_replica_update_checksum": (
                ctypes.c_int,
                [u8p, u32, Checksum, Checksum, u32, u32, ctypes.c_int, u32, ctypes.c_int, ctypes.POINTER(Checksum)],
            ),
            "orc_replica_update_checksum_case": (
                ctypes.c_int,
                [u8p, u32, Checksum, Checksum, u32, u32, ctypes.c_int, u32, ctypes.c_int, ctypes.POINTER(Checksum),
                 ctypes.POINTER(ctypes.c_int)],
            ),
            "orc_engine_write_case": (
                ctypes.c_int,
                [u8p, ctypes.POINTER(u32), ctypes.POINTER(u32), u32, u8p, u32, u32, u32, ctypes.c_int, ctypes.c_int,
                 ctypes.c_int, ctypes.POINTER(ctypes.c_int)],
            ),
            "orc_engine_write": (
                ctypes.c_int,
                [u8p, ctypes.POINTER(u32), ctypes.POINTER(u32), u32, u8p, u32, u32, u32, ctypes.c_int, ctypes.c_int,
                 ctypes.c_int],
            ),
            "orc_read_result_checksum": (
                ctypes.c_int,
                [ctypes.c_uint8, Checksum, u32, u32, u32, u8p, u8p, ctypes.c_int, ctypes.POINTER(Checksum)],
            ),
            "orc_calc_serde": (u32, [u8p, sz, ctypes.c_int]),
            "orc_create_batch": (None, [u8p, sz, sz, sz, u8p, ctypes.c_int, ctypes.c_int]),
            "orc_fill_synth": (None, [u8p, sz, u64, u64, u64]),
            "orc_replica_update_batch": (None, [u8p, sz, u8p, sz, u8p, u8p, u8p, u8p, u8p, u8p, sz, ctypes.c_int]),
            "orc_verify_blocks": (sz, [u8p, u8p, u8p, u8p, u8p, sz, ctypes.c_int]),
            "orc_file_digest_batch": (None, [u8p, u8p, u64, ctypes.c_int, u8p, ctypes.c_int]),
            "orc_combine_batch": (None, [u8p, u8p, u8p, sz, u32, ctypes.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _buf(data):
    """Return (pointer, length, keepalive) for bytes / bytearray / numpy uint8."""
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data, dtype=np.uint8)
        return a.ctypes.data, a.nbytes, a
    a = np.frombuffer(bytes(data), dtype=np.uint8)
    return (a.ctypes.data if a.nbytes else None), a.nbytes, a


def crc32c_raw(data, start=0xFFFFFFFF, kind="hw"):
    """kind: "hw" SSE4.2 3-way (folly's crc32 instruction stream), "sw" slicing-by-8,
    "clmul" carry-less folding (VPCLMULQDQ / PCLMULQDQ, whichever the CPU has), "pclmul128"."""
    p, n, _k = _buf(data)
    f = {"hw": lib().orc_crc32c_hw, "sw": lib().orc_crc32c_sw, "clmul": lib().orc_crc32c_clmul,
         "pclmul128": lib().orc_crc32c_pclmul128}[kind]
    return f(start, p, n)


def crc32_raw(data, start=0xFFFFFFFF):
    p, n, _k = _buf(data)
    return lib().orc_crc32_sw(start, p, n)


def bitwise(data, start, poly):
    p, n, _k = _buf(data)
    return lib().orc_crc_bitwise(start, p, n, poly)


def shift(crc, n, poly=POLY_CRC32C):
    return lib().orc_shift(crc, n, poly)


def crc32c_combine(c1, c2, n):
    return lib().orc_crc32c_combine(c1, c2, n)


def crc32_combine(c1, c2, n):
    return lib().orc_crc32_combine(c1, c2, n)


def create(ctype, data, start=0xFFFFFFFF):
    p, n, _k = _buf(data)
    return lib().orc_checksum_create(ctype, p, n, start).tup()


def combine(a, b, length):
    """ChecksumInfo::combine on tuples; returns (status, (type, value))."""
    s = Checksum(*a)
    rc = lib().orc_checksum_combine(ctypes.byref(s), Checksum(*b), length)
    return rc, s.tup()


def rs_crc32c(data):
    p, n, _k = _buf(data)
    return lib().orc_rs_crc32c(p, n)


def rs_append(crc, data):
    p, n, _k = _buf(data)
    return lib().orc_rs_crc32c_append(crc, p, n)


def rs_combine(c1, c2, n):
    return lib().orc_rs_crc32c_combine(c1, c2, n)


def replica_update(chunk_after, size_after, chunk_ck, write_ck, off, length, trunc_or_extend, size_before,
                   is_append, with_case=False):
    """-> (rc, (type, value)), or with_case (rc, (type, value), case): case = the counter
    ChunkReplica::updateChecksum bumps (1 none, 2 reuse, 3 combine, 4 read_chunk)."""
    p, _n, _k = _buf(chunk_after)
    out = Checksum()
    kase = ctypes.c_int(0)
    rc = lib().orc_replica_update_checksum_case(p, size_after, Checksum(*chunk_ck), Checksum(*write_ck), off,
                                                length, int(trunc_or_extend), size_before, int(is_append),
                                                ctypes.byref(out), ctypes.byref(kase))
    return (rc, out.tup(), kase.value) if with_case else (rc, out.tup())


def calc_serde(data, compressed=False):
    p, n, _k = _buf(data)
    return lib().orc_calc_serde(p, n, int(compressed))


def create_batch(arr2d, threads=1, kind=0):
    """Raw CRC32C (start ~0) of each row of a 2-D uint8 array."""
    a = np.ascontiguousarray(arr2d, dtype=np.uint8)
    out = np.zeros(a.shape[0], dtype=np.uint32)
    lib().orc_create_batch(a.ctypes.data, a.strides[0], a.shape[1], a.shape[0], out.ctypes.data, threads, kind)
    return out


def replica_update_batch(chunks2d, payload2d, sizes, cks, offs, lens, wcks, threads=1):
    """CPU baseline of d3: ChunkReplica::update per row (verify, write, prefix/suffix re-hash).
    sizes / cks (uint32 arrays) are updated in place; returns the status array."""
    n = chunks2d.shape[0]
    st = np.zeros(n, dtype=np.int32)
    arrs = [np.ascontiguousarray(a, dtype=np.uint32) for a in (offs, lens, wcks)]
    lib().orc_replica_update_batch(chunks2d.ctypes.data, chunks2d.strides[0], payload2d.ctypes.data,
                                   payload2d.strides[0], sizes.ctypes.data, cks.ctypes.data, arrs[0].ctypes.data,
                                   arrs[1].ctypes.data, arrs[2].ctypes.data, st.ctypes.data, n, threads)
    return st


def verify_blocks(arena, offs, lens, expected, threads=1):
    """CPU baseline of d5: mismatch flags of KV blocks (offset, length) against expected raw CRCs."""
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    expected = np.ascontiguousarray(expected, dtype=np.uint32)
    mism = np.zeros(offs.size, dtype=np.uint8)
    bad = lib().orc_verify_blocks(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, expected.ctypes.data,
                                  mism.ctypes.data, offs.size, threads)
    return int(bad), mism


def fill_synth(n, seed, chunk_id, byte_off=0):
    out = np.empty(n, dtype=np.uint8)
    lib().orc_fill_synth(out.ctypes.data, n, seed, chunk_id, byte_off)
    return out


# ---- ChunkReplica::update driver (ChunkReplica.cc:132-317) -------------------
WRITE, TRUNCATE, EXTEND = 1, 4, 8


def replica_apply(chunk, size, ck, io_type, off, length, payload=b"", write_ck=(NONE, 0), chunk_size=None,
                  with_case=False):
    """Apply one UpdateIO to an in-memory replica the way ChunkReplica::update does.

    chunk: bytearray (capacity >= chunk_size); size/ck: ChunkMetadata.size and
    (checksumType, checksumValue).  Returns (status, new_size, new_ck); on error
    the chunk and metadata are unchanged.  with_case appends the checksum case
    (replica_update; 0 when the IO failed before updateChecksum).
    """
    if chunk_size is None:
        chunk_size = len(chunk)
    if io_type == WRITE and (off >= chunk_size or off + length > chunk_size):  # :139-145
        return (INVALID_ARG, size, ck, 0) if with_case else (INVALID_ARG, size, ck)
    if io_type == WRITE and write_ck[0] != NONE and length != 0:  # :193-207
        if create(write_ck[0], payload[:length]) != tuple(write_ck):
            return (CHECKSUM_MISMATCH, size, ck, 0) if with_case else (CHECKSUM_MISMATCH, size, ck)
    size_before = size
    is_append = off == size  # :243
    if io_type in (TRUNCATE, EXTEND):  # :255-269
        if length <= size:
            if io_type == TRUNCATE:
                size = length
        else:
            chunk[size:length] = bytes(length - size)
            size = length
    else:
        if size < off:  # :281-284 gap zero-fill
            chunk[size:off] = bytes(off - size)
        chunk[off:off + length] = payload[:length]
        size = max(size, off + length)
    rc, out, kase = replica_update(bytes(chunk[:max(size, 1)]), size, ck, write_ck, off, length,
                                   io_type in (TRUNCATE, EXTEND), size_before, is_append, with_case=True)
    return (rc, size, out, kase) if with_case else (rc, size, out)


def engine_apply(buf, length, ck, data, off, capacity, truncate=False, is_syncing=False, exists=True, data_ck=None,
                 with_case=False):
    """Chunk engine write (engine.rs:288-420, chunk.rs:89-281): returns (rc, new_len, new_fin_ck),
    with_case also the engine's checksum counter (1 none, 2 reuse, 3 combine, 4 recalculate)."""
    a = np.frombuffer(buf, dtype=np.uint8) if isinstance(buf, bytearray) else buf
    L = ctypes.c_uint32(length)
    C = ctypes.c_uint32(ck)
    d = np.frombuffer(bytes(data), dtype=np.uint8)
    if data_ck is None:
        data_ck = rs_crc32c(bytes(data))
    kase = ctypes.c_int(0)
    rc = lib().orc_engine_write_case(a.ctypes.data, ctypes.byref(L), ctypes.byref(C), capacity,
                                     d.ctypes.data if d.nbytes else None, len(d), off, data_ck, int(truncate),
                                     int(is_syncing), int(exists), ctypes.byref(kase))
    return (rc, int(L.value), int(C.value), kase.value) if with_case else (rc, int(L.value), int(C.value))


def read_result(batch_type, chunk_ck, read_off, read_data, chunk_len, full_chunk=None, recalculate=False):
    """AioReadJob::setResult checksum part (BatchReadJob.cc:24-63) -> (rc, (type, value))."""
    rp, rn, _k1 = _buf(read_data)
    fp, _fn, _k2 = _buf(full_chunk if full_chunk is not None else b"")
    out = Checksum()
    rc = lib().orc_read_result_checksum(batch_type, Checksum(*chunk_ck), read_off, rn, chunk_len, rp, fp,
                                        int(recalculate), ctypes.byref(out))
    return rc, out.tup()


_ZEROS = bytearray()


def file_digest(blocks, fill_zero=True):
    """FileWrapper::readFile's checksum fold (src/client/cli/admin/FileWrapper.cc:
    119-164): blocks = [(read_len, block_len, (type, value)[, missing])] in file order
    -> (status, (type, value)).  missing = the read failed with kChunkNotFound.
    With fill_zero (the admin --fill-zero option) holes are hashed as real zero
    bytes through create(CRC32C, zeros, needFill) and combine, a missing chunk as a
    read of 0 bytes with the default checksum (:134-135); without it the first
    missing chunk ends the fold with its read error (kChunkNotFound 7007, :136-138)
    and the first read of another length with kInvalidFormat (33, :153-160)."""
    global _ZEROS
    blocks = [b if len(b) == 4 else (b[0], b[1], b[2], False) for b in blocks]
    # Malformed blocks are rejected before the fold (kInvalidArg); the reference
    # cannot represent them (needFill would underflow, ChecksumType is an enum).
    for read_len, block_len, ck, missing in blocks:
        if ck[0] not in (NONE, CRC32C, CRC32) or (fill_zero and not missing and read_len > block_len):
            return 3, (NONE, 0)
    acc = (NONE, 0)
    for read_len, block_len, ck, missing in blocks:
        if missing:
            if not fill_zero:
                return 7007, (NONE, 0)
            read_len, ck = 0, (NONE, 0)
        succ = read_len
        if succ != block_len:
            if not fill_zero:
                return 33, (NONE, 0)
            need = block_len - succ
            if len(_ZEROS) < need:
                _ZEROS = bytearray(need)
            zeros = create(CRC32C, bytes(memoryview(_ZEROS)[:need]))
            rc, ck = combine(ck, zeros, need)
            if rc:
                return rc, (NONE, 0)
            succ = block_len
        rc, acc = combine(acc, ck, succ)
        if rc:
            return rc, (NONE, 0)
    return 0, acc


def combine_batch(acc, crc2, len2, poly=POLY_CRC32C, threads=1):
    """Element-wise ChecksumInfo::combine in C (crc_oracle.c orc_combine_batch): returns a new
    array acc' with acc'[i] = combine(~acc[i], crc2[i], len2[i]) where len2[i] > 0."""
    out = np.ascontiguousarray(acc, dtype=np.uint32).copy()
    crc2 = np.ascontiguousarray(crc2, dtype=np.uint32)
    len2 = np.ascontiguousarray(len2, dtype=np.uint64)
    lib().orc_combine_batch(out.ctypes.data, crc2.ctypes.data, len2.ctypes.data, out.size, poly, threads)
    return out


BLOCK_DIGEST_DT = np.dtype([("read_len", "<u8"), ("block_len", "<u8"), ("checksum", "<u4"), ("type", "u1"),
                            ("missing", "u1"), ("res", "u1", (2,))])
FILE_RESULT_DT = np.dtype([("status", "<i4"), ("type", "u1"), ("pad", "u1", (3,)), ("value", "<u4")])


def file_digest_batch(blocks, file_off, fill_zero=True, threads=1):
    """file_digest over many files in C (crc_oracle.c orc_file_digest_batch, the same fold):
    blocks = BLOCK_DIGEST_DT array (the layout of hf3fs_crc_block_digest), file f = blocks
    [file_off[f], file_off[f + 1]).  Returns a FILE_RESULT_DT array (status, type, value)."""
    blocks = np.ascontiguousarray(blocks).view(BLOCK_DIGEST_DT)
    file_off = np.ascontiguousarray(file_off, dtype=np.uint64)
    n = file_off.size - 1
    out = np.zeros(n, dtype=FILE_RESULT_DT)
    lib().orc_file_digest_batch(blocks.ctypes.data, file_off.ctypes.data, n, 1 if fill_zero else 0, out.ctypes.data,
                                threads)
    return out


def scrub(ctype, fin, data, stored):
    """Recompute-and-compare of a stored chunk against its persisted checksum,
    as AioReadJob::setResult's full-chunk resync check (BatchReadJob.cc:43-54):
    create(type, bytes, len) != stored -> kChecksumMismatch.  Chunk-engine
    records persist the finalized value (ChunkEngine.cc:42,66): raw = ~fin.
    NONE records have nothing to check.  Returns (status, computed_raw)."""
    if ctype == NONE:
        return OK, 0
    computed = create(ctype, data)[1]
    want = (~stored & 0xFFFFFFFF) if fin else stored
    return (OK if computed == want else CHECKSUM_MISMATCH), computed
