"""ctypes binding of the C ABI in include/hf3fs_crc.h (libhf3fs_crc.so).

This is the Python-side view of the drop-in boundary used by tests, bench.py
and smoke().  It never computes a checksum itself: every call goes to the HIP
library, and a missing library raises instead of falling back to anything.
"""
import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
# HF3FS_CRC_LIB: load another build of the library (same-tree A/B of kernel variants)
LIB_PATH = os.environ.get("HF3FS_CRC_LIB") or os.path.join(HERE, "lib", "libhf3fs_crc.so")
HEADER = os.path.join(REPO, "include", "hf3fs_crc.h")

NONE, CRC32C, CRC32 = 0, 1, 2
UPDATE_WRITE, UPDATE_TRUNCATE, UPDATE_EXTEND = 1, 4, 8
MODE_REFERENCE, MODE_DELTA = 0, 1
OK, INVALID_ARG, CHUNK_READ_FAILED, CHECKSUM_MISMATCH, CLIENT_CHECKSUM_MISMATCH, DEVICE_ERROR = (
    0, 3, 4010, 4080, 7015, 9001)
SERDE_INSUFFICIENT_LENGTH = 40


class Hf3fsCrcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"hf3fs_crc error {code}: {msg}")
        self.code = code


class UpdateIO(ctypes.Structure):
    """hf3fs_crc_update_io (include/hf3fs_crc.h)."""
    _fields_ = [
        ("chunk", ctypes.c_uint64),
        ("payload", ctypes.c_uint64),
        ("offset", ctypes.c_uint32),
        ("length", ctypes.c_uint32),
        ("chunk_size", ctypes.c_uint32),
        ("update_type", ctypes.c_uint8),
        ("chunk_checksum_type", ctypes.c_uint8),
        ("write_checksum_type", ctypes.c_uint8),
        ("flags", ctypes.c_uint8),
        ("chunk_checksum", ctypes.c_uint32),
        ("write_checksum", ctypes.c_uint32),
        ("out_size", ctypes.c_uint32),
        ("out_checksum", ctypes.c_uint32),
        ("out_checksum_type", ctypes.c_uint8),
        ("checksum_case", ctypes.c_uint8),
        ("reserved1", ctypes.c_uint8 * 2),
        ("status", ctypes.c_int32),
    ]


assert ctypes.sizeof(UpdateIO) == 56
UPDATE_FLAG_ENGINE = 1
DIGEST_FILL_ZERO = 1  # hf3fs_crc_file_digest_batch_ex flags
# UpdateIO.checksum_case (HF3FS_CKCASE_*): the reference's checksum counter for the IO
CKCASE_NONE, CKCASE_REUSE, CKCASE_COMBINE, CKCASE_RECOMPUTE = 1, 2, 3, 4


class ReadIO(ctypes.Structure):
    """hf3fs_crc_read_io (include/hf3fs_crc.h): AioReadJob::setResult inputs/outputs."""
    _fields_ = [
        ("data", ctypes.c_uint64),
        ("offset", ctypes.c_uint32),
        ("length", ctypes.c_uint32),
        ("chunk_len", ctypes.c_uint32),
        ("batch_checksum_type", ctypes.c_uint8),
        ("chunk_checksum_type", ctypes.c_uint8),
        ("recalculate", ctypes.c_uint8),
        ("reserved0", ctypes.c_uint8),
        ("chunk_checksum", ctypes.c_uint32),
        ("out_checksum", ctypes.c_uint32),
        ("out_checksum_type", ctypes.c_uint8),
        ("reserved1", ctypes.c_uint8 * 3),
        ("status", ctypes.c_int32),
        ("reserved2", ctypes.c_uint32),
    ]


assert ctypes.sizeof(ReadIO) == 48


class BlockDigest(ctypes.Structure):
    """hf3fs_crc_block_digest: one chunk read of a file (FileWrapper.cc:133-160)."""
    _fields_ = [
        ("read_len", ctypes.c_uint64),
        ("block_len", ctypes.c_uint64),
        ("checksum", ctypes.c_uint32),
        ("checksum_type", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 3),
    ]


class FileDigest(ctypes.Structure):
    """hf3fs_crc_file_digest: ChecksumInfo of one file (or replica) + status."""
    _fields_ = [
        ("length", ctypes.c_uint64),
        ("value", ctypes.c_uint32),
        ("type", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 3),
        ("status", ctypes.c_int32),
        ("reserved2", ctypes.c_uint32),
    ]


assert ctypes.sizeof(BlockDigest) == 24 and ctypes.sizeof(FileDigest) == 24

class ScrubIO(ctypes.Structure):
    """hf3fs_crc_scrub_io: one stored chunk vs its persisted checksum."""
    _fields_ = [
        ("data", ctypes.c_uint64),
        ("length", ctypes.c_uint32),
        ("checksum_type", ctypes.c_uint8),
        ("fin", ctypes.c_uint8),
        ("reserved", ctypes.c_uint16),
        ("checksum", ctypes.c_uint32),
        ("computed", ctypes.c_uint32),
        ("status", ctypes.c_int32),
        ("reserved2", ctypes.c_uint32),
    ]


class Frame(ctypes.Structure):
    """hf3fs_crc_frame: one serde message of a receive buffer."""
    _fields_ = [
        ("offset", ctypes.c_uint64),
        ("size", ctypes.c_uint32),
        ("checksum", ctypes.c_uint32),
        ("computed", ctypes.c_uint32),
        ("status", ctypes.c_int32),
    ]


class EngineMeta(ctypes.Structure):
    """hf3fs_crc_engine_meta: the chunk engine's ChunkMeta (chunk_meta.rs:7-20)."""
    _fields_ = [
        ("pos", ctypes.c_uint64),
        ("chain_ver", ctypes.c_uint32),
        ("chunk_ver", ctypes.c_uint32),
        ("len", ctypes.c_uint32),
        ("checksum", ctypes.c_uint32),
        ("timestamp", ctypes.c_uint64),
        ("last_request_id", ctypes.c_uint64),
        ("last_client_low", ctypes.c_uint64),
        ("last_client_high", ctypes.c_uint64),
        ("etag_len", ctypes.c_uint8),
        ("uncommitted", ctypes.c_uint8),
        ("etag", ctypes.c_uint8 * 62),
    ]


assert ctypes.sizeof(ScrubIO) == 32 and ctypes.sizeof(Frame) == 24 and ctypes.sizeof(EngineMeta) == 120


class Anomaly(ctypes.Structure):
    """hf3fs_crc_anomaly: the update self-check's record."""
    _fields_ = [
        ("count", ctypes.c_uint32),
        ("kinds", ctypes.c_uint32),
        ("kind", ctypes.c_uint32),
        ("pipeline", ctypes.c_uint32),
        ("io", ctypes.c_uint64),
        ("pipeline_hash", ctypes.c_uint32),
        ("rehash", ctypes.c_uint32),
        ("client_checksum", ctypes.c_uint32),
        ("pre_max", ctypes.c_uint32),
        ("pre_addr", ctypes.c_uint64),
        ("pre_len", ctypes.c_uint64),
        ("payload", ctypes.c_uint64),
        ("length", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


assert ctypes.sizeof(Anomaly) == 72
ANOMALY_PAYLOAD_HASH, ANOMALY_PRE_JOB, ANOMALY_PRE_MAX, ANOMALY_START_ONLY, ANOMALY_RUN_COVER = 1, 2, 4, 8, 16


class CoalescerOptions(ctypes.Structure):
    """hf3fs_crc_coalescer_options (include/hf3fs_crc.h)."""
    _fields_ = [
        ("device", ctypes.c_int),
        ("max_batch", ctypes.c_uint32),
        ("max_wait_us", ctypes.c_uint32),
        ("slots", ctypes.c_uint32),
        ("inflight", ctypes.c_uint32),
        ("service_wgs", ctypes.c_uint32),
        ("stage_bytes", ctypes.c_uint64),
        ("service_ring", ctypes.c_uint32),
        ("service_idle_us", ctypes.c_uint32),
        ("service_stage", ctypes.c_uint64),
    ]


assert ctypes.sizeof(CoalescerOptions) == 48
REQ_HOST_COPY = 1
DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32)

_vp, _u8, _u32, _u64, _int = ctypes.c_void_p, ctypes.c_uint8, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
SIGNATURES = {
    "hf3fs_crc_init": (_int, [_int]),
    "hf3fs_crc_shutdown": (None, []),
    "hf3fs_crc_last_error": (ctypes.c_char_p, []),
    "hf3fs_crc_version": (ctypes.c_char_p, []),
    "hf3fs_crc32c_combine": (_u32, [_u32, _u32, _u64]),
    "hf3fs_crc32_combine": (_u32, [_u32, _u32, _u64]),
    "hf3fs_crc_shift": (_u32, [_u8, _u32, _u64]),
    "hf3fs_checksum_combine": (_int, [ctypes.POINTER(_u8), ctypes.POINTER(_u32), _u8, _u32, _u64]),
    "hf3fs_crc_create_batch": (_int, [_u8, _vp, _vp, _vp, _vp, _u64, _u64, _vp]),
    "hf3fs_crc_create_strided": (_int, [_u8, _vp, _u64, _u64, _u64, _u32, _vp, _vp]),
    "hf3fs_crc_verify_batch": (_int, [_u8, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _u64, _vp]),
    "hf3fs_crc_verify_strided": (_int, [_u8, _vp, _u64, _u64, _u64, _vp, _vp, _vp, _vp, _vp]),
    "hf3fs_crc_verify_blocks": (_int, [_u8, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _u32, _vp]),
    "hf3fs_crc_combine_batch": (_int, [_u8, _vp, _vp, _vp, _u64, _vp]),
    "hf3fs_crc_update_batch": (_int, [_u8, _vp, _u64, _u32, _int, _vp]),
    "hf3fs_crc_update_scratch_bytes": (ctypes.c_size_t, [_u64, _int]),
    "hf3fs_crc_read_result_batch": (_int, [_u8, _vp, _u64, _u32, _vp]),
    "hf3fs_crc_file_digest_batch": (_int, [_vp, _vp, _vp, _u64, _u64, _vp]),
    "hf3fs_crc_file_digest_batch_ex": (_int, [_vp, _vp, _vp, _u64, _u64, _u32, _vp]),
    "hf3fs_crc_create_host": (_int, [_u8, _vp, _vp, _vp, _vp, _u64]),
    "hf3fs_crc_fill_synth": (_int, [_vp, _u64, _u64, _u64, _u64, _u64, _vp]),
    "hf3fs_crc_scrub_batch": (_int, [_u8, _vp, _u64, _u32, _vp, _vp]),
    "hf3fs_crc_engine_meta_decode": (_int, [_vp, _u64, ctypes.POINTER(EngineMeta), ctypes.POINTER(_u64)]),
    "hf3fs_crc_engine_meta_encode": (_int, [ctypes.POINTER(EngineMeta), _vp, _u64, ctypes.POINTER(_u64)]),
    "hf3fs_crc_default_etag": (_u32, [_u32, _vp]),
    "hf3fs_crc_frame_walk": (_int, [_vp, _u64, _vp, _u64, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "hf3fs_crc_frame_verify_batch": (_int, [_vp, _vp, _u64, _u32, _vp, _vp]),
    "hf3fs_crc_coalescer_default_options": (None, [ctypes.POINTER(CoalescerOptions)]),
    "hf3fs_crc_coalescer_create": (_int, [ctypes.POINTER(CoalescerOptions), ctypes.POINTER(_vp)]),
    "hf3fs_crc_coalescer_destroy": (None, [_vp]),
    "hf3fs_crc_coalescer_submit": (_int, [_vp, _u8, _vp, _u64, _u32, _u32, DONE_FN, _vp]),
    "hf3fs_crc_coalescer_create_one": (_int, [_vp, _u8, _vp, _u64, _u32, _u32, ctypes.POINTER(_u32)]),
    "hf3fs_crc_coalescer_stats": (_int, [_vp, ctypes.POINTER(_u64)]),
    "hf3fs_crc_host_register": (_int, [_vp, _u64, ctypes.POINTER(_vp)]),
    "hf3fs_crc_host_unregister": (_int, [_vp]),
    "hf3fs_checksum_serialize": (_u32, [_u8, _u32, _vp]),
    "hf3fs_checksum_deserialize": (_int, [_vp, _u64, ctypes.POINTER(_u8), ctypes.POINTER(_u32), ctypes.POINTER(_u64)]),
    "hf3fs_crc_serialize_batch": (_int, [_u8, _vp, _u64, _vp, _vp]),
    "hf3fs_crc_finalize_batch": (_int, [_vp, _u64, _vp]),
    "hf3fs_crc32c_combine_fin": (_u32, [_u32, _u32, _u64]),
    "hf3fs_crc_release_stream": (_int, [_vp]),
    "hf3fs_crc_release_graph_scratch": (_int, []),
    "hf3fs_crc_graph_scratch_stats": (_int, [_vp, _vp, _vp]),
    "hf3fs_crc_stream_wait": (_int, [_vp, _u32]),
    "hf3fs_crc_set_option": (_int, [ctypes.c_char_p, ctypes.c_char_p]),
    "hf3fs_crc_get_option": (_int, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]),
    "hf3fs_crc_anomalies": (_int, [_int, ctypes.c_void_p, _int]),
}

_lib = None


def header_symbols():
    """Function names declared in include/hf3fs_crc.h."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(hf3fs_[a-z0-9_]+)\s*\(", text)))


def load():
    """Load the HIP library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: run `python 3fs_amd/build.py` (hipcc --offload-arch=gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    ab_build = bool(os.environ.get("HF3FS_CRC_LIB"))  # an A/B build may predate newer entry points
    for name, (res, args) in SIGNATURES.items():
        if ab_build and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != OK:
        msg = load().hf3fs_crc_last_error()
        raise Hf3fsCrcError(rc, msg.decode() if msg else "")
    return rc


def _p(x):
    """Device/host address of a torch tensor, an int, or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


def _s(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


# ---- thin wrappers (addresses may be torch tensors or ints) ------------------
def create_strided(ctype, base, stride, length, n, out, start=0xFFFFFFFF, stream=None):
    return check(load().hf3fs_crc_create_strided(ctype, _p(base), stride, length, n, start, _p(out), _s(stream)))


def create_batch(ctype, bufs, lens, out, n, max_len, starts=None, stream=None):
    return check(load().hf3fs_crc_create_batch(ctype, _p(bufs), _p(lens), _p(starts), _p(out), n, max_len,
                                               _s(stream)))


def verify_batch(ctype, bufs, lens, expected, mismatch, count, n, max_len, computed=None, stream=None):
    return check(load().hf3fs_crc_verify_batch(ctype, _p(bufs), _p(lens), _p(expected), _p(mismatch), _p(count),
                                               _p(computed), n, max_len, _s(stream)))


def verify_strided(ctype, base, stride, length, n, expected, mismatch, count, computed=None, stream=None):
    return check(load().hf3fs_crc_verify_strided(ctype, _p(base), stride, length, n, _p(expected), _p(mismatch),
                                                 _p(count), _p(computed), _s(stream)))


def verify_blocks(ctype, arena, offsets, lens, expected, mismatch, count, n, max_len, computed=None, stream=None):
    return check(load().hf3fs_crc_verify_blocks(ctype, _p(arena), _p(offsets), _p(lens), _p(expected),
                                                _p(mismatch), _p(count), _p(computed), n, max_len, _s(stream)))


def combine_batch(ctype, acc, crc2, len2, n, stream=None):
    return check(load().hf3fs_crc_combine_batch(ctype, _p(acc), _p(crc2), _p(len2), n, _s(stream)))


def update_batch(ctype, ios, n, max_len, mode=MODE_REFERENCE, stream=None):
    """hf3fs_crc_update_batch; REFERENCE by default (DELTA trusts the stored checksum)."""
    return check(load().hf3fs_crc_update_batch(ctype, _p(ios), n, max_len, mode, _s(stream)))


def update_scratch_bytes(n, mode=MODE_REFERENCE):
    """Bytes of library-owned scratch one update_batch of n IOs takes (the calling
    (stream, thread) pair's buffer, or a captured call's own; never the stream-ordered pool)."""
    return int(load().hf3fs_crc_update_scratch_bytes(n, mode))


def set_option(name, value):
    """hf3fs_crc_set_option: a tuning / test switch for every later call."""
    return check(load().hf3fs_crc_set_option(name.encode(), str(value).encode()))


def get_option(name):
    out = ctypes.create_string_buffer(32)
    check(load().hf3fs_crc_get_option(name.encode(), out, 32))
    return out.value.decode()


class option:
    """with option("update_pipeline", "fused"): ... -- set for the block, restored after."""

    def __init__(self, name, value):
        self.name, self.value = name, value

    def __enter__(self):
        self.old = get_option(self.name)
        set_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_option(self.name, self.old)


def anomalies(device=0, reset=False):
    """hf3fs_crc_anomalies: the update self-check's record as a dict (device-synchronizes)."""
    a = Anomaly()
    check(load().hf3fs_crc_anomalies(device, ctypes.byref(a), 1 if reset else 0))
    return a.as_dict()


def release_stream(stream):
    return check(load().hf3fs_crc_release_stream(_s(stream)))


def release_graph_scratch():
    return check(load().hf3fs_crc_release_graph_scratch())


def stream_wait(stream=None, poll_us=20):
    """Wait for the stream's queued work, polling with a poll_us sleep (0: hipStreamSynchronize)."""
    return check(load().hf3fs_crc_stream_wait(_s(stream), poll_us))


def graph_scratch_stats():
    """{live, live_bytes, dead}: buffers of captured calls still owned by a graph, and
    those whose graph is gone, awaiting the next uncaptured call's free."""
    v = (ctypes.c_uint64 * 3)()
    check(load().hf3fs_crc_graph_scratch_stats(ctypes.addressof(v), ctypes.addressof(v) + 8, ctypes.addressof(v) + 16))
    return {"live": int(v[0]), "live_bytes": int(v[1]), "dead": int(v[2])}


def read_result_batch(ctype, ios, n, max_len, stream=None):
    return check(load().hf3fs_crc_read_result_batch(ctype, _p(ios), n, max_len, _s(stream)))


def file_digest_batch(blocks, file_off, out, n_files, max_blocks, stream=None, fill_zero=True):
    """blocks: device array of hf3fs_crc_block_digest; file_off: n_files+1 uint64;
    out: n_files hf3fs_crc_file_digest (see include/hf3fs_crc.h).  fill_zero=False:
    the admin command without --fill-zero (first missing / short block is the status)."""
    return check(load().hf3fs_crc_file_digest_batch_ex(_p(blocks), _p(file_off), _p(out), n_files, max_blocks,
                                                       DIGEST_FILL_ZERO if fill_zero else 0, _s(stream)))


def scrub_batch(ctype, ios, n, max_len, count, stream=None):
    """ios: device array of hf3fs_crc_scrub_io (updated in place); count: device u32."""
    return check(load().hf3fs_crc_scrub_batch(ctype, _p(ios), n, max_len, _p(count), _s(stream)))


def frame_verify_batch(buf, frames, n, max_size, count, stream=None):
    return check(load().hf3fs_crc_frame_verify_batch(_p(buf), _p(frames), n, max_size, _p(count), _s(stream)))


def frame_walk(data, max_frames=None):
    """Processor::unpackMsg framing walk over host bytes -> (status, [Frame], consumed)."""
    b = bytes(data)
    cap = max_frames if max_frames is not None else max(1, len(b) // 8)
    frames = (Frame * max(1, cap))()
    nf, used = ctypes.c_uint64(), ctypes.c_uint64()
    buf = ctypes.create_string_buffer(b, max(1, len(b)))
    rc = load().hf3fs_crc_frame_walk(buf, len(b), frames, cap, ctypes.byref(nf), ctypes.byref(used))
    return rc, [frames[i] for i in range(nf.value)], int(used.value)


def engine_meta_decode(data):
    """derse ChunkMeta bytes -> (status, EngineMeta, consumed)."""
    b = bytes(data)
    m = EngineMeta()
    used = ctypes.c_uint64()
    buf = ctypes.create_string_buffer(b, max(1, len(b)))
    rc = load().hf3fs_crc_engine_meta_decode(buf, len(b), ctypes.byref(m), ctypes.byref(used))
    return rc, m, int(used.value)


def engine_meta_encode(m):
    out = ctypes.create_string_buffer(256)
    w = ctypes.c_uint64()
    rc = load().hf3fs_crc_engine_meta_encode(ctypes.byref(m), out, 256, ctypes.byref(w))
    return rc, out.raw[:w.value]


def default_etag(checksum_fin):
    out = ctypes.create_string_buffer(8)
    k = load().hf3fs_crc_default_etag(checksum_fin, out)
    return out.raw[:k].decode()


def fill_synth(dst, stride, chunk_len, n_chunks, seed, first_chunk_id=0, stream=None):
    return check(load().hf3fs_crc_fill_synth(_p(dst), stride, chunk_len, n_chunks, seed, first_chunk_id,
                                             _s(stream)))


def create_host(ctype, buffers, starts=None):
    """ChecksumInfo::create over a list of host bytes-like objects -> list of raw values."""
    n = len(buffers)
    keep = [ctypes.create_string_buffer(bytes(b), max(1, len(b))) for b in buffers]
    ptrs = (ctypes.c_void_p * max(1, n))(*[ctypes.addressof(k) for k in keep])
    lens = (ctypes.c_uint64 * max(1, n))(*[len(b) for b in buffers])
    st = (ctypes.c_uint32 * max(1, n))(*starts) if starts is not None else None
    out = (ctypes.c_uint32 * max(1, n))()
    check(load().hf3fs_crc_create_host(ctype, ptrs, lens, st, out, n))
    return [int(out[i]) for i in range(n)]


def checksum_serialize(ctype, value):
    """ChecksumInfo in serde binary form (6 bytes)."""
    out = ctypes.create_string_buffer(6)
    k = load().hf3fs_checksum_serialize(ctype, value, out)
    return out.raw[:k]


def checksum_deserialize(data):
    """-> (status, (type, value), consumed)."""
    b = bytes(data)
    t, v, used = ctypes.c_uint8(), ctypes.c_uint32(), ctypes.c_uint64()
    buf = ctypes.create_string_buffer(b, max(1, len(b)))
    rc = load().hf3fs_checksum_deserialize(buf, len(b), ctypes.byref(t), ctypes.byref(v), ctypes.byref(used))
    return rc, (int(t.value), int(v.value)), int(used.value)


def serialize_batch(ctype, values, n, out, stream=None):
    return check(load().hf3fs_crc_serialize_batch(ctype, _p(values), n, _p(out), _s(stream)))


def finalize_batch(values, n, stream=None):
    return check(load().hf3fs_crc_finalize_batch(_p(values), n, _s(stream)))


def crc32c_combine_fin(f1, f2, len2):
    return int(load().hf3fs_crc32c_combine_fin(f1, f2, len2))


def crc32c_combine(c1, c2, len2):
    return int(load().hf3fs_crc32c_combine(c1, c2, len2))


def crc32_combine(c1, c2, len2):
    return int(load().hf3fs_crc32_combine(c1, c2, len2))


def shift(ctype, crc, nbytes):
    return int(load().hf3fs_crc_shift(ctype, crc, nbytes))


def checksum_combine(a, b, length):
    """ChecksumInfo::combine on (type, value) tuples -> (status, (type, value))."""
    t = ctypes.c_uint8(a[0])
    v = ctypes.c_uint32(a[1])
    rc = load().hf3fs_checksum_combine(ctypes.byref(t), ctypes.byref(v), b[0], b[1], length)
    return rc, (int(t.value), int(v.value))


class Coalescer:
    """hf3fs_crc_coalescer: per-IO ChecksumInfo::create requests from many
    threads, hashed in batched device launches (include/hf3fs_crc.h)."""

    def __init__(self, device=None, **opts):
        L = load()
        o = CoalescerOptions()
        L.hf3fs_crc_coalescer_default_options(ctypes.byref(o))
        if device is not None:
            o.device = device
        for k, v in opts.items():
            setattr(o, k, v)
        h = ctypes.c_void_p()
        check(L.hf3fs_crc_coalescer_create(ctypes.byref(o), ctypes.byref(h)))
        self._h = h

    def create_one(self, ctype, buf, length, start=0xFFFFFFFF, flags=0):
        """Blocking create; `buf` is an address (int), a torch tensor or, with
        REQ_HOST_COPY, any host buffer exposing the buffer protocol."""
        out = ctypes.c_uint32()
        check(load().hf3fs_crc_coalescer_create_one(self._h, ctype, _host_or_dev(buf, flags), length, start, flags,
                                                    ctypes.byref(out)))
        return int(out.value)

    def submit(self, ctype, buf, length, fn, start=0xFFFFFFFF, flags=0):
        """Asynchronous create; fn must be a DONE_FN kept alive until it runs."""
        return check(load().hf3fs_crc_coalescer_submit(self._h, ctype, _host_or_dev(buf, flags), length, start,
                                                       flags, fn, None))

    def stats(self):
        a = (ctypes.c_uint64 * 4)()
        check(load().hf3fs_crc_coalescer_stats(self._h, a))
        return dict(requests=a[0], batches=a[1], bytes=a[2], max_batch=a[3])

    def close(self):
        if self._h:
            load().hf3fs_crc_coalescer_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _host_or_dev(buf, flags):
    if isinstance(buf, int) or buf is None:
        return buf
    if hasattr(buf, "data_ptr"):
        return buf.data_ptr()
    if hasattr(buf, "ctypes"):  # numpy array
        return buf.ctypes.data
    return ctypes.addressof(ctypes.c_char.from_buffer(buf))


def host_register(ptr, length):
    d = ctypes.c_void_p()
    check(load().hf3fs_crc_host_register(ptr, length, ctypes.byref(d)))
    return int(d.value)


def host_unregister(ptr):
    return check(load().hf3fs_crc_host_unregister(ptr))
