"""Python mirror of hf3fs::storage::ChecksumInfo (src/fbs/storage/Common.h:113-202).

Same names, argument meaning and error behaviour as the reference struct; the
bytes are hashed by the HIP library (hf3fs_crc_create_host / create_batch) and
combine goes through the library's C ABI.  The C++ drop-in with identical
semantics is include/hf3fs/storage/ChecksumInfo.h.
"""
import enum
from dataclasses import dataclass

from . import _lib


class ChecksumType(enum.IntEnum):  # Common.h:66-70
    NONE = 0
    CRC32C = 1
    CRC32 = 2


class StorageCode(enum.IntEnum):  # src/common/utils/StatusCodeDetails.h
    kChecksumMismatch = 4080


K_CHUNK_SIZE = 1 << 20  # ChecksumInfo::kChunkSize = 1_MB (Common.h:118)


@dataclass
class ChecksumInfo:
    type: ChecksumType = ChecksumType.NONE
    value: int = 0

    @staticmethod
    def create(type, data, length=None, starting_checksum=0xFFFFFFFF):
        """ChecksumInfo::create(type, buffer, length, startingChecksum) (Common.h:146-177)."""
        type = ChecksumType(type)
        if type == ChecksumType.NONE:
            return ChecksumInfo(ChecksumType.NONE, 0)
        mv = memoryview(bytes(data) if not isinstance(data, (bytes, bytearray, memoryview)) else data)
        if length is None:
            length = len(mv)
        if length > len(mv):
            # an iterator that runs dry before `length` bytes -> {NONE, 0} (:166-169)
            return ChecksumInfo(ChecksumType.NONE, 0)
        (value,) = _lib.create_host(int(type), [bytes(mv[:length])], starts=[starting_checksum])
        return ChecksumInfo(type, value)

    def combine(self, other, length):
        """ChecksumInfo::combine (Common.h:179-198); returns 0 or kChecksumMismatch."""
        rc, (t, v) = _lib.checksum_combine((int(self.type), self.value), (int(other.type), other.value), length)
        if rc == 0:
            self.type, self.value = ChecksumType(t), v
        return rc

    def serialize(self):
        """serde::serialize(ChecksumInfo): 6 bytes (TestCommonStruct.cc:46-55)."""
        return _lib.checksum_serialize(int(self.type), self.value)

    @staticmethod
    def deserialize(data):
        """serde::deserialize -> (status, ChecksumInfo or None)."""
        rc, (t, v), _ = _lib.checksum_deserialize(data)
        return rc, (ChecksumInfo(ChecksumType(t), v) if rc == 0 else None)

    def __str__(self):  # formatter prints ~value (Common.h:768-773)
        return f"{self.type.name}#{(~self.value) & 0xFFFFFFFF:08X}"
