"""3fs_amd -- MI355X-native batched chunk-integrity engine for 3FS's ChecksumInfo path.

Import with importlib (the directory name starts with a digit):
    hf = importlib.import_module("3fs_amd")

Contents:
  csrc/           HIP kernels (gfx950) + the C ABI (include/hf3fs_crc.h)
  lib/            built libhf3fs_crc.so (python 3fs_amd/build.py)
  _lib.py         ctypes binding of the C ABI
  checksum.py     ChecksumInfo mirror (Common.h:113-202)
  node.py         multi-GPU sharding by chain id + RCCL digest all-gather
"""
from . import _lib  # noqa: F401
from ._lib import (CHECKSUM_MISMATCH, CRC32, CRC32C, DEVICE_ERROR, INVALID_ARG, MODE_DELTA, MODE_REFERENCE, NONE, OK,  # noqa: F401
                   UPDATE_EXTEND, UPDATE_TRUNCATE, UPDATE_WRITE, Hf3fsCrcError, UpdateIO, load)
from .checksum import ChecksumInfo, ChecksumType  # noqa: F401
