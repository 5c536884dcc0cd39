"""Run the C++ drop-in test (tests/cpp/test_checksuminfo.cpp) on the GPU: the
reference's own checksum tests written against include/hf3fs/storage/ChecksumInfo.h."""
import importlib
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def test_cpp_dropin_binary():
    b = importlib.import_module("3fs_amd.build")
    assert os.path.exists(b.CPP_TEST_BIN), "built by __graft_entry__.build() / 3fs_amd/build.py"
    r = subprocess.run([b.CPP_TEST_BIN], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout


def test_cpp_pageable_staging():
    """One reused device payload buffer, a pageable hipMemcpy of distinct bytes per IO,
    update_batch on the null stream: 100 IOs per (chunk size 512 B / 128 KiB, REFERENCE /
    DELTA, fused / three-pass), every status, checksum and chunk byte vs the oracle
    (tests/cpp/test_staging.cpp)."""
    b = importlib.import_module("3fs_amd.build")
    assert os.path.exists(b.CPP_TEST_STAGING), "built by __graft_entry__.build() / 3fs_amd/build.py"
    r = subprocess.run([b.CPP_TEST_STAGING], capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
    assert r.stdout.count("fails=0") == 8, r.stdout
