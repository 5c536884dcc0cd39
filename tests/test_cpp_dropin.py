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
