"""ASAN/UBSAN on the host-only code (the reference's sanitizer builds,
cmake/Sanitizers.cmake:18-): tests/cpp/fuzz_host_codec.cpp links the C ABI's parsers of
untrusted bytes (3fs_amd/csrc/host_codec.cc: ChecksumInfo serde, the serde frame walk,
the chunk engine's ChunkMeta codec, the checksum algebra) and the CPU oracle
(oracle/crc_oracle.c), all compiled with -fsanitize=address,undefined, and feeds them
truncated, oversize and random inputs.  No GPU: it runs in the CPU suite."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    out = tmp_path_factory.mktemp("san")
    orc = str(out / "crc_oracle.o")
    subprocess.check_call(["gcc", "-std=c11", "-pthread", *SAN, "-c", os.path.join(REPO, "oracle", "crc_oracle.c"),
                           "-o", orc])
    exe = str(out / "fuzz_host_codec")
    subprocess.check_call(["g++", "-std=c++17", "-pthread", *SAN, os.path.join(REPO, "tests", "cpp", "fuzz_host_codec.cpp"),
                           os.path.join(REPO, "3fs_amd", "csrc", "host_codec.cc"), orc, "-o", exe])
    return exe


def test_host_codec_and_oracle_under_asan_ubsan(fuzz_bin):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("LD_PRELOAD", None)  # the sanitizer runtime must come first in the process
    r = subprocess.run([fuzz_bin], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert '"fuzz_host_codec":"ok"' in r.stdout, r.stdout
