"""Build libhf3fs_crc.so (gfx950) in-tree with hipcc.

The library is plain HIP C++ behind a C ABI; no torch extension machinery is
involved.  Output: 3fs_amd/lib/libhf3fs_crc.so (git-ignored, travels to the GPU
box with the gpurun snapshot).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libhf3fs_crc.so")
SOURCES = ["crc_kernels.hip", "update_kernels.hip", "hf3fs_crc_api.hip"]
HEADERS = ["crc_kernels.h", "update_kernels.h", "gf2.h"]
ARCH = os.environ.get("HF3FS_CRC_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "hf3fs_crc.h"), __file__]
    if not force and not _stale(LIB, deps):
        return LIB
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-result", "-I", os.path.join(REPO, "include"), "-o", LIB] + srcs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
