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
SOURCES = ["crc_kernels.hip", "update_kernels.hip", "digest_kernels.hip", "hf3fs_crc_api.hip",
           "coalescer.hip", "aux_kernels.hip", "frame_kernels.hip", "host_codec.cc", "options.cc"]
HEADERS = ["crc_kernels.h", "crc_device.h", "update_kernels.h", "digest_kernels.h", "gf2.h", "internal.h", "aux_kernels.h", "frame_kernels.h", "options.h"]
ARCH = os.environ.get("HF3FS_CRC_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(args):
    cmd, verbose = args
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)


def build(force=False, verbose=False):
    """Each source to an object in parallel (hipcc -c, only the stale ones), then one link."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(REPO, "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    common = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "hf3fs_crc.h"), __file__]
    flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result", "-I", os.path.join(REPO, "include")]
    objs, jobs = [], []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + common):
            jobs.append((["hipcc", f"--offload-arch={ARCH}"] + flags + ["-c", src, "-o", obj], verbose))
    if jobs:
        with ThreadPoolExecutor(max_workers=min(len(jobs), os.cpu_count() or 4)) as ex:
            list(ex.map(_compile, jobs))
    if not force and not jobs and not _stale(LIB, objs):
        return LIB
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return LIB




CPP_DIR = os.path.join(REPO, "tests", "cpp")
CPP_TEST_BIN = os.path.join(CPP_DIR, "test_checksuminfo")
CPP_BENCH_COALESCER = os.path.join(CPP_DIR, "bench_coalescer")
CPP_TEST_STAGING = os.path.join(CPP_DIR, "test_staging")
CPP_BENCH_READ = os.path.join(CPP_DIR, "bench_read_batch")
CPP_PROGRAMS = [CPP_TEST_BIN, CPP_BENCH_COALESCER, CPP_TEST_STAGING, CPP_BENCH_READ]
HIP_PROGRAMS = {CPP_TEST_STAGING}  # carry a probe kernel of their own: compiled by hipcc


def build_cpp_tests(force=False, verbose=False):
    """Host-code C++ programs linked against libhf3fs_crc.so with the CPU oracle
    as their checker: the ChecksumInfo drop-in test and the coalescer bench."""
    lib = build(verbose=verbose)
    oracle_c = os.path.join(REPO, "oracle", "crc_oracle.c")
    headers = [os.path.join(REPO, "include", "hf3fs", "storage", "ChecksumInfo.h"),
               os.path.join(REPO, "include", "hf3fs_crc.h")]
    stale = [b for b in CPP_PROGRAMS if force or _stale(b, [b + ".cpp", oracle_c, lib] + headers)]
    if not stale:
        return CPP_TEST_BIN
    obj = os.path.join(CPP_DIR, "_oracle.o")
    subprocess.check_call(["gcc", "-O2", "-fPIC", "-std=c11", "-c", oracle_c, "-o", obj])
    try:
        for b in stale:
            if b in HIP_PROGRAMS:
                cc = ["hipcc", f"--offload-arch={ARCH}", "-O2", "-std=c++20", "-x", "hip", b + ".cpp", "-x", "none"]
            else:
                cc = ["g++", "-O2", "-std=c++20", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", b + ".cpp"]
            cmd = cc + ["-o", b, obj, f"-L{LIBDIR}", "-lhf3fs_crc", f"-Wl,-rpath,{LIBDIR}", "-L/opt/rocm/lib",
                        "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-pthread"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.check_call(cmd)
    finally:
        os.remove(obj)
    return CPP_TEST_BIN


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_cpp_tests(force="--force" in sys.argv, verbose=True))
