"""Host AddressSanitizer run of the native library (SURVEY 5.2 "optional HIP address sanitizer
builds of the native extension"). GPU ASan is not available on the test pool, so every kernel
source is compiled with ``-fsanitize=address`` on the HOST side only (``-Xarch_host``) into a
separate ``libheat_amd_kernels_asan.so`` (cached under ``heat_amd/ops/_lib/asan``), and
``tools/asan/host_abi_check.cpp`` - itself ASan-instrumented - drives every host-only entry
point (workspace / capacity calculators over many shapes) and the launch wrappers' argument
rejection paths. Any heap / stack / global overflow or use-after-free in that host code aborts the
driver with an ASan report."""
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from heat_amd.ops import _build

ASAN_DIR = os.path.join(_build.LIBDIR, "asan")
ASAN_LIB = os.path.join(ASAN_DIR, "libheat_amd_kernels_asan.so")
DRIVER_SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "asan",
                          "host_abi_check.cpp")
DRIVER = os.path.join(ASAN_DIR, "host_abi_check")
HOST_ASAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]


def _stale(target, deps):
    return not os.path.exists(target) or any(os.path.getmtime(d) > os.path.getmtime(target) for d in deps)


def _build_asan():
    hipcc = _build.hipcc()
    obj_dir = os.path.join(ASAN_DIR, "obj")   # per-source objects: only changed sources recompile
    os.makedirs(obj_dir, exist_ok=True)
    deps = _build.sources() + _build.headers() + [__file__]
    if _stale(ASAN_LIB, deps):
        flags = ["--offload-arch=" + _build.ARCH, "-O1", "-g", "-std=c++17", "-fPIC", "-Wno-unused-value",
                 "-Wno-unused-result", "-I" + _build.CSRC] + HOST_ASAN
        objs = [os.path.join(obj_dir, os.path.basename(s) + ".o") for s in _build.sources()]
        common = _build.headers() + [__file__]
        todo = [(src, obj) for src, obj in zip(_build.sources(), objs) if _stale(obj, [src] + common)]

        def cc(so):
            src, obj = so
            subprocess.run([hipcc] + flags + _build.file_flags(src) + ["-c", src, "-o", obj + ".part"], check=True,
                           capture_output=True)
            os.replace(obj + ".part", obj)

        jobs = max(1, min(max(len(todo), 1), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 16))
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(cc, todo))
        subprocess.run([hipcc, "--offload-arch=" + _build.ARCH, "-shared", "-fPIC"] + HOST_ASAN + objs +
                       ["-ldl", "-o", ASAN_LIB], check=True, capture_output=True)
    if _stale(DRIVER, [ASAN_LIB, DRIVER_SRC]):
        # the driver is plain host C++ (ROCm's clang, the same ASan runtime as the library's host code)
        clang = os.path.join(os.path.dirname(os.path.realpath(hipcc)), "..", "lib", "llvm", "bin", "clang++")
        if not os.path.exists(clang):
            clang = "/opt/rocm/lib/llvm/bin/clang++"
        subprocess.run([clang, "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer", DRIVER_SRC, ASAN_LIB,
                        "-Wl,-rpath," + ASAN_DIR, "-ldl", "-o", DRIVER], check=True, capture_output=True)


@pytest.mark.timeout(1200)
def test_native_host_code_under_asan():
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    try:
        _build_asan()
    except subprocess.CalledProcessError as e:
        pytest.fail("ASan build failed:\n" + (e.stderr or b"").decode()[-3000:])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    res = subprocess.run([DRIVER], env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0 and "asan host check ok" in res.stdout, res.stdout[-3000:] + res.stderr[-6000:]
    assert "AddressSanitizer" not in res.stderr, res.stderr[-6000:]
