"""
Build the native CDNA4 kernel library in-tree:
``hipcc --offload-arch=gfx950 -O3 -fPIC -c`` per ``heat_amd/ops/csrc/*.hip`` (in parallel), linked into
``heat_amd/ops/_lib/libheat_amd_kernels.so``.

The library exports a plain C ABI (``ha_*`` functions taking device pointers and a ``hipStream_t``)
and is loaded with ctypes after torch, so it shares torch's HIP runtime (same SONAME
``libamdhip64.so.7``) and runs on torch's current stream. No torch headers are compiled, so a
full rebuild takes seconds and cross-compiles without a GPU.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIBNAME = "libheat_amd_kernels.so"
LIBPATH = os.path.join(LIBDIR, LIBNAME)
ARCH = os.environ.get("HEAT_AMD_ARCH", "gfx950")


def sources():
    """The ``.hip`` kernel sources compiled into the library."""
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def headers():
    """The shared ``.h`` headers of the kernel sources."""
    return sorted(glob.glob(os.path.join(CSRC, "*.h")))


def file_flags(src: str) -> list:
    """Extra per-source flags from a ``// hipcc-flags: ...`` line in the file's first 40 lines
    (e.g. ``-fno-slp-vectorize`` for MFMA kernels: SLP-packed f32 VALU beside MFMAs costs ~5x a
    scalar op's issue slot on gfx950)."""
    with open(src) as f:
        for _, line in zip(range(40), f):
            if line.startswith("// hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def hipcc() -> str:
    """Path of the hipcc compiler (``$HIPCC``, PATH, then /opt/rocm/bin)."""
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found; the native kernels need ROCm's hipcc")


def stale_sources() -> list:
    """Sources / headers (and this script) newer than the built library."""
    if not os.path.exists(LIBPATH):
        return sources() + headers()
    t = os.path.getmtime(LIBPATH)
    return [s for s in sources() + headers() + [__file__] if os.path.getmtime(s) > t]


def needs_build() -> bool:
    """True when the library is missing or older than a source, a header or this build script."""
    return bool(stale_sources())


OBJDIR = os.path.join(LIBDIR, "obj")  # per-source object cache (git- and gpurun-ignored)


def _stale_objects(objs, flags) -> list:
    """Indices of the sources whose cached object is missing or older than the source, a header
    or this script, or was compiled with other flags."""
    stamp = os.path.join(OBJDIR, "flags.txt")
    same_flags = os.path.exists(stamp) and open(stamp).read() == " ".join(flags)
    dep_t = max([os.path.getmtime(h) for h in headers()] + [os.path.getmtime(__file__)])
    out = []
    for i, (src, obj) in enumerate(zip(sources(), objs)):
        if not same_flags or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), dep_t):
            out.append(i)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile the kernels into one shared library (atomic replace) and return its path. Sources
    whose cached object is current are not recompiled unless ``force``."""
    if not force and not needs_build():
        return LIBPATH
    os.makedirs(OBJDIR, exist_ok=True)
    fd, tmp = tempfile.mkstemp(suffix=".so", dir=LIBDIR)
    os.close(fd)
    flags = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-Wno-unused-value", "-Wno-unused-result",
             "-I" + CSRC]

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True, capture_output=not verbose)

    # one hipcc per stale source in parallel (the template-heavy kernel files dominate a serial build)
    objs = [os.path.join(OBJDIR, os.path.basename(src) + ".o") for src in sources()]
    todo = list(range(len(objs))) if force else _stale_objects(objs, flags)
    jobs = max(1, min(max(len(todo), 1), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 16))
    srcs = sources()

    def compile_one(i):
        part = objs[i] + ".part"
        run([hipcc()] + flags + file_flags(srcs[i]) + ["-c", srcs[i], "-o", part])
        os.replace(part, objs[i])

    try:
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(compile_one, todo))
        with open(os.path.join(OBJDIR, "flags.txt"), "w") as f:
            f.write(" ".join(flags))
        run([hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC"] + objs + ["-ldl", "-o", tmp])
    except subprocess.CalledProcessError as e:
        os.unlink(tmp)
        msg = e.stderr.decode() if e.stderr else ""
        src = next((a for a in e.cmd if str(a).endswith(".hip")), None)
        where = " ({})".format(os.path.basename(src)) if src else ""
        raise RuntimeError("building the native kernels failed{}:\n{}".format(where, msg)) from e
    os.replace(tmp, LIBPATH)
    return LIBPATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
