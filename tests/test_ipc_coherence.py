"""The xGMI IPC kernels rely on system-scope fences for the coherence of their coarse-grained data
slots (``ops/csrc/ipc_allreduce.hip``, header comment): the writer's release must write its L2
back and the reader's acquire must invalidate its L2. This compiles the file for gfx950 on the CPU
and checks every IPC kernel's assembly for that pair (no GPU needed)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "heat_amd", "ops", "csrc", "ipc_allreduce.hip")


def _hipcc():
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    return None


@pytest.mark.skipif(_hipcc() is None, reason="hipcc not available")
def test_ipc_kernels_write_back_and_invalidate_l2(tmp_path):
    out = tmp_path / "ipc.s"
    subprocess.run([_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.dirname(SRC),
                    "--cuda-device-only", "-S", "-o", str(out), SRC], check=True, capture_output=True)
    asm = out.read_text()
    # split into functions at their entry labels
    funcs = re.split(r"\n(?=_Z\S*ipc_\S*:\s*(?:;.*)?\n)", asm)
    kernels = [f for f in funcs if re.match(r"_Z\S*ipc_", f)]
    assert len(kernels) >= 3 * 7 * 2, len(kernels)   # 3 dtypes x world 2..8 x (one-/two-shot) at least
    for body in kernels:
        name = body.split(":", 1)[0]
        wb = body.count("buffer_wbl2 sc0 sc1")
        inv = body.count("buffer_inv sc0 sc1")
        assert wb >= 1 and inv >= 1, (name, wb, inv)
