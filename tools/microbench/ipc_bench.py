"""IPC collective latency table: ``python tools/microbench/ipc_bench.py N`` runs N ranks sharing
the GPU (tests/ipc_checks.py:bench_ipc) and prints rank 0's JSON lines."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests._dist import run_distributed  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
outs = run_distributed("tests.ipc_checks:bench_ipc", n, timeout=300, keep_gpu=True)
print("\n".join(l for l in outs[0].splitlines() if l.startswith("{")))
