"""Latency of the one-shot IPC all-reduce (``parallel/ipc.py``) per call, ranks sharing one GPU
(what a 1-GPU box can measure: the handshake + copy + sum kernel, not xGMI link time).

Run: ``python tools/microbench/ipc_bench.py`` (spawns the ranks itself, gloo control plane)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rank_main():
    import torch

    import heat_amd as ht
    from heat_amd.parallel.ipc import IpcAllreduce

    comm = ht.MPI_WORLD
    ar = IpcAllreduce(comm, capacity_bytes=4 << 20, blocks=32)
    dev = torch.device("cuda", torch.cuda.current_device())
    res = {}
    for name, n, dt in (("8B f64", 1, torch.float64), ("64KB f32", 16384, torch.float32),
                        ("532KB f64 (k-means k=1024 f=64)", 1024 * 65, torch.float64),
                        ("4MB f32", 1 << 20, torch.float32)):
        t = torch.ones(n, dtype=dt, device=dev)
        for _ in range(20):
            ar.allreduce_(t)
        torch.cuda.synchronize()
        comm.Barrier()
        reps = 300
        t0 = time.perf_counter()
        for _ in range(reps):
            ar.allreduce_(t)
        torch.cuda.synchronize()
        dt_us = (time.perf_counter() - t0) / reps * 1e6
        res[name] = round(comm.allreduce(dt_us, ht.MPI.MAX), 2)
    assert ar.error() == 0
    if comm.rank == 0:
        print(json.dumps({"bench": "ipc_allreduce_us_per_call", "ranks": comm.size, "shared_gpu": True, **res}))
    ar.close()


def main():
    nprocs = int(os.environ.get("IPC_BENCH_RANKS", "2"))
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(nprocs),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HEAT_COMM_BACKEND="gloo",
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank"], env=env))
    rc = 0
    for p in procs:
        rc |= p.wait(timeout=300)
    sys.exit(rc)


if __name__ == "__main__":
    if "--rank" in sys.argv:
        rank_main()
    else:
        main()
