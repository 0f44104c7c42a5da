"""
SPMD launcher: ``python -m heat_amd.run -n 8 script.py [args]`` (or ``-m module``).

Starts one process per rank (one per MI355X when GPUs are present) with the standard rendezvous
environment (RANK, WORLD_SIZE, LOCAL_RANK, LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT);
``import heat_amd`` in each process initialises the process group (RCCL for device buffers, gloo
for host buffers). Replaces ``mpirun`` of the reference's workflow. Children are started as
subprocesses (never exec), their output is prefixed with the rank, and the first failing rank
terminates the job.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading


def free_port() -> int:
    """A bindable port BELOW the kernel's ephemeral range (32768+ on Linux): a port the OS hands
    out for bind(0) can be taken again, before rank 0 listens on it, as the source port of some
    outgoing connection (gloo opens many) - random picks from 15000-32767 cannot."""
    import random

    rng = random.Random()
    for _ in range(64):
        port = rng.randrange(15000, 32768)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", port))
            except OSError:
                continue
            return port
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pump(stream, rank: int, out, prefix: bool):
    for line in iter(stream.readline, b""):
        text = line.decode(errors="replace")
        out.write("[{}] {}".format(rank, text) if prefix else text)
        out.flush()



def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="python -m heat_amd.run", description=__doc__.splitlines()[1])
    p.add_argument("-n", "--nprocs", type=int, default=1, help="number of ranks (processes)")
    p.add_argument("--port", type=int, default=0, help="rendezvous port (default: a free one)")
    p.add_argument("--backend", default=None, choices=[None, "rccl", "gloo", "mixed"],
                   help="force the communication backend (HEAT_COMM_BACKEND)")
    p.add_argument("--no-prefix", action="store_true", help="do not prefix output lines with the rank")
    p.add_argument("-m", dest="module", default=None, help="run a module instead of a script")
    p.add_argument("target", nargs="?", help="script to run")
    p.add_argument("args", nargs=argparse.REMAINDER)
    ns = p.parse_args(argv)
    if ns.module is None and ns.target is None:
        p.error("a script or -m module is required")
    port = ns.port or free_port()
    cmd_tail = (["-m", ns.module] + ([ns.target] if ns.target else []) if ns.module else [ns.target]) + ns.args
    procs = []
    for r in range(ns.nprocs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(ns.nprocs), "LOCAL_RANK": str(r),
                    "LOCAL_WORLD_SIZE": str(ns.nprocs), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if ns.backend:
            env["HEAT_COMM_BACKEND"] = ns.backend
        procs.append(subprocess.Popen([sys.executable] + cmd_tail, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, start_new_session=True))
    threads = [threading.Thread(target=_pump, args=(pr.stdout, r, sys.stdout, not ns.no_prefix), daemon=True)
               for r, pr in enumerate(procs)]
    for t in threads:
        t.start()
    rc = 0
    try:
        alive = list(range(ns.nprocs))
        while alive:
            for r in list(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.remove(r)
                if code != 0 and rc == 0:
                    rc = code
                    for q in alive:
                        try:
                            os.killpg(procs[q].pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
            if alive:
                procs[alive[0]].wait(timeout=None) if len(alive) == 1 else threading.Event().wait(0.05)
    except KeyboardInterrupt:
        for pr in procs:
            try:
                os.killpg(pr.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        rc = 130
    for t in threads:
        t.join(timeout=1)
    return rc


if __name__ == "__main__":
    sys.exit(main())
