"""Multi-process test harness: run a check function in N ranks over gloo on 127.0.0.1.

``run_distributed("tests.dist_checks:check_x", 3)`` starts N fresh interpreters with the
launcher environment (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT); each imports heat_amd,
which initialises the process group, then runs the function. Any rank failing fails the test.
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    from heat_amd.run import free_port

    return free_port()


def run_distributed(target: str, nprocs: int, timeout: int = 300, env_extra=None, keep_gpu: bool = False):
    """``keep_gpu``: the ranks keep the visible GPU(s) (several ranks may share one device; the
    control plane stays gloo)."""
    port = _free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(nprocs),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HEAT_COMM_BACKEND": "gloo",
                    "OMP_NUM_THREADS": "1", "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
        if not keep_gpu:
            env.update({"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen([sys.executable, "-m", "tests._dist_runner", target], cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs, failed = [], []
    for r, p in enumerate(procs):
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("distributed test {} timed out on rank {}".format(target, r))
        outs.append(out.decode(errors="replace"))
        if p.returncode != 0:
            failed.append(r)
    if failed:
        msg = "\n".join("----- rank {} -----\n{}".format(r, outs[r][-6000:]) for r in failed)
        raise AssertionError("distributed test {} failed on ranks {}\n{}".format(target, failed, msg))
    return outs


def run_distributed_batch(module: str, names, nprocs: int, timeout: int = 1200, env_extra=None,
                          keep_gpu: bool = False):
    """Run the check functions ``names`` of ``module`` in one job of ``nprocs`` ranks; returns
    {name: (ok, error)} (checks missing from the report - a job that died - count as failed).
    A job whose rendezvous port was taken by a concurrent job (pytest -n) is started again."""
    for attempt in range(3):
        res = _run_batch_once(module, names, nprocs, timeout, env_extra, keep_gpu)
        if not any("EADDRINUSE" in (err or "") for ok, err in res.values() if not ok):
            break
    return res


def _run_batch_once(module, names, nprocs, timeout, env_extra, keep_gpu):
    import json
    import tempfile

    port = _free_port()
    fd, out_path = tempfile.mkstemp(suffix=".jsonl")
    os.close(fd)
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(r), "LOCAL_WORLD_SIZE": str(nprocs),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "HEAT_COMM_BACKEND": "gloo",
                    "HEAT_COMM_TIMEOUT": "120", "OMP_NUM_THREADS": "1",
                    "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
        if not keep_gpu:
            env.update({"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen([sys.executable, "-m", "tests._dist_batch_runner", out_path, module] + list(names),
                                      cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            out = b"timeout"
        logs.append(out.decode(errors="replace"))
    res = {}
    with open(out_path) as f:
        for line in f:
            rec = json.loads(line)
            res[rec["name"]] = (rec["ok"], rec["error"])
    os.unlink(out_path)
    tail = "\n".join(l[-2000:] for l in logs)
    for n in names:
        res.setdefault(n, (False, "job ended before this check ran:\n" + tail))
    return res
