#!/usr/bin/env python
"""
Flagship benchmark: one k-means Lloyd iteration (assign + update + all-reduce) on split=0 float32
data, the BASELINE.json config "k-means k=1024 on 1e8 x 64 float32 split=0, 8 x MI355X".

Weak scaling: every GPU holds ``--n-per-gpu`` points (default 1.25e7, so 8 GPUs = 1e8 points).
Data are synthetic (Threefry normal samples generated on the device, random-init centroids).
``value`` is the whole-job GFLOP/s of the distance computation (2*n*k*f per iteration, the
quantity the reference's benchmark scales with); ``ms_per_step`` the wall time of one iteration.

Run: ``python bench.py`` (1 GPU), ``python bench.py --gpus N`` (starts N rank processes itself) or
``torchrun --nproc-per-node N bench.py --gpus N`` (WORLD_SIZE must equal ``--gpus``).
``--comm {pg,native,ipc}`` picks the device collective path of the timed loop, ``--ring
{ring,direct}`` the Y-block circulation; at world > 1 the k-means all-reduce payload is also timed
on every path (``extra.comm_ab``) and ``extra.comm.collective_paths`` counts the path each
collective of the run took.
Secondary workloads: ``--workload cdist`` (distance_matrix, streamed), ``--workload knn`` (the
distance_matrix config reduced to each row's ``--topk`` nearest rows by the fused kernel, no
matrix), ``--workload moments`` (statistical_moments mean/var of 1e9 float32) and ``--workload qr``
(the tall-skinny QR config: ht.linalg.qr of 1.25e6 x 4096 float32 per GPU, split=0, Q and R).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="kmeans", choices=["kmeans", "cdist", "knn", "moments", "qr"])
    p.add_argument("--n-per-gpu", type=int, default=None,
                   help="kmeans: points per GPU (1.25e7); moments: elements per GPU (1e9)")
    p.add_argument("--rows", type=int, default=1_000_000, help="cdist: total rows (strong scaling)")
    p.add_argument("--k", type=int, default=1024)
    p.add_argument("--topk", type=int, default=8, help="knn: neighbours per row")
    p.add_argument("--f", type=int, default=None, help="features (kmeans 64, cdist 128)")
    p.add_argument("--precision", default="fast", choices=["fast", "exact"],
                   help="kmeans: 'fast' = distances by a 3-term fp16 split on the matrix cores (fp32-GEMM "
                        "accuracy, checked against fp64 in tests/test_gpu_kernels.py); 'exact' = fp32-input MFMA")
    p.add_argument("--exact-steps", type=int, default=5,
                   help="kmeans fast: also time this many steps of the exact fp32-MFMA path (0 = skip)")
    p.add_argument("--with-reference", action="store_true",
                   help="also time a reference-style (heat 1.1 algorithm) iteration on torch-ROCm")
    p.add_argument("--comm", default="pg", choices=["pg", "native", "ipc"],
                   help="device collectives of the timed loop: torch ProcessGroupNCCL (RCCL), the native "
                        "stream-ordered RCCL communicator (comm.hip) or the xGMI IPC kernels (ipc_allreduce.hip)")
    p.add_argument("--ring", default="ring", choices=["ring", "direct"],
                   help="Y-block circulation of the cdist/knn workloads: neighbour ring or all-peer direct posts")
    p.add_argument("--comm-ab", type=int, default=1,
                   help="world > 1: also time the k-means all-reduce payload on every comm path after the timed "
                        "loop (0 = skip), in a separate child job so a failing path cannot cost the result")
    p.add_argument("--comm-ab-child", default=None, help=argparse.SUPPRESS)
    return p.parse_args()


def _free_port() -> int:
    """A bindable rendezvous port below Linux's ephemeral range (heat_amd.run.free_port; not
    imported from there: importing heat_amd in the launcher would initialise the GPU)."""
    import random
    import socket

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


def launch_or_check(args) -> int:
    """Rank bookkeeping BEFORE anything touches the GPU (no torch.cuda call other than
    device_count here, never exec): -1 = this process is a rank, go on; else an exit code.

    * under a launcher (WORLD_SIZE set) the launcher's world must equal ``--gpus``;
    * without one, ``--gpus N > 1`` starts N rank processes itself (subprocesses with
      RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* = 127.0.0.1), relays rank 0's stdout, and fails if any
      rank fails (the first failure terminates the others)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print("bench.py: --gpus {} but the launcher started WORLD_SIZE={} ranks".format(args.gpus, ws),
                  file=sys.stderr, flush=True)
            return 2
        return -1
    if args.gpus <= 1:
        return -1
    ndev = torch.cuda.device_count()  # does not initialise HIP on this image
    if 0 < ndev < args.gpus and not shared_gpu():
        print("bench.py: --gpus {} but only {} GPUs are visible (HEAT_BENCH_SHARED_GPU=1 runs the ranks on "
              "shared GPUs over gloo, as a rehearsal, never a scaling point)".format(args.gpus, ndev),
              file=sys.stderr, flush=True)
        return 2
    import signal
    import subprocess
    import threading

    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE, start_new_session=True))

    def relay(r, pr):
        for line in iter(pr.stdout.readline, b""):
            if r == 0:
                sys.stdout.write(line.decode(errors="replace"))
                sys.stdout.flush()
            else:
                sys.stderr.write("[rank {}] {}".format(r, line.decode(errors="replace")))

    pumps = [threading.Thread(target=relay, args=(r, pr), daemon=True) for r, pr in enumerate(procs)]
    for t in pumps:
        t.start()
    rc, alive = 0, set(range(args.gpus))
    while alive:
        for r in sorted(alive):
            code = procs[r].poll()
            if code is None:
                continue
            alive.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print("bench.py: rank {} exited with {}; stopping the others".format(r, code), file=sys.stderr,
                      flush=True)
                for q in alive:
                    try:
                        os.killpg(procs[q].pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        if alive:
            time.sleep(0.05)
    for t in pumps:
        t.join(timeout=5)
    return rc


def shared_gpu() -> bool:
    """``HEAT_BENCH_SHARED_GPU=1``: a rehearsal of an N-rank job on fewer GPUs (ranks share a
    device; RCCL refuses two ranks on one GPU, so the world group is gloo and device buffers are
    host-staged). Every code path of the N-rank job runs, but the timing is NOT a scaling point:
    the record says ``shared_gpu: true``."""
    return os.environ.get("HEAT_BENCH_SHARED_GPU", "0") == "1"


def apply_comm_env(args) -> None:
    """Select the collective paths of this rank before ``heat_amd`` is imported."""
    if shared_gpu():
        os.environ["HEAT_COMM_BACKEND"] = "gloo"
    os.environ["HEAT_COMM_NATIVE"] = "1" if args.comm == "native" else os.environ.get("HEAT_COMM_NATIVE", "0")
    os.environ["HEAT_IPC_ALLREDUCE"] = "1" if args.comm == "ipc" else os.environ.get("HEAT_IPC_ALLREDUCE", "0")
    os.environ["HEAT_RING_MODE"] = args.ring


def main():
    args = parse()
    rc = launch_or_check(args)
    if rc >= 0:
        sys.exit(rc)
    apply_comm_env(args)
    if args.comm_ab_child:
        comm_ab_child(args.comm_ab_child)
        return
    import heat_amd as ht
    from heat_amd.core.communication import MPI_WORLD

    comm = MPI_WORLD
    if torch.cuda.is_available():
        ht.use_device("gpu")
    dev = ht.get_device()

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        comm.Barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    n_gpus = comm.size
    extra = {"world_size_seen_by_rccl": rccl_world_size(comm)}
    scaling = "weak"
    if args.workload == "kmeans":
        # 1.25e7 points per GPU (8 GPUs = the BASELINE's 1e8); a CPU-only host (the gloo contract
        # tests, no GPU) defaults to 2^16 so that a plain ``--gpus N`` finishes in seconds
        args.n_per_gpu = args.n_per_gpu or (12_500_000 if torch.cuda.is_available() else 1 << 16)
        n, k, f = args.n_per_gpu * n_gpus, args.k, args.f or 64
        ht.random.seed(1234)
        x = ht.random.randn(n, f, split=0, device=dev)
        km = ht.cluster.KMeans(n_clusters=k, init="random", max_iter=1, tol=None, random_state=42)
        km.precision = args.precision
        for _ in range(args.warmup):
            km.step(x)
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            km.step(x)
        sync()
        dt = time.perf_counter() - t0
        # slowest rank defines the step
        ms = rank_times(comm, dt, args.steps, extra)
        flops = 2.0 * n * k * f
        value = flops / (ms * 1e-3) / 1e9
        metric = "kmeans_iter_gflops"
        unit = "GFLOP/s"
        cfg = {"model": "kmeans k={} f={} float32 split=0 (assign+update+allreduce)".format(k, f),
               "precision": args.precision,
               "global_batch": n, "seq_len": f, "parallelism": "dp{}".format(n_gpus), "k": k,
               "n_per_gpu": args.n_per_gpu}
        extra["iter_ms"] = ms
        extra["precision"] = ("fp32 data and centroids; distance GEMM as a 3-term fp16 split with fp32 "
                              "accumulation (fp32-GEMM accuracy, per-row power-of-two scales for points "
                              "AND centroids); value is an fp32-EQUIVALENT rate (2*n*k*f per iteration), "
                              "not an fp32-MFMA rate" if args.precision == "fast"
                              else "fp32-input MFMA (exact fp32 products)")
        extra["tflops_per_gpu"] = value / n_gpus / 1e3
        if args.precision == "fast" and args.exact_steps > 0:
            # the exact fp32-MFMA path on the same data, for an honest side-by-side
            km_exact = ht.cluster.KMeans(n_clusters=k, init="random", max_iter=1, tol=None, random_state=42)
            km_exact.precision = "exact"
            for _ in range(2):
                km_exact.step(x)
            sync()
            t0 = time.perf_counter()
            for _ in range(args.exact_steps):
                km_exact.step(x)
            sync()
            dte = time.perf_counter() - t0
            dte = comm.allreduce(dte, ht.MPI.MAX) if comm.size > 1 else dte
            extra["exact_ms_per_step"] = dte / args.exact_steps * 1e3
            extra["exact_gflops_fp32"] = flops / (extra["exact_ms_per_step"] * 1e-3) / 1e9
        extra.update(validate_kmeans(km, x, comm, k))
        if args.with_reference:
            extra["reference_impl_ms"] = reference_iteration(x, km, k)
            extra["speedup_vs_reference_impl"] = extra["reference_impl_ms"] / ms
    elif args.workload == "cdist":
        # BASELINE distance_matrix config: 1e6 x 128 vs itself (strong scaling). The 4 TB fp32
        # matrix cannot be held, so it is produced tile by tile (65536^2 tiles, MFMA quadratic
        # expansion kernel with fused sqrt epilogue) into a reused HBM buffer; Y blocks circulate
        # around the ring. Every one of the n*n distances is computed and stored each step.
        n, f = args.rows, args.f or 128
        ht.random.seed(7)
        x = ht.random.rand(n, f, split=0, device=dev)
        tiles = [0]

        def consume(d, i, j):
            tiles[0] += 1

        def one():
            ht.spatial.cdist_stream(x, x, consume, tile=65536)

        for _ in range(args.warmup):
            one()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one()
        sync()
        dt = time.perf_counter() - t0
        ms = rank_times(comm, dt, args.steps, extra)
        value = 2.0 * n * n * f / (ms * 1e-3) / 1e9
        metric, unit = "cdist_gflops", "GFLOP/s"
        cfg = {"model": "cdist euclidean n={} f={} float32 split=0 (streamed tiles)".format(n, f),
               "global_batch": n, "seq_len": f, "parallelism": "dp{}".format(n_gpus)}
        extra["flop_convention"] = "2*n*n*f (the distance GEMM of the quadratic expansion)"
        extra["distances_per_s"] = n * n / (ms * 1e-3)
        extra.update(validate_cdist(x, comm))
        scaling = "strong"
    elif args.workload == "knn":
        # the same 1e6 x 128 self-distance problem, each row reduced to its topk nearest rows by the
        # fused MFMA distance + register top-k kernel (Y blocks around the ring; no distance matrix)
        n, f = args.rows, args.f or 128
        ht.random.seed(7)
        x = ht.random.rand(n, f, split=0, device=dev)
        for _ in range(args.warmup):
            ht.spatial.cdist_topk(x, x, args.topk)
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            d, idx = ht.spatial.cdist_topk(x, x, args.topk)
        sync()
        dt = time.perf_counter() - t0
        ms = rank_times(comm, dt, args.steps, extra)
        value = 2.0 * n * n * f / (ms * 1e-3) / 1e9
        metric, unit = "knn_gflops", "GFLOP/s (fp32-equivalent)"
        cfg = {"model": "cdist_topk euclidean n={} f={} k={} float32 split=0".format(n, f, args.topk),
               "global_batch": n, "seq_len": f, "parallelism": "dp{}".format(n_gpus)}
        extra["flop_convention"] = "2*n*n*f (the distance GEMM of the quadratic expansion)"
        from heat_amd.ops import kernels as _k

        st = _k._KNN_STATS
        extra["certified_queries"] = st["queries"]
        extra["certified_rechecked_fraction"] = st["rechecked"] / st["queries"] if st["queries"] else None
        extra.update(validate_knn(x, d, idx, comm))
        scaling = "strong"
    elif args.workload == "qr":
        # BASELINE tall-skinny QR config: 1e7 x 4096 float32 split=0 on 8 GPUs = 1.25e6 rows per GPU
        # (weak scaling), ht.linalg.qr (CholeskyQR2: Gram + fp64 Cholesky + triangular-B products,
        # R replicated, Q split like A) at float32 matmul precision "highest" (exact fp32 products)
        args.n_per_gpu = args.n_per_gpu or (1_250_000 if torch.cuda.is_available() else 4096)
        f = args.f or (4096 if torch.cuda.is_available() else 64)
        n = args.n_per_gpu * n_gpus
        torch.set_float32_matmul_precision("highest")
        ht.random.seed(11)
        a = ht.random.randn(n, f, split=0, device=dev)
        q = r = None
        for _ in range(args.warmup):
            q = r = None
            q, r = ht.linalg.qr(a, mode="reduced")
        sync()
        t0 = time.perf_counter()
        q = r = None
        for _ in range(args.steps):
            q = r = None     # the previous step's 20 GB Q is released before the next is allocated
            q, r = ht.linalg.qr(a, mode="reduced")
        sync()
        dt = time.perf_counter() - t0
        ms = rank_times(comm, dt, args.steps, extra)
        flops = 4.0 * n * f * f - 4.0 * f ** 3 / 3
        value = flops / (ms * 1e-3) / 1e9
        metric, unit = "tsqr_gflops", "GFLOP/s"
        cfg = {"model": "tsqr Q,R m={} n={} float32 split=0 (CholeskyQR2)".format(n, f), "global_batch": n,
               "seq_len": f, "parallelism": "dp{}".format(n_gpus), "n_per_gpu": args.n_per_gpu}
        extra["flop_convention"] = "4 m n^2 - 4 n^3 / 3 (Householder QR with Q formed)"
        extra.update(validate_qr(a, q, r, comm))
    else:
        args.n_per_gpu = args.n_per_gpu or 1_000_000_000
        n = args.n_per_gpu * n_gpus
        x = ht.random.rand(n, split=0, device=dev)
        for _ in range(args.warmup):
            ht.mean(x), ht.var(x)
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            m = ht.mean(x)
            v = ht.var(x)
        sync()
        dt = time.perf_counter() - t0
        ms = rank_times(comm, dt, args.steps, extra)
        value = 2 * n * 4 / (ms * 1e-3) / 1e9
        metric, unit = "moments_GB_per_s", "GB/s"
        extra.update(validate_moments(x, m, v, comm))
        cfg = {"model": "mean+var float32 split=0", "global_batch": n, "seq_len": 1,
               "parallelism": "dp{}".format(n_gpus)}
    if args.workload == "kmeans" and args.precision == "fast":
        unit = "GFLOP/s (fp32-equivalent)"
    from heat_amd.core.communication import PATH_COUNTS
    from heat_amd.parallel.ring import PASSES

    extra["comm"] = {"requested": args.comm, "ring_mode": args.ring, "collective_paths": dict(PATH_COUNTS),
                     "ring_passes": dict(PASSES)}
    cfg["comm"] = args.comm
    if shared_gpu():
        # ranks time-share devices over a gloo world: a rehearsal of the N-rank paths, never a scaling point
        extra["shared_gpu"] = cfg["shared_gpu"] = True
        extra["devices_visible"] = torch.cuda.device_count()
    out = {"metric": metric, "value": value, "unit": unit, "n_gpus": n_gpus, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": scaling,
           "vs_baseline": None, "dtype": "fp32", "data": "synthetic (device Threefry normal samples)",
           "config": cfg, "extra": extra}
    if comm.size > 1 and args.comm_ab:
        # after the timed loop and its result: the all-reduce of the k-means payload on every
        # path, in a SEPARATE job (one child per rank, its own rendezvous): a path that crashes or
        # hangs on this node costs that record, never the measurement above
        payload = (args.k * (args.f or 64) + args.k) * 8
        extra["comm_ab"] = comm_ab_isolated(comm, [8, payload])
    if comm.rank == 0:
        print(json.dumps(out), flush=True)


def comm_ab_isolated(comm, sizes) -> dict:
    """Run :func:`comm_ab` in a child job of the same ranks (every rank starts one child with the
    launcher's RANK / WORLD_SIZE / LOCAL_RANK and a fresh MASTER_PORT from rank 0), bounded by
    ``HEAT_BENCH_AB_TIMEOUT`` seconds; rank 0's child prints the record."""
    import subprocess

    import heat_amd as ht

    port = None
    if comm.rank == 0:
        port = _free_port()
    port = comm.bcast(port, root=0)
    # a fresh rendezvous: not torchrun's agent store (TORCHELASTIC_USE_AGENT_STORE would make the
    # child connect to the agent's store on the new port, where nobody listens)
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC_")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(comm.rank), WORLD_SIZE=str(comm.size))
    env.setdefault("LOCAL_RANK", str(comm.rank))
    env.setdefault("LOCAL_WORLD_SIZE", str(comm.size))
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(comm.size), "--comm-ab-child",
           ",".join(str(x) for x in sizes)]
    res = {}
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True,
                           timeout=float(os.environ.get("HEAT_BENCH_AB_TIMEOUT", "120")))
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        if lines:
            res = json.loads(lines[-1])
        if r.returncode != 0:
            res["error"] = "child exited with {}: {}".format(r.returncode, r.stderr[-300:])
    except subprocess.TimeoutExpired:
        res = {"error": "timed out"}
    ok = comm.allreduce(int("error" not in res), ht.MPI.MIN)
    if not ok and "error" not in res:
        res["error"] = "failed on another rank"
    return res


def comm_ab_child(sizes) -> None:
    """Entry point of the isolated comm A/B job (``--comm-ab-child``)."""
    import heat_amd as ht
    from heat_amd.core.communication import MPI_WORLD

    if torch.cuda.is_available():
        ht.use_device("gpu")
    res = comm_ab(MPI_WORLD, None, [int(x) for x in sizes.split(",")])
    if MPI_WORLD.rank == 0:
        print(json.dumps(res), flush=True)


def comm_ab(comm, dev, sizes) -> dict:
    """Microseconds per all-reduce (SUM, fp64, max over ranks, 20 back-to-back calls after 3
    warm-up calls) of each payload in ``sizes`` bytes on each device path: torch ProcessGroup
    (RCCL via ProcessGroupNCCL, or gloo on a CPU job), the native RCCL communicator (``comm.hip``)
    and the xGMI IPC one-/two-shot kernels (``ipc_allreduce.hip``); every result is checked
    (sum of ones == world size). A path whose construction fails on any rank is skipped on all."""
    import torch.distributed as dist

    import heat_amd as ht

    res = {}
    reps = 20
    paths = [("pg", lambda b: dist.all_reduce(b))]
    if torch.cuda.is_available():
        from heat_amd.parallel import ipc as _ipc
        from heat_amd.parallel import native_comm as _nc

        def agree(make):
            obj, err = None, None
            try:
                obj = make()
            except Exception as e:  # noqa: BLE001 - reported, and the path skipped on every rank
                err = "{}: {}".format(type(e).__name__, e)[:300]
            ok = comm.allreduce(int(err is None), ht.MPI.MIN)
            return (obj if ok else None), err

        nc, err = agree(lambda: comm._native() or _nc.NativeComm(comm))
        if nc is not None:
            paths.append(("native", lambda b: nc.allreduce_(b, "sum")))
        else:
            res["native_error"] = err or "failed on another rank"
        ar, err = agree(lambda: getattr(comm, "_ipc", None) or _ipc.IpcAllreduce(comm, capacity_bytes=max(sizes)))
        if ar is not None:
            paths.append(("ipc", lambda b: ar.allreduce_(b)))
        else:
            res["ipc_error"] = err or "failed on another rank"
    device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    for name, fn in paths:
        for nbytes in sizes:
            buf = torch.ones(max(1, nbytes // 8), dtype=torch.float64, device=device)
            fn(buf)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            ok = bool((buf == comm.size).all())
            for _ in range(2):
                fn(buf)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            comm.Barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn(buf)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / reps * 1e6
            res["{}_{}B_us".format(name, nbytes)] = comm.allreduce(us, ht.MPI.MAX)
            res["{}_{}B_ok".format(name, nbytes)] = bool(comm.allreduce(int(ok), ht.MPI.MIN))
    return res


def validate_kmeans(km, x, comm, k: int) -> dict:
    """Self-check of the distributed step, outside the timed region: one more Lloyd step, then
    (1) its centroids recomputed in fp64 from its labels (index_add over the local points + one
    all-reduce) against the kernel path's centroids, (2) the all-reduced cluster counts summing to
    n, (3) a centroid checksum identical on every rank (MAX == MIN over the ranks), and (4) the
    time of the packed (k*f + k) fp64 all-reduce alone."""
    import heat_amd as ht

    X = x.larray
    c_prev = km.cluster_centers_.larray.clone()
    km.step(x)
    lab = km._last_labels.reshape(-1).long()
    c_new = km.cluster_centers_.larray
    f = X.shape[1]
    packed = torch.zeros(k * f + k, dtype=torch.float64, device=X.device)
    sums = packed[: k * f].view(k, f)
    sums.index_add_(0, lab, X.double())
    packed[k * f:].index_add_(0, lab, torch.ones_like(lab, dtype=torch.float64))
    if comm.size > 1:
        comm.Allreduce(ht.MPI.IN_PLACE, packed, ht.MPI.SUM)
    counts = packed[k * f:]
    ref = torch.where(counts.unsqueeze(1) > 0, sums / counts.clamp(min=1).unsqueeze(1), c_prev.double())
    scale = float(ref.abs().max()) or 1.0
    err = float((c_new.double() - ref).abs().max()) / scale
    chk = float((c_new.double() * torch.arange(1, c_new.numel() + 1, device=X.device,
                                                dtype=torch.float64).view_as(c_new)).sum())
    hi = comm.allreduce(chk, ht.MPI.MAX) if comm.size > 1 else chk
    lo = comm.allreduce(chk, ht.MPI.MIN) if comm.size > 1 else chk
    buf = torch.ones(k * f + k, dtype=torch.float64, device=X.device)
    reps = 20
    for _ in range(3):
        comm.Allreduce(ht.MPI.IN_PLACE, buf, ht.MPI.SUM)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    comm.Barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        comm.Allreduce(ht.MPI.IN_PLACE, buf, ht.MPI.SUM)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / reps * 1e6
    us = comm.allreduce(us, ht.MPI.MAX) if comm.size > 1 else us
    res = {"centroids_agree": hi == lo, "count_sum_ok": int(round(float(counts.sum()))) == x.gshape[0],
           "centroid_max_rel_err_vs_fp64": err, "allreduce_us": us,
           "allreduce_bytes": buf.numel() * buf.element_size()}
    res.update(check_labels(X, c_prev, lab, comm))
    return res


def check_labels(X, C, lab, comm, sample: int = 65536) -> dict:
    """The step's labels are the nearest centroids: a sample of every rank's points (evenly
    strided, ``sample`` in total per rank) against an fp64 argmin over the centroids the step
    used. A label counts as correct when it is the fp64 argmin, or ties it within fp32-GEMM
    accuracy: d(x, c_label) - d_min <= 4e-6 (|x|^2 + |c_label|^2 + |c_min|^2), the bound of
    tests/test_gpu_kernels.py:_local_minimality. ``label_agreement`` is the exact-match fraction,
    ``label_max_excess`` the largest (d_label - d_min) in units of that scale (<= 4e-6 passes)."""
    import heat_amd as ht

    n = X.shape[0]
    idx = torch.linspace(0, max(n - 1, 0), steps=min(sample, n), device=X.device).round().long() if n else \
        torch.zeros(0, dtype=torch.long, device=X.device)
    Xs, ls = X[idx].double(), lab[idx]
    Cd = C.double()
    cn = (Cd * Cd).sum(1)
    xn = (Xs * Xs).sum(1)
    agree, excess, total = 0.0, 0.0, float(idx.numel())
    for i in range(0, idx.numel(), 4096):
        xs = Xs[i: i + 4096]
        d = torch.cdist(xs, Cd) ** 2
        dmin, amin = d.min(1)
        li = ls[i: i + 4096]
        chosen = d.gather(1, li.unsqueeze(1)).squeeze(1)
        scale = xn[i: i + 4096] + cn[li] + cn[amin]
        agree += float((li == amin).sum())
        if xs.shape[0]:
            excess = max(excess, float(((chosen - dmin) / scale).max()))
    if comm.size > 1:
        agree = comm.allreduce(agree, ht.MPI.SUM)
        total = comm.allreduce(total, ht.MPI.SUM)
        excess = comm.allreduce(excess, ht.MPI.MAX)
    return {"label_agreement": agree / max(total, 1.0), "label_max_excess": excess,
            "labels_checked": int(total), "labels_ok": excess <= 4e-6}


def validate_qr(a, q, r, comm) -> dict:
    """The timed QR's factors against fp64, outside the timed region: orthogonality of the first
    64 columns of Q (Q[:, :64]^T Q[:, :64] summed over the ranks), the reconstruction Q R = A on the
    first 4096 local rows of every rank (relative to max |A|), R upper triangular."""
    import heat_amd as ht

    Q, A = q.larray, a.larray
    R = ht.resplit(r, None).larray if r.is_distributed() else r.larray
    G = Q[:, :64].double().T @ Q[:, :64].double()
    if comm.size > 1:
        comm.Allreduce(ht.MPI.IN_PLACE, G, ht.MPI.SUM)
    orth = float((G - torch.eye(G.shape[0], dtype=torch.float64, device=G.device)).abs().max())
    rows = min(4096, A.shape[0])
    rec = float((Q[:rows].double() @ R.double() - A[:rows].double()).abs().max() / A[:rows].abs().max()) if rows else 0.0
    rec = comm.allreduce(rec, ht.MPI.MAX) if comm.size > 1 else rec
    upper = bool(torch.equal(R, torch.triu(R)))
    return {"q_orth_err_64cols": orth, "qr_rec_rel_err": rec, "r_upper": upper,
            "qr_ok": bool(orth < 1e-4 and rec < 1e-4 and upper)}


def validate_moments(x, m, v, comm) -> dict:
    """Global mean / variance of the timed calls against an fp64 recompute (chunked sums over the
    local block + all-reduce), outside the timed region."""
    import heat_amd as ht

    X = x.larray.reshape(-1)
    step = 1 << 27
    s = torch.zeros(2, dtype=torch.float64, device=X.device)
    for i in range(0, X.numel(), step):
        s[0] += X[i: i + step].sum(dtype=torch.float64)
    if comm.size > 1:
        comm.Allreduce(ht.MPI.IN_PLACE, s, ht.MPI.SUM)
    n = x.gnumel
    mu = s[0] / n
    for i in range(0, X.numel(), step):
        s[1] += ((X[i: i + step].double() - mu) ** 2).sum()
    q = s[1:].clone()
    if comm.size > 1:
        comm.Allreduce(ht.MPI.IN_PLACE, q, ht.MPI.SUM)
    var = float(q[0]) / n
    return {"mean_abs_err_vs_fp64": abs(float(m.item()) - float(mu)),
            "var_rel_err_vs_fp64": abs(float(v.item()) - var) / max(abs(var), 1e-300)}


def validate_cdist(x, comm) -> dict:
    """Distances of a 4096-row sample (through ht.spatial.cdist, the same kernels) against fp64:
    the error of the SQUARED distances relative to |x|^2 + |y|^2 (the quadratic expansion's
    cancellation scale; near-zero distances have no relative accuracy in any fp32 expansion)."""
    import heat_amd as ht

    sub = x[:4096]
    d = ht.spatial.cdist(sub, sub, quadratic_expansion=True).larray
    loc = sub.resplit_(None).larray if sub.is_distributed() else sub.larray
    L = loc.double()
    ref = torch.cdist(L, L)
    nrm = (L * L).sum(1)
    rows = d.shape[0]
    off = 0 if not x.is_distributed() else sum(comm.allgather(rows)[: comm.rank])
    err = 0.0
    if rows:
        scale = nrm[off: off + rows].unsqueeze(1) + nrm.unsqueeze(0)
        err = float(((d.double() ** 2 - ref[off: off + rows] ** 2).abs() / scale).max())
    err = comm.allreduce(err, ht.MPI.MAX) if comm.size > 1 else err
    return {"sample_max_sq_err_rel_vs_fp64": err}


def validate_knn(x, d, idx, comm) -> dict:
    """Rank 0's first 64 local queries against an fp64 brute force over the gathered data (the
    self-match must come first at distance 0)."""
    xs = x.larray
    full = comm.allgather_tensor(xs.contiguous(), 0, x.split_counts()) if x.is_distributed() else xs
    q = xs[:64].double()
    ok = {}
    if q.shape[0]:
        ref = torch.cdist(q, full.double())
        rd, ri = torch.topk(ref, idx.gshape[1], dim=1, largest=False)
        r0 = x.counts_displs()[1][comm.rank] if x.is_distributed() else 0
        ok["self_first"] = bool((idx.larray[:64, 0] == torch.arange(q.shape[0], device=q.device) + r0).all())
        ok["index_agreement"] = float((idx.larray[:64] == ri).float().mean())
        ok["max_rel_dist_err"] = float(((d.larray[:64].double() - rd).abs() / rd.clamp(min=1e-6)).max())
    if comm.size > 1:
        ok = comm.bcast(ok, root=0)
    return ok


def rccl_world_size(comm) -> int:
    """Number of ranks a DEVICE all-reduce actually reaches (RCCL on a GPU job, gloo on CPU)."""
    import torch.distributed as dist

    import heat_amd as ht

    if comm.size == 1 or not dist.is_initialized():
        return 1
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    one = torch.ones(1, dtype=torch.int32, device=dev)
    comm.Allreduce(ht.MPI.IN_PLACE, one, ht.MPI.SUM)   # the device-buffer path (host-staged on gloo)
    return int(one.item())


def rank_times(comm, dt: float, steps: int, extra: dict) -> float:
    """ms per step of the SLOWEST rank (the job's step time); per-rank spread into ``extra``."""
    per_rank = comm.allgather(dt) if comm.size > 1 else [dt]
    extra["rank_ms_per_step_min"] = min(per_rank) / steps * 1e3
    extra["rank_ms_per_step_max"] = max(per_rank) / steps * 1e3
    return max(per_rank) / steps * 1e3


def reference_iteration(x, km, k):
    """Time ONE iteration of the reference's algorithm (heat 1.1 kmeans.py:73-100 + _kcluster
    assign) expressed with torch on the same data: cdist by quadratic expansion (n x k matrix),
    argmin, then k masked passes for the update + one all-reduce per cluster."""
    import heat_amd as ht

    X = x.larray
    C = km.cluster_centers_.larray
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d2 = torch.clamp((X * X).sum(1, keepdim=True) + (C * C).sum(1) - 2 * X @ C.T, min=0).sqrt()
    lab = d2.argmin(1, keepdim=True)
    del d2
    newc = torch.empty_like(C)
    for i in range(k):
        sel = (lab == i).to(X.dtype)
        s = (X * sel).sum(0)
        cnt = sel.sum().clamp(min=1)
        if x.comm.size > 1:
            x.comm.Allreduce(ht.MPI.IN_PLACE, s, ht.MPI.SUM)
            x.comm.Allreduce(ht.MPI.IN_PLACE, cnt, ht.MPI.SUM)
        newc[i] = s / cnt
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


if __name__ == "__main__":
    main()
