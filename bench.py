#!/usr/bin/env python
"""
Flagship benchmark: one k-means Lloyd iteration (assign + update + all-reduce) on split=0 float32
data, the BASELINE.json config "k-means k=1024 on 1e8 x 64 float32 split=0, 8 x MI355X".

Weak scaling: every GPU holds ``--n-per-gpu`` points (default 1.25e7, so 8 GPUs = 1e8 points).
Data are synthetic (Threefry normal samples generated on the device, random-init centroids).
``value`` is the whole-job GFLOP/s of the distance computation (2*n*k*f per iteration, the
quantity the reference's benchmark scales with); ``ms_per_step`` the wall time of one iteration.

Run: ``python bench.py`` (1 GPU) or ``torchrun --nproc-per-node N bench.py --gpus N``.
Secondary workloads: ``--workload cdist`` (distance_matrix, streamed), ``--workload knn`` (the
distance_matrix config reduced to each row's ``--topk`` nearest rows by the fused kernel, no
matrix) and ``--workload moments`` (statistical_moments mean/var of 1e9 float32).
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
    p.add_argument("--workload", default="kmeans", choices=["kmeans", "cdist", "knn", "moments"])
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
    return p.parse_args()


def main():
    args = parse()
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
        args.n_per_gpu = args.n_per_gpu or 12_500_000
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
    if comm.rank == 0:
        out = {"metric": metric, "value": value, "unit": unit, "n_gpus": n_gpus, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": scaling,
               "vs_baseline": None, "dtype": "fp32", "data": "synthetic (device Threefry normal samples)",
               "config": cfg, "extra": extra}
        print(json.dumps(out), flush=True)


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
    return {"centroids_agree": hi == lo, "count_sum_ok": int(round(float(counts.sum()))) == x.gshape[0],
            "centroid_max_rel_err_vs_fp64": err, "allreduce_us": us,
            "allreduce_bytes": buf.numel() * buf.element_size()}


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

    if comm.size == 1 or not dist.is_initialized():
        return 1
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    one = torch.ones(1, dtype=torch.int32, device=dev)
    dist.all_reduce(one)
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
