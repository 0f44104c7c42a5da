"""
Python entry points of the native kernels (device tensors) with PyTorch reference paths (host
tensors; also the numerics oracle of the tests).
"""
from __future__ import annotations

import contextlib
import ctypes
import weakref
import os
import threading
from typing import NamedTuple, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import check, lib, stream_ptr, use_native

__all__ = ["kmeans_finalize", "pack_blocks", "unpack_blocks", "pack_supported", "kmeans_assign", "kmeans_pack_points", "PackedPoints", "cdist_pack", "PackedRows", "kmeans_update", "moments", "merge_moments", "num_cus", "cdist", "lasso_epoch", "lasso_prepare", "LassoSweep", "gemm_f16x3",
           "split_planes", "gram_product", "gemm_f32_small", "knn_topk", "kmeans_step_small", "kmeans_lloyd_small", "lasso_gram", "lasso_cd", "argreduce_keys",
           "argreduce_decode", "argreduce_supported", "topk_rows", "gemm_f32", "gemm_h3", "h3_planes", "H3Planes",
           "gemm_h3_planes", "gemm64", "cholesky_upper", "tri_inv_upper", "householder_qr",
           "householder_factor", "householder_apply", "householder_block", "vtc64", "gram64",
           "radix_sort_supported", "sort_rows"]

_NUM_CUS = {}


def num_cus(device) -> int:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _NUM_CUS:
        _NUM_CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _NUM_CUS[idx]


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# --------------------------------------------------------------------------------------------- k-means
def _rows_f32_aligned(X: torch.Tensor) -> torch.Tensor:
    """fp32, row-contiguous, feature count a multiple of 4 (zero padding changes no dot product)."""
    if X.dtype != torch.float32:
        X = X.float()
    if X.stride(-1) != 1 or X.stride(0) % 4 != 0 or X.data_ptr() % 16 != 0:
        X = X.contiguous()
    f = X.shape[1]
    if f % 4 != 0:
        X = F.pad(X, (0, 4 - f % 4))
    if X.stride(0) % 4 != 0 or X.data_ptr() % 16 != 0:
        X = X.contiguous()
    return X


class PackedPoints(NamedTuple):
    """Points split once per fit into fp16 hi/lo planes with a power-of-two row scale (see
    ``csrc/kmeans_f16x3.hip``); reused by every assignment against new centroids."""
    planes: torch.Tensor   # [n, 2 * fpad] float16
    sx: torch.Tensor       # [n] float32
    n: int
    f: int
    key: tuple


def _points_key(X: torch.Tensor) -> tuple:
    return (X.data_ptr(), tuple(X.shape), tuple(X.stride()), X._version, X.device)


def kmeans_pack_points(X: torch.Tensor) -> Optional[PackedPoints]:
    """fp16x3 planes of X for :func:`kmeans_assign` (None where the fast path does not apply)."""
    if not (use_native(X) and X.dtype == torch.float32 and X.dim() == 2):
        return None
    L = lib()
    n, f = X.shape
    fpad = L.ha_h3_fpad(f)
    if fpad < 0:
        return None
    Xc = X if X.stride(-1) == 1 else X.contiguous()
    planes = torch.empty((n, 2 * fpad), dtype=torch.float16, device=X.device)
    sx = torch.empty(n, dtype=torch.float32, device=X.device)
    check(L.ha_h3_pack_points(_ptr(Xc), n, f, Xc.stride(0), _ptr(planes), _ptr(sx),
                              ctypes.c_void_p(stream_ptr(X.device))), "ha_h3_pack_points")
    return PackedPoints(planes, sx, n, f, _points_key(X))


_H3_RESIDENT = os.environ.get("HEAT_H3_RESIDENT", "1") != "0"  # 0: chunk-staged h3_assign_p
_H3_RESIDENT_ALL = os.environ.get("HEAT_H3_RESIDENT") == "all"  # also k beyond LDS (phases)


def _small_k_ok(X: torch.Tensor, k: int) -> bool:
    return (use_native(X) and X.dtype == torch.float32 and X.dim() == 2 and 0 < k <= 16
            and 0 < X.shape[1] <= 64 and X.stride(-1) == 1)


def _ks_step(X: torch.Tensor, C: torch.Tensor, want_mind: bool, update: bool):
    L = lib()
    n, f = X.shape
    k = C.shape[0]
    dev = X.device
    Cc = C.to(device=dev, dtype=torch.float32)
    Cc = Cc if Cc.stride(-1) == 1 else Cc.contiguous()
    labels = torch.empty(n, dtype=torch.int32, device=dev)
    mind = torch.empty(n, dtype=torch.float32, device=dev) if want_mind else None
    ncu = num_cus(dev)
    ws = torch.empty(max(1, L.ha_ks_workspace_floats(k, ncu)), dtype=torch.float32, device=dev)
    sums = torch.empty((k, f), dtype=torch.float32, device=dev) if update else None
    counts = torch.empty(k, dtype=torch.float32, device=dev) if update else None
    check(L.ha_ks_step(_ptr(X), n, f, X.stride(0), _ptr(Cc), k, Cc.stride(0), _ptr(labels), _ptr(mind), _ptr(sums),
                       _ptr(counts), _ptr(ws), ncu, ctypes.c_void_p(stream_ptr(dev))), "ha_ks_step")
    return labels, mind, sums, counts


_KS_LLOYD = {}   # (device, stream, k) -> [workspace, (weakref, version) of the centroids padded in it]


def kmeans_lloyd_small(X: torch.Tensor, C: torch.Tensor,
                       reuse_pad: bool = False) -> Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
    """One whole Lloyd step for few clusters on ONE process (k <= 16, f <= 64, device fp32): (int32
    labels, new centroids [k, f] fp32, squared shift 0-d fp64) from one pass over the points plus ONE
    epilogue launch (``csrc/kmeans_smallk.hip: ha_ks_lloyd`` - reduction, new centroids, shift and
    the next pass's padded centroids), instead of the pass's reduction + ``kmeans_finalize`` + the
    next pass's padding. None where it does not apply."""
    if not _small_k_ok(X, C.shape[0]) or X.shape[0] == 0 or not hasattr(lib(), "ha_ks_lloyd"):
        return None
    if torch.cuda.is_current_stream_capturing():
        return None   # the pad reuse below is host state: not for graph capture
    L = lib()
    n, f = X.shape
    k = C.shape[0]
    dev = X.device
    Cc = C.to(device=dev, dtype=torch.float32)
    Cc = Cc if Cc.stride(-1) == 1 else Cc.contiguous()
    ncu = num_cus(dev)
    sp = stream_ptr(dev)
    # one workspace per stream: launches on one stream are ordered, so its partial slots, arrival
    # counter and padded centroids are never used by two passes at once
    state = _KS_LLOYD.get((dev, sp, k))
    if state is None:
        ws = torch.zeros(max(1, L.ha_ks_lloyd_workspace_floats(k, ncu)), dtype=torch.float32, device=dev)
        state = _KS_LLOYD[(dev, sp, k)] = [ws, None]
    # the padded chunks in the workspace belong to the previous call's newC: valid for this call
    # only if the caller owns C as that output (``reuse_pad``: the KMeans loop, which never writes
    # its centroids by a path that skips ``_version`` - .data, DLPack, raw-pointer kernels) and C
    # IS that tensor object, alive and unmodified; an address match alone could be a new tensor in
    # the freed block
    prev = state[1]
    pad_ready = bool(reuse_pad) and prev is not None and prev[0]() is Cc and prev[1] == Cc._version
    labels = torch.empty(n, dtype=torch.int32, device=dev)
    newC = torch.empty((k, f), dtype=torch.float32, device=dev)
    shift = torch.empty((), dtype=torch.float64, device=dev)
    check(L.ha_ks_lloyd(_ptr(X), n, f, X.stride(0), _ptr(Cc), k, Cc.stride(0), _ptr(labels), _ptr(newC), _ptr(shift),
                        _ptr(state[0]), ncu, int(pad_ready), ctypes.c_void_p(sp)), "ha_ks_lloyd")
    state[1] = (weakref.ref(newC), newC._version)
    return labels, newC, shift


def kmeans_step_small(X: torch.Tensor, C: torch.Tensor) -> Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
    """One fused Lloyd pass for few clusters (k <= 16, f <= 64, device fp32): (int32 labels,
    per-cluster sums [k, f], counts [k]) reading the points once; None where it does not apply."""
    if not _small_k_ok(X, C.shape[0]):
        return None
    labels, _, sums, counts = _ks_step(X, C, want_mind=False, update=True)
    return labels, sums, counts


def kmeans_assign(X: torch.Tensor, C: torch.Tensor, want_mind: bool = True,
                  packed: Optional[PackedPoints] = None,
                  certified: bool = False) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Nearest centroid (squared L2) of every row of X. Returns (int32 labels, min squared distance).

    k <= 16 and f <= 64: exact fp32 VALU kernel (difference form, HBM-bound) whatever ``packed``
    says.

    Device tensors, fused kernels with a running argmin (no n x k intermediate):
    ``packed`` given (from :func:`kmeans_pack_points`) -> fp16x3 split on the FP16 matrix cores
    (accuracy of an fp32 GEMM, ~5x faster); otherwise the exact f32-input MFMA kernel.
    ``certified`` (fp16x3 path, labels only): a one-term fp16 pass assigns every point whose best
    centroid wins by more than a rigorous error bound, and only the others are re-run with three
    terms. Same labels; ~2x faster on well-separated clusters, ~2x slower where nearly every point
    is a near-tie (diffuse data) - callers decide adaptively from ``kmeans_assign.last_rechecked``
    (device int32: number of re-checked points of the last certified call)."""
    n, f = X.shape
    k = C.shape[0]
    if n == 0:
        return (torch.empty(0, dtype=torch.int32, device=X.device),
                torch.empty(0, dtype=torch.float32, device=X.device) if want_mind else None)
    if _small_k_ok(X, k):
        # few clusters: exact VALU kernel over LDS-staged tiles, HBM-bound (csrc/kmeans_smallk.hip)
        labels, mind, _, _ = _ks_step(X, C, want_mind=want_mind, update=False)
        if certified:
            kmeans_assign.last_rechecked = torch.zeros((), dtype=torch.int32, device=X.device)
        return labels, mind
    if packed is not None and use_native(X):
        if packed.n != n or packed.f != f:
            raise ValueError("packed points do not match X")
        L = lib()
        Cc = C.to(device=X.device, dtype=torch.float32)
        Cc = Cc if Cc.stride(-1) == 1 else Cc.contiguous()
        ws = torch.empty(L.ha_h3_workspace_bytes(k, f), dtype=torch.uint8, device=X.device)
        labels = torch.empty(n, dtype=torch.int32, device=X.device)
        if certified and not want_mind:
            # uncertain-point lists (one per shard of the filter's workgroups) + their counts
            cap = L.ha_h3_amb_rows(n)
            amb = torch.empty(cap + L.ha_h3_amb_shards(), dtype=torch.int32, device=X.device)
            rc = L.ha_h3_assign_certified(_ptr(packed.planes), _ptr(packed.sx), n, f, _ptr(Cc), k, Cc.stride(0),
                                          _ptr(ws), _ptr(labels), _ptr(amb), _ptr(amb[cap:]),
                                          ctypes.c_void_p(stream_ptr(X.device)))
            check(rc, "ha_h3_assign_certified")
            kmeans_assign.last_rechecked = amb[cap:].sum(dtype=torch.int32)
            return labels, None
        mind = torch.empty(n, dtype=torch.float32, device=X.device) if want_mind else None
        phases = L.ha_h3r_phases(k, f)
        if _H3_RESIDENT and (phases == 1 or _H3_RESIDENT_ALL):
            # centroids resident in LDS, one workgroup per CU streaming the points. Only where they
            # all fit: in phases (k = 1024 at f = 64) the full Lloyd step measured 5.28 vs 5.07 ms
            scratch = torch.empty(2 * n if phases > 1 else 1, dtype=torch.float32, device=X.device)
            rc = L.ha_h3_assign_r(_ptr(packed.planes), _ptr(packed.sx), n, f, _ptr(Cc), k, Cc.stride(0), _ptr(ws),
                                  _ptr(scratch), num_cus(X.device), _ptr(labels), _ptr(mind),
                                  ctypes.c_void_p(stream_ptr(X.device)))
            check(rc, "ha_h3_assign_r")
            return labels, mind
        rc = L.ha_h3_assign(_ptr(packed.planes), _ptr(packed.sx), n, f, _ptr(Cc), k, Cc.stride(0), _ptr(ws),
                            _ptr(labels), _ptr(mind), ctypes.c_void_p(stream_ptr(X.device)))
        check(rc, "ha_h3_assign")
        return labels, mind
    if use_native(X) and f <= 128:
        Xa = _rows_f32_aligned(X)
        Ca = _rows_f32_aligned(C.to(X.device))
        fa = Xa.shape[1]
        L = lib()
        fpad, kpad = ctypes.c_int(), ctypes.c_int()
        wsz = L.ha_km_workspace_floats(k, fa, ctypes.byref(fpad), ctypes.byref(kpad))
        ws = torch.empty(wsz, dtype=torch.float32, device=X.device)
        labels = torch.empty(n, dtype=torch.int32, device=X.device)
        mind = torch.empty(n, dtype=torch.float32, device=X.device) if want_mind else None
        rc = L.ha_km_assign(_ptr(Xa), n, fa, Xa.stride(0), _ptr(Ca), k, Ca.stride(0), _ptr(ws), _ptr(labels),
                            _ptr(mind), ctypes.c_void_p(stream_ptr(X.device)))
        check(rc, "ha_km_assign")
        return labels, mind
    Xf = X.float() if X.dtype not in (torch.float32, torch.float64) else X
    Cf = C.to(Xf.dtype)
    cn = (Cf * Cf).sum(1)
    d = torch.addmm(cn.unsqueeze(0), Xf, Cf.t(), beta=1.0, alpha=-2.0)
    best, labels = torch.min(d, dim=1)
    mind = None
    if want_mind:
        mind = torch.clamp(best + (Xf * Xf).sum(1), min=0).float()
    return labels.to(torch.int32), mind


kmeans_assign.last_rechecked = None


def _lex_key(d: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """int64 keys ordering non-negative float32 distances, equal distances by index: the float
    bits of d >= 0 are monotone as integers, so (bits << 32) | idx sorts lexicographically."""
    bits = (d.float() + 0.0).contiguous().view(torch.int32).to(torch.int64)   # + 0.0: -0.0 -> +0.0
    return (bits << 32) | (idx.to(torch.int64) & 0xFFFFFFFF)


def _lex_split(key: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    d = (key >> 32).to(torch.int32).view(torch.float32)
    i = (key & 0xFFFFFFFF)
    return d, torch.where(i == 0xFFFFFFFF, torch.full_like(i, -1), i)


def _topk_lex(d: torch.Tensor, idx: Optional[torch.Tensor], k: int,
              max_index: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """k smallest distances per row with ties ordered by (global) index - the same answer for any
    blocking of the candidates, hence for any number of ranks. ``max_index`` bounds the indices
    (the caller's row count): the packed keys hold 32-bit indices, so from 2^32 - 1 rows on the
    selection runs as two stable sorts instead (index, then distance)."""
    if idx is None:
        max_index = d.shape[1] - 1
        idx = torch.arange(d.shape[1], device=d.device).expand(d.shape[0], -1)
    if max_index is None or max_index >= 0xFFFFFFFF:
        o = torch.sort(idx, dim=1, stable=True).indices
        dd, ii = torch.gather(d, 1, o), torch.gather(idx.to(torch.int64), 1, o)
        o = torch.sort(dd.float() + 0.0, dim=1, stable=True).indices[:, :k]
        return torch.gather(dd, 1, o).float(), torch.gather(ii, 1, o)
    key = _lex_key(d, idx)
    key = torch.topk(key, k, dim=1, largest=False).values if k < key.shape[1] else torch.sort(key, dim=1).values
    return _lex_split(key)


_KNN_CERTIFIED = os.environ.get("HEAT_KNN_CERTIFIED", "1") != "0"
# candidates per query of the certified one-term pass: 32 keeps both lane halves' lists whole (a
# wider certification margin: fewer queries re-run through the 3-term kernel) at the price of
# rescoring twice the rows, which the fused rescoring kernel makes cheap; 16 merges them
_KNN_KP = 32 if os.environ.get("HEAT_KNN_KP", "32") == "32" else 16


def _knn_exact_select(Q: torch.Tensor, T: torch.Tensor, idx: torch.Tensor, k: int):
    """Exact (difference-form) squared distances of the candidate rows ``idx`` [nq, c] (-1 =
    none), the k smallest per query, equal distances ordered by index. Device fp32 with c <= 32:
    one fused kernel (``csrc/knn_rescore.hip``: a 32-lane group per query, a bitonic sort of the
    (distance, index) keys); otherwise torch over [rows, c, f] blocks."""
    nq, c = idx.shape
    f = Q.shape[1]
    if (Q.is_cuda and use_native(Q) and Q.dtype == torch.float32 and T.dtype == torch.float32 and 0 < k <= c <= 32
            and nq > 0 and T.shape[0] < 2 ** 32 - 1):
        Qc = Q if Q.stride(-1) == 1 else Q.contiguous()
        Tc = T if T.stride(-1) == 1 else T.contiguous()
        ic = idx.contiguous()
        dist = torch.empty((nq, k), dtype=torch.float32, device=Q.device)
        out_i = torch.empty((nq, k), dtype=torch.int64, device=Q.device)
        check(lib().ha_knn_rescore(_ptr(Qc), Qc.stride(0) if nq > 1 else f, _ptr(Tc),
                                   Tc.stride(0) if T.shape[0] > 1 else f, T.shape[0], nq, f, _ptr(ic),
                                   int(ic.dtype == torch.int64), c, k, _ptr(dist), _ptr(out_i),
                                   ctypes.c_void_p(stream_ptr(Q.device))), "ha_knn_rescore")
        return dist, out_i
    dist = torch.empty((nq, k), dtype=torch.float32, device=Q.device)
    out_i = torch.empty((nq, k), dtype=torch.int64, device=Q.device)
    step = max(1, (1 << 26) // (c * f))
    for q0 in range(0, nq, step):
        ib = idx[q0: q0 + step]
        nb = T[ib.clamp(min=0)].float()
        d = ((Q[q0: q0 + step].float().unsqueeze(1) - nb) ** 2).sum(-1)
        d = torch.where(ib >= 0, d, torch.full_like(d, float("inf")))
        dv, di = _topk_lex(d, ib, k, max_index=T.shape[0] - 1)
        dist[q0: q0 + step] = dv
        out_i[q0: q0 + step] = di
    return dist, out_i


def _knn_certified(Q, T, Tc, k, packed, ws, exact_distances: bool = True):
    """k <= 8 nearest rows of T through the certified one-term kernel (``h1_topk``: 1 fp16 MFMA
    per k-step instead of 3, a rigorous error bound per query): ``_KNN_KP`` candidates per query,
    the queries whose candidates are not certified to contain the true k nearest re-run through
    the 3-term kernel (16 candidates), then every candidate list is rescored exactly."""
    L = lib()
    nq, f = Q.shape
    nt = T.shape[0]
    dev = Q.device
    kp = _KNN_KP
    st = ctypes.c_void_p(stream_ptr(dev))
    dist = torch.empty((nq, kp), dtype=torch.float32, device=dev)
    idx = torch.empty((nq, kp), dtype=torch.int32, device=dev)
    cert = torch.empty(nq, dtype=torch.uint8, device=dev)
    check(L.ha_h1_topk(_ptr(packed.planes), _ptr(packed.sx), nq, f, _ptr(Tc), nt, Tc.stride(0), _ptr(ws), k, kp,
                       _ptr(dist), _ptr(idx), _ptr(cert), st), "ha_h1_topk")
    unc = torch.nonzero(cert == 0).flatten()
    _KNN_STATS["queries"] += nq
    _KNN_STATS["rechecked"] += int(unc.numel())
    if unc.numel():
        pl = packed.planes.index_select(0, unc).contiguous()
        sxu = packed.sx.index_select(0, unc).contiguous()
        nu = int(unc.numel())
        qblocks = (nu + 127) // 128
        splits = max(1, min(L.ha_h3_topk_chunks(nt, f) // 4, (4 * num_cus(dev) + qblocks - 1) // qblocks))
        k3 = min(kp, 16)   # the 3-term kernel's list length
        d3 = torch.empty((splits, nu, k3), dtype=torch.float32, device=dev)
        i3 = torch.empty((splits, nu, k3), dtype=torch.int32, device=dev)
        check(L.ha_h3_topk(_ptr(pl), _ptr(sxu), nu, f, _ptr(Tc), nt, Tc.stride(0), _ptr(ws), k3, splits, _ptr(d3),
                           _ptr(i3), st), "ha_h3_topk")
        if splits == 1:
            i3 = i3[0].long()
        else:
            _, i3 = _topk_lex(d3.permute(1, 0, 2).reshape(nu, splits * k3), i3.permute(1, 0, 2).reshape(nu, splits * k3),
                              k3, max_index=nt - 1)
        idx = idx.long()
        idx[unc] = -1
        idx[unc, :k3] = i3
    else:
        idx = idx.long()
    # the k nearest are certified to be AMONG the candidates, not ranked: always rescore exactly
    return _knn_exact_select(Q, T, idx, k)


_KNN_STATS = {"queries": 0, "rechecked": 0}


def knn_topk(Q: torch.Tensor, T: torch.Tensor, k: int, packed: Optional[PackedPoints] = None,
             exact_distances: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """The ``k`` nearest rows of ``T`` for every row of ``Q``: (squared distances [nq, k] ascending,
    int64 row indices [nq, k]; +inf / -1 where T has fewer than k rows).

    Device fp32 with k <= 16 and f <= 128: ONE fused kernel (fp16x3 MFMA scores + a running top-k
    per point in registers, ``csrc/kmeans_f16x3.hip: h3_topk_p``), no nq x nt distance matrix;
    for k <= 8 (and enough queries to fill the GPU) the certified one-term pass first
    (``h1_topk``, :func:`_knn_certified`). The selected neighbours' distances are then recomputed
    exactly (difference form) and re-sorted (``exact_distances``). Otherwise: distance tiles +
    torch.topk, in query blocks."""
    nq, f = Q.shape
    nt = T.shape[0]
    dev = Q.device
    if nq == 0 or nt == 0 or k <= 0:
        return (torch.full((nq, max(k, 0)), float("inf"), device=dev),
                torch.full((nq, max(k, 0)), -1, dtype=torch.int64, device=dev))
    if use_native(Q) and Q.dtype == torch.float32 and T.dtype == torch.float32 and k <= 16 \
            and lib().ha_h3_fpad(f) > 0 and nt < 2 ** 31 - 256:
        L = lib()
        if packed is None or packed.key != _points_key(Q):
            packed = kmeans_pack_points(Q)
        Tc = T if T.stride(-1) == 1 else T.contiguous()
        # the certified pass pads the training rows to whole 128-row chunks: size for both kernels
        ws = torch.empty(max(L.ha_h3_workspace_bytes(nt, f), L.ha_h1_workspace_bytes(nt, f)), dtype=torch.uint8,
                         device=dev)
        # fill the GPU: with few query blocks, divide the training chunks over workgroup columns
        # (>= 4 waves of 128 queries per CU overall) and merge the partial lists
        qblocks = (nq + 127) // 128
        splits = max(1, min(L.ha_h3_topk_chunks(nt, f) // 4, (4 * num_cus(dev) + qblocks - 1) // qblocks))
        if splits == 1 and k <= 8 and _KNN_CERTIFIED and hasattr(L, "ha_h1_topk"):
            return _knn_certified(Q, T, Tc, k, packed, ws, exact_distances)
        dist = torch.empty((splits, nq, k), dtype=torch.float32, device=dev)
        idx = torch.empty((splits, nq, k), dtype=torch.int32, device=dev)
        check(L.ha_h3_topk(_ptr(packed.planes), _ptr(packed.sx), nq, f, _ptr(Tc), nt, Tc.stride(0), _ptr(ws), k,
                           splits, _ptr(dist), _ptr(idx), ctypes.c_void_p(stream_ptr(dev))), "ha_h3_topk")
        if splits == 1:
            dist, idx = dist[0], idx[0].long()
        else:
            dist = dist.permute(1, 0, 2).reshape(nq, splits * k)
            idx = idx.permute(1, 0, 2).reshape(nq, splits * k)
            dist, idx = _topk_lex(dist, idx, k, max_index=nt - 1)
    else:
        kk = min(k, nt)
        step = max(1, (1 << 28) // max(nt, 1))
        ds, ids = [], []
        for q0 in range(0, nq, step):
            d = cdist(Q[q0: q0 + step].float(), T.float(), "sqeuclidean", exact=True)
            dv, di = _topk_lex(d, None, kk)   # equal distances ordered by index
            ds.append(dv)
            ids.append(di)
        dist, idx = torch.cat(ds), torch.cat(ids)
        if kk < k:
            dist = torch.cat([dist, torch.full((nq, k - kk), float("inf"), device=dev)], 1)
            idx = torch.cat([idx, torch.full((nq, k - kk), -1, dtype=torch.int64, device=dev)], 1)
        return dist, idx
    if exact_distances:
        return _knn_exact_select(Q, T, idx, k)
    return dist, idx


def kmeans_update(X: torch.Tensor, labels: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-cluster feature sums [k, f] and counts [k] (float32) of the rows of X."""
    n, f = X.shape
    if use_native(X) and X.dtype == torch.float32:
        L = lib()
        ncu = num_cus(X.device)
        wsize = L.ha_km_update_workspace(n, k, f, ncu)
        if wsize >= 0:
            Xc = X if X.stride(-1) == 1 else X.contiguous()
            lab = labels.to(torch.int32).contiguous()
            sums = torch.empty((k, f), dtype=torch.float32, device=X.device)
            counts = torch.empty(k, dtype=torch.float32, device=X.device)
            ws = torch.empty(max(1, wsize), dtype=torch.int32, device=X.device)
            rc = L.ha_km_update(_ptr(Xc), n, f, Xc.stride(0), _ptr(lab), k, _ptr(sums), _ptr(counts), _ptr(ws),
                                ncu, ctypes.c_void_p(stream_ptr(X.device)))
            check(rc, "ha_km_update")
            return sums, counts
    lab = labels.to(torch.int64)
    sums = torch.zeros((k, f), dtype=X.dtype if X.is_floating_point() else torch.float32, device=X.device)
    sums.index_add_(0, lab, X.to(sums.dtype))
    counts = torch.bincount(lab, minlength=k).to(sums.dtype)
    return sums, counts


# --------------------------------------------------------------------------------------------- moments
def merge_moments(n: torch.Tensor, mean: torch.Tensor, m2: torch.Tensor, dim: int):
    """Chan/Golub/LeVeque merge of (count, mean, M2) partials along ``dim`` (fp64)."""
    N = n.sum(dim)
    safe = torch.where(N > 0, N, torch.ones_like(N))
    mu = (n * mean).sum(dim) / safe
    M2 = (m2 + n * (mean - mu.unsqueeze(dim)) ** 2).sum(dim)
    return N, mu, M2


_MOM_KINDS = {None: 0, "mean": 1, "var": 2, "std": 3}
_MOM_COUNTERS = {}


def _mom_counters(device, n: int) -> torch.Tensor:
    """Zeroed arrival counters of the fused moments epilogue (the kernels reset what they use).
    One set per (device, stream): launches on one stream run in order, so a set is never shared by
    two kernels in flight."""
    dev = device.index if device.index is not None else torch.cuda.current_device()
    key = (dev, stream_ptr(device))
    c = _MOM_COUNTERS.get(key)
    if c is None or c.numel() < n:
        c = torch.zeros(max(n, 4096), dtype=torch.int32, device=device)
        _MOM_COUNTERS[key] = c
    return c


def _mom_rows_workspace(device, nrows: int, nchunks: int):
    """Partials + arrival counters of ha_moments_rows' fused epilogue (counters None if unused)."""
    pd, nc = ctypes.c_int64(), ctypes.c_int64()
    lib().ha_moments_rows_workspace(nrows, nchunks, ctypes.byref(pd), ctypes.byref(nc))
    part = torch.empty(max(pd.value, 1), dtype=torch.float64, device=device)
    return part, (_mom_counters(device, nc.value) if nc.value > 0 else None)


def _moments_native(x: torch.Tensor, axis, final=None, ddof: int = 0):
    """One launch (``csrc/moments.hip``): per-chunk partials merged by each output's last block.
    final None: (N, mean, M2) fp64 triples; 'mean' / 'var' / 'std': the fp32 result itself."""
    L = lib()
    s = ctypes.c_void_p(stream_ptr(x.device))
    ncu = num_cus(x.device)
    kind = _MOM_KINDS[final]

    def out_for(shape):
        if kind == 0:
            return torch.empty(tuple(shape) + (3,), dtype=torch.float64, device=x.device)
        return torch.empty(tuple(shape), dtype=torch.float32, device=x.device)

    def finish(out, shape):
        if kind:
            return out
        return out[..., 0], out[..., 1], out[..., 2]

    if axis is None:
        flat = x.reshape(-1)
        if not flat.is_contiguous():
            flat = flat.contiguous()
        numel = flat.numel()
        cpc = int(os.environ.get("HEAT_MOM_ROW_CHUNKS_PER_CU", "4"))
        nchunks = max(1, min(cpc * ncu, (numel + 16383) // 16384))
        part, cnt = _mom_rows_workspace(x.device, 1, nchunks)
        out = out_for(())
        check(L.ha_moments_rows(_ptr(flat), 1, numel, numel, nchunks, _ptr(part), _ptr(out), kind, float(ddof),
                                _ptr(cnt), s), "ha_moments_rows")
        return finish(out, ())
    if not x.is_contiguous():
        x = x.contiguous()
    shape = list(x.shape)
    red = shape[axis]
    outer = 1
    for d in shape[:axis]:
        outer *= d
    inner = 1
    for d in shape[axis + 1:]:
        inner *= d
    out_shape = shape[:axis] + shape[axis + 1:]
    if inner == 1:
        nrows = outer
        nchunks = max(1, min((2 * 8 * ncu + nrows - 1) // max(nrows, 1), (red + 4095) // 4096))
        part, cnt = _mom_rows_workspace(x.device, nrows, nchunks)
        out = out_for(out_shape)
        check(L.ha_moments_rows(_ptr(x), nrows, red, red, nchunks, _ptr(part), _ptr(out), kind, float(ddof),
                                _ptr(cnt), s), "ha_moments_rows")
        return finish(out, out_shape)
    if outer == 1:
        ncols = inner
        col_blocks = max(1, (ncols + 1023) // 1024)
        # row chunks per CU (8 rows in flight per thread); the chunk partials are merged by a
        # two-level tree inside the kernel (moments.hip), so many chunks cost no serial merge
        cpc = int(os.environ.get("HEAT_MOM_COL_CHUNKS_PER_CU", "1"))
        nchunks = max(1, min(65535, (cpc * ncu + col_blocks - 1) // col_blocks, (red + 63) // 64))
        pd, nc = ctypes.c_int64(), ctypes.c_int64()
        L.ha_moments_cols_workspace(ncols, nchunks, ctypes.byref(pd), ctypes.byref(nc))
        part = torch.empty(pd.value, dtype=torch.float64, device=x.device)
        out = out_for(out_shape)
        check(L.ha_moments_cols(_ptr(x), red, ncols, ncols, nchunks, _ptr(part), _ptr(out), kind, float(ddof),
                                _ptr(_mom_counters(x.device, nc.value)), s), "ha_moments_cols")
        return finish(out, out_shape)
    y = x.movedim(axis, -1).contiguous()
    return _moments_native(y, y.dim() - 1, final, ddof)


def moments(x: torch.Tensor, axis: Optional[int] = None, final: Optional[str] = None, ddof: int = 0):
    """(count, mean, M2) over ``axis`` (None = all) as float64 tensors; with ``final`` in
    ('mean', 'var', 'std') the float32 result itself (variance with ``ddof``).

    Device fp32 tensors: ONE kernel launch - one HBM pass with 16-byte loads and the chunk merge
    fused into each output's last block (``moments.hip``)."""
    if use_native(x) and x.dtype == torch.float32 and x.numel() > 0:
        return _moments_native(x, axis, final, ddof)
    xd = x.double() if not x.is_complex() else x
    if axis is None:
        n = torch.tensor(float(x.numel()), dtype=torch.float64, device=x.device)
        if x.numel() == 0:
            z = torch.tensor(0.0, dtype=torch.float64, device=x.device)
            n, mean, m2 = n, z, z.clone()
        else:
            var, mean = torch.var_mean(xd, correction=0)
            m2 = var * n
    else:
        n = torch.full([s for i, s in enumerate(x.shape) if i != axis], float(x.shape[axis]), dtype=torch.float64,
                       device=x.device)
        if x.shape[axis] == 0:
            z = torch.zeros_like(n)
            mean, m2 = z, z.clone()
        else:
            var, mean = torch.var_mean(xd, dim=axis, correction=0)
            m2 = var * n
    if final is None:
        return n, mean, m2
    if final == "mean":
        return mean
    v = m2 / (n - ddof)
    return v.sqrt() if final == "std" else v


# --------------------------------------------------------------------------------------------- cdist
_CDIST_MODES = {"euclidean": 0, "sqeuclidean": 1, "gaussian": 2, "manhattan": 3}
_CDIST_EXACT = {"euclidean": 4, "sqeuclidean": 5, "gaussian": 6, "manhattan": 3}


class PackedRows(NamedTuple):
    """Rows split into fp16 hi/lo planes (power-of-two row scale) + {|x|^2, 1/scale} for the
    fp16x3 cdist kernels (``csrc/cdist_f16x3.hip``), in the fragment-blocked layout: rows padded
    to a multiple of 128, each 32-row block stored as the 1 KB MFMA operand fragments of its
    16-feature k-steps. ``rows(lo, hi)`` views a row range starting at a multiple of 128."""
    planes: torch.Tensor  # [padded_rows, 2 * fpad] float16 (blocked, not row-major)
    aux: torch.Tensor     # [padded_rows, 2] float32
    f: int
    n: int                # live rows

    def rows(self, lo: int, hi: int) -> "PackedRows":
        hi = min(hi, self.n)
        if lo % 128:
            raise ValueError("packed row slices must start at a multiple of 128")
        return PackedRows(self.planes[lo:], self.aux[lo:], self.f, max(0, hi - lo))


def cdist_pack(X: torch.Tensor) -> PackedRows:
    """Pack the rows of a float32 device matrix for :func:`cdist` (quadratic-expansion path)."""
    L = lib()
    n, f = X.shape
    fpad = L.ha_cdist_h3_fpad(f)
    rows = L.ha_cdist_h3_rows(n)
    Xc = X if X.stride(-1) == 1 else X.contiguous()
    planes = torch.empty((rows, 2 * fpad), dtype=torch.float16, device=X.device)
    aux = torch.empty((rows, 2), dtype=torch.float32, device=X.device)
    check(L.ha_cdist_h3_pack(_ptr(Xc), n, f, Xc.stride(0), _ptr(planes), _ptr(aux),
                             ctypes.c_void_p(stream_ptr(X.device))), "ha_cdist_h3_pack")
    return PackedRows(planes, aux, f, n)


def _cdist_h3(px: PackedRows, py: PackedRows, mode: int, scale: float, C: torch.Tensor) -> None:
    m, n = px.n, py.n
    if px.f != py.f:
        raise ValueError("packed operands have different feature counts")
    if m and n:
        if C.stride(1) != 1 or C.shape[0] < m or C.shape[1] < n:
            raise ValueError("cdist output must be row-contiguous and at least {} x {}".format(m, n))
        check(lib().ha_cdist_h3(_ptr(px.planes), _ptr(px.aux), m, _ptr(py.planes), _ptr(py.aux), n, px.f, _ptr(C),
                                C.stride(0), mode, ctypes.c_float(scale), ctypes.c_void_p(stream_ptr(C.device))),
              "ha_cdist_h3")


def cdist(X: torch.Tensor, Y: torch.Tensor, metric: str = "euclidean", sigma: float = 1.0,
          out: Optional[torch.Tensor] = None, exact: bool = False, precision: str = "f16x3",
          packed_x: Optional[PackedRows] = None, packed_y: Optional[PackedRows] = None,
          symmetric: bool = False) -> torch.Tensor:
    """Pairwise distances between the rows of X [m, f] and Y [n, f] as an [m, n] float32 matrix.

    Device tensors, L2 family with ``exact=False`` (quadratic expansion, fused norm/clamp/
    sqrt|exp epilogue): ``precision="f16x3"`` -> 3-term fp16 split on the FP16 matrix cores
    (fp32-GEMM accuracy; ``packed_x/packed_y`` from :func:`cdist_pack` skip the packing),
    ``"fp32"`` -> f32-input MFMA kernel. ``exact=True`` (and manhattan) -> VALU tile kernel on the
    differences (no cancellation for near-identical points). No m x n x f intermediate.
    ``symmetric`` (Y is X, difference kernels): only the tiles on or above the diagonal are
    computed, each off-diagonal tile stored twice (the result is exactly symmetric)."""
    m, f = X.shape
    n = Y.shape[0]
    if metric not in _CDIST_MODES:
        raise ValueError("unknown metric {}".format(metric))
    if use_native(X) and X.dtype == torch.float32 and Y.dtype == torch.float32:
        L = lib()
        if not exact and metric != "manhattan" and precision == "f16x3":
            C = out if out is not None else torch.empty((m, n), dtype=torch.float32, device=X.device)
            px = packed_x if packed_x is not None else cdist_pack(X)
            py = packed_y if packed_y is not None else (px if Y is X else cdist_pack(Y.to(X.device)))
            _cdist_h3(px, py, _CDIST_MODES[metric], 1.0 / (2.0 * sigma * sigma), C)
            return C
        mode = (_CDIST_EXACT if exact else _CDIST_MODES)[metric]
        if mode < 3:
            Xa = _rows_f32_aligned(X)
            Ya = _rows_f32_aligned(Y.to(X.device))
        else:
            Xa = X if X.stride(-1) == 1 else X.contiguous()
            if Y is X:
                Ya = Xa
            else:
                Ya = Y.to(X.device)
                Ya = Ya if Ya.stride(-1) == 1 else Ya.contiguous()
        C = out if out is not None else torch.empty((m, n), dtype=torch.float32, device=X.device)
        sym = symmetric and mode >= 3 and Y is X and Xa is Ya and m == n
        if m and n:
            rc = L.ha_cdist(_ptr(Xa), m, _ptr(Ya), n, Xa.shape[1], Xa.stride(0), Ya.stride(0), _ptr(C), C.stride(0),
                            mode | (256 if sym else 0), ctypes.c_float(1.0 / (2.0 * sigma * sigma)),
                            ctypes.c_void_p(stream_ptr(X.device)))
            if sym and rc == _HA_UNSUPPORTED:
                rc = L.ha_cdist(_ptr(Xa), m, _ptr(Ya), n, Xa.shape[1], Xa.stride(0), Ya.stride(0), _ptr(C),
                                C.stride(0), mode, ctypes.c_float(1.0 / (2.0 * sigma * sigma)),
                                ctypes.c_void_p(stream_ptr(X.device)))
            check(rc, "ha_cdist")
        return C
    Xf = X if X.is_floating_point() else X.float()
    Yf = Y.to(Xf.dtype)
    if metric == "manhattan":
        res = torch.cdist(Xf, Yf, p=1)
    elif exact:
        d2 = torch.cdist(Xf, Yf, p=2, compute_mode="donot_use_mm_for_euclid_dist") ** 2
        res = {"euclidean": lambda: d2.sqrt(), "sqeuclidean": lambda: d2,
               "gaussian": lambda: torch.exp(-d2 / (2.0 * sigma * sigma))}[metric]()
    else:
        xn = (Xf * Xf).sum(1, keepdim=True)
        yn = (Yf * Yf).sum(1).unsqueeze(0)
        d2 = torch.clamp(torch.addmm(xn + yn, Xf, Yf.t(), beta=1.0, alpha=-2.0), min=0)
        if metric == "euclidean":
            res = torch.sqrt(d2)
        elif metric == "sqeuclidean":
            res = d2
        else:
            res = torch.exp(-d2 / (2.0 * sigma * sigma))
    if out is not None:
        out.copy_(res)
        return out
    return res


# --------------------------------------------------------------------------------------------- lasso
_GRAM_UNROLL = int(os.environ.get("HEAT_GRAM_UNROLL", "0"))   # rows in flight per thread (0: kernel default)
_GRAM_BLOCKS_PER_CU = int(os.environ.get("HEAT_GRAM_BLOCKS_PER_CU", "0"))  # 0: kernel default (2 per CU)


def _gram_blocked(X: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """[X | y]^T [X | y] in fp64 from fp32 GEMMs (the device path of ``lasso_gram`` beyond the
    native kernel's column limit)."""
    m, n = X.shape
    dev = X.device
    # wider device rows: X^T X as a batched split-K GEMM (rows grouped into nb slabs of r rows, one
    # [n, r] x [r, n] product per slab: a plain X^T X has only (n / tile)^2 output tiles and leaves
    # the chip idle), X^T y likewise; slab partials summed in the data precision (fp32, or fp64 for
    # fp64 data), row blocks accumulated in fp64.
    # No [X | y] copy is materialised.
    Xc = X if X.is_contiguous() else X.contiguous()
    cd_t = torch.float64 if X.dtype == torch.float64 else torch.float32   # fp64 data stays fp64
    yv = y.reshape(-1).to(cd_t)
    G = torch.zeros((n + 1, n + 1), dtype=torch.float64, device=dev)
    nb = max(1, min(256, (256 << 20) // (4 * n * n)))
    step = max(nb * 1024, 1 << 20)
    for r0 in range(0, m, step):
        xb = Xc[r0: r0 + step].to(cd_t)
        yb = yv[r0: r0 + step]
        rows = xb.shape[0]
        r = rows // nb
        if r >= 256:
            x3 = xb[: nb * r].reshape(nb, r, n)
            y3 = yb[: nb * r].reshape(nb, r, 1)
            xtx = torch.bmm(x3.transpose(1, 2), x3).sum(0)
            xy = torch.bmm(x3.transpose(1, 2), y3).sum(0).reshape(n)
            xb, yb = xb[nb * r:], yb[nb * r:]
        else:
            xtx = torch.zeros((n, n), dtype=cd_t, device=dev)
            xy = torch.zeros(n, dtype=cd_t, device=dev)
        if xb.shape[0]:
            xtx = xtx + xb.T @ xb
            xy = xy + xb.T @ yb
        G[:n, :n] += xtx.double()
        G[:n, n] += xy.double()
        G[n, :n] += xy.double()
        G[n, n] += torch.dot(yv[r0: r0 + step].double(), yv[r0: r0 + step].double())
    return G


def lasso_gram(X: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Unnormalised augmented Gram matrix [X | y]^T [X | y] of the local rows, float64
    [(n+1), (n+1)] (``csrc/lasso_gram.hip``: one pass, register accumulators, fp64 block partials).

    Device fp32 with n + 1 <= 24 columns: the native kernel. Otherwise row blocks of fp32 GEMMs
    accumulated in fp64 (host tensors: fp64 GEMM)."""
    m, n = X.shape
    dev = X.device
    if m == 0:
        return torch.zeros((n + 1, n + 1), dtype=torch.float64, device=dev)
    if use_native(X) and X.dtype == torch.float32 and n + 1 <= lib().ha_lasso_gram_max_cols():
        L = lib()
        Xc = X if X.stride(-1) == 1 else X.contiguous()
        yc = y.reshape(-1).to(torch.float32).contiguous()
        blocks = L.ha_lasso_gram_blocks(m, num_cus(dev))
        if _GRAM_BLOCKS_PER_CU > 0:
            blocks = max(1, min(blocks, _GRAM_BLOCKS_PER_CU * num_cus(dev)))
        nc = n + 1
        T = nc * (nc + 1) // 2
        part = torch.empty((blocks, T), dtype=torch.float64, device=dev)
        check(L.ha_lasso_gram(_ptr(Xc), m, n, Xc.stride(0), _ptr(yc), _ptr(part), blocks, _GRAM_UNROLL,
                              ctypes.c_void_p(stream_ptr(dev))), "ha_lasso_gram")
        tri = part.sum(0)
        iu = torch.triu_indices(nc, nc, device=dev)
        G = torch.zeros((nc, nc), dtype=torch.float64, device=dev)
        G[iu[0], iu[1]] = tri
        return G + torch.triu(G, 1).T
    if not X.is_cuda:
        A = torch.cat([X, y.reshape(-1, 1).to(X.dtype)], dim=1).double()
        return A.T @ A
    return _gram_blocked(X, y)


def lasso_cd(G: torch.Tensor, b: torch.Tensor, lam: float, max_iter: int, tol: Optional[float],
             theta: torch.Tensor) -> int:
    """Cyclic coordinate descent on the normal equations (``G`` = X^T X / m, ``b`` = X^T y / m,
    float64), updating ``theta`` (float64, start values) in place with the reference's rule
    (feature 0 = intercept, not thresholded); sweeps stop when the RMS change of theta drops
    below ``tol``. Device: ONE single-wavefront kernel runs every sweep. Returns the sweep count."""
    n = G.shape[0]
    t = -1.0 if tol is None else float(tol)
    if use_native(G) and n <= 2048:
        L = lib()
        Gc = G if G.stride(-1) == 1 else G.contiguous()
        bc = b.contiguous()
        it = torch.zeros(1, dtype=torch.int32, device=G.device)
        check(L.ha_lasso_cd(_ptr(Gc), n, Gc.stride(0), _ptr(bc), ctypes.c_double(lam), int(max_iter),
                            ctypes.c_double(t), _ptr(theta), _ptr(it), ctypes.c_void_p(stream_ptr(G.device))),
              "ha_lasso_cd")
        return int(it.item())
    import numpy as np

    g = G.detach().cpu().numpy()
    bb = b.detach().cpu().numpy()
    th = theta.detach().cpu().numpy().astype(np.float64).copy()
    it = 0
    while it < max_iter:
        it += 1
        d2 = 0.0
        for j in range(n):
            old = th[j]
            rho = bb[j] - float(g[j] @ th) + g[j, j] * old
            nw = rho if j == 0 else (rho + lam if rho < -lam else (rho - lam if rho > lam else 0.0))
            th[j] = nw
            d2 += (nw - old) ** 2
        if t >= 0 and (d2 / n) ** 0.5 < t:
            break
    theta.copy_(torch.from_numpy(th))
    return it


def lasso_prepare(X: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(X^T contiguous [n, m], sum of squares per column [n]) in one pass over X."""
    m, n = X.shape
    if use_native(X) and X.dtype == torch.float32 and X.stride(-1) == 1:
        L = lib()
        XT = torch.empty((n, m), dtype=torch.float32, device=X.device)
        colsq = torch.empty(n, dtype=torch.float32, device=X.device)
        colpart = torch.empty(max(1, L.ha_lasso_prepare_scratch(m, n)), dtype=torch.float32, device=X.device)
        check(L.ha_lasso_prepare(_ptr(X), m, n, X.stride(0), _ptr(XT), XT.stride(0), _ptr(colsq), _ptr(colpart),
                                 ctypes.c_void_p(stream_ptr(X.device))), "ha_lasso_prepare")
        return XT, colsq
    XT = X.t().contiguous()
    return XT, (XT * XT).sum(1)


class LassoSweep:
    """A reusable coordinate-descent sweep over fixed (XT, r, theta, colsq) buffers.

    On a single device the sweep's 2n+1 launches are captured ONCE into a hipGraph
    (``torch.cuda.CUDAGraph``) and replayed, so a sweep costs one graph launch instead of
    2n+1 kernel launches plus the per-call Python/ctypes overhead. Distributed sweeps (a scalar
    all-reduce per coordinate) and host tensors run :func:`lasso_epoch` directly."""

    def __init__(self, XT: torch.Tensor, r: torch.Tensor, theta: torch.Tensor, colsq: torch.Tensor, lam: float,
                 m_global: int, allreduce=None, use_graph: bool = True):
        self.args = (XT, r, theta, colsq, lam, m_global, allreduce)
        self.graph = None
        self.use_graph = (use_graph and allreduce is None and XT.is_cuda and use_native(XT)
                          and XT.dtype == torch.float32 and XT.shape[0] >= 2
                          and os.environ.get("HEAT_AMD_NO_GRAPHS", "0") != "1")

    def __call__(self) -> None:
        if not self.use_graph:
            lasso_epoch(*self.args)
            return
        if self.graph is None:
            side = torch.cuda.Stream(device=self.args[0].device)
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                lasso_epoch(*self.args)  # this call's sweep (and the warm-up torch requires)
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                lasso_epoch(*self.args)  # captured, not executed
            self.graph = g
            return
        self.graph.replay()


def lasso_epoch(XT: torch.Tensor, r: torch.Tensor, theta: torch.Tensor, colsq: torch.Tensor, lam: float,
                m_global: int, allreduce=None):
    """One cyclic coordinate-descent sweep over all features (in place on ``r`` and ``theta``).

    ``XT`` [n_features, m_local] (features contiguous), ``r`` residual [m_local], ``theta`` [n],
    ``colsq`` = <X_j, X_j>/m [n]. ``allreduce(t)`` sums a 1-element device tensor over the ranks
    (None for a single process). Feature 0 is the intercept column (not thresholded)."""
    n = XT.shape[0]
    m = XT.shape[1]
    inv_m = 1.0 / float(m_global)
    if use_native(XT) and XT.dtype == torch.float32:
        L = lib()
        s = ctypes.c_void_p(stream_ptr(XT.device))
        ncu = num_cus(XT.device)
        # [result, arrival counter (zero), pad, per-workgroup slots]: deterministic dot products
        partial = torch.zeros(L.ha_lasso_partial_floats(ncu), dtype=torch.float32, device=XT.device)
        delta = torch.zeros(1, dtype=torch.float32, device=XT.device)
        for j in range(n):
            check(L.ha_lasso_pass(_ptr(XT), m, XT.stride(0), j - 1, j, _ptr(delta), _ptr(r), _ptr(partial), ncu, s),
                  "ha_lasso_pass")
            if allreduce is not None:
                allreduce(partial[:1])
            check(L.ha_lasso_update(_ptr(theta), j, _ptr(partial), _ptr(colsq), ctypes.c_float(lam),
                                    ctypes.c_float(inv_m), _ptr(delta), 1 if j == 0 else 0, s), "ha_lasso_update")
        # apply the last coordinate's change to the residual
        check(L.ha_lasso_pass(_ptr(XT), m, XT.stride(0), n - 1, -1, _ptr(delta), _ptr(r), _ptr(partial), ncu, s),
              "ha_lasso_pass")
        return
    for j in range(n):
        xj = XT[j]
        p = (xj * r).sum().reshape(1)
        if allreduce is not None:
            allreduce(p)
        old = theta[j].clone()
        rho = p[0] * inv_m + old * colsq[j]
        if j == 0:
            new = rho
        else:
            new = torch.where(rho < -lam, rho + lam, torch.where(rho > lam, rho - lam, torch.zeros_like(rho)))
        theta[j] = new
        r -= (new - old) * xj


# ------------------------------------------------------------------------------- fp16x3 split GEMM
def split_planes(X: torch.Tensor, axis: int, pattern: str, contract_dim: int):
    """fp16x3 operand of :func:`gemm_f16x3` (see ``csrc/gemm_split.hip``).

    ``X`` is a logical 2-D fp32 operand whose dimension ``1 - contract_dim`` carries the power-of-two
    scales; the result is the logical operand with the contraction dimension tripled into the
    segments named by ``pattern`` ("hhl": hi, hi, lo; "hlh": hi, lo, hi), laid out in X's own
    memory order (row- or column-major) so the split streams coalesced. Returns (planes, int32
    exponents, non-finite flag tensor)."""
    L = lib()
    st = ctypes.c_void_p(stream_ptr(X.device))
    colmajor = X.stride(0) == 1 and X.stride(1) != 1
    P = X.t() if colmajor else (X if X.stride(1) == 1 else X.contiguous())
    if P.stride(1) != 1:
        P = P.contiguous()
    R, C = P.shape
    # physical axis carrying the scales
    scale_dim = 1 - contract_dim
    phys_axis = (1 - scale_dim) if colmajor else scale_dim
    ex = torch.empty(R if phys_axis == 0 else C, dtype=torch.int32, device=X.device)
    flag = torch.zeros(1, dtype=torch.int32, device=X.device)
    # physical contraction axis = the one that is not the scale axis
    pc = 1 - phys_axis
    if pc == 1:
        out = torch.empty((R, 3 * C), dtype=torch.float16, device=X.device)
        seg = [out[:, i * C:(i + 1) * C] for i in range(3)]
    else:
        out = torch.empty((3 * R, C), dtype=torch.float16, device=X.device)
        seg = [out[i * R:(i + 1) * R] for i in range(3)]
    h0, h1, lo = (seg[0], seg[1], seg[2]) if pattern == "hhl" else (seg[0], seg[2], seg[1])
    rc = 2
    if phys_axis == 0:   # per-row scales: absmax and split fused (one wave per row)
        rc = L.ha_split3_rows(_ptr(P), R, C, P.stride(0), _ptr(h0), _ptr(h1), _ptr(lo), out.stride(0), _ptr(ex),
                              _ptr(flag), st)
    if rc == 2:
        mx = torch.empty(ex.shape[0], dtype=torch.float32, device=X.device)
        check(L.ha_split_absmax(_ptr(P), R, C, P.stride(0), phys_axis, _ptr(mx), _ptr(flag), st),
              "ha_split_absmax")
        rc = L.ha_split3(_ptr(P), R, C, P.stride(0), phys_axis, _ptr(mx), _ptr(h0), _ptr(h1), _ptr(None),
                         _ptr(lo), out.stride(0), _ptr(ex), st)
    check(rc, "ha_split3")
    return (out.t() if colmajor else out), ex, flag


def _is_gram(a: torch.Tensor, b: torch.Tensor) -> bool:
    """a is the transposed view of a row-major b (X^T X)."""
    return (a.data_ptr() == b.data_ptr() and a.shape == (b.shape[1], b.shape[0]) and b.stride(1) == 1
            and a.stride() == (b.stride(1), b.stride(0)))


def _split_gram(X: torch.Tensor):
    """Both operands of X^T X from one split: column scales of X, buffer W = [h; h; l; h]
    (4 planes instead of 6, one absmax and one split pass instead of two each)."""
    L = lib()
    st = ctypes.c_void_p(stream_ptr(X.device))
    R, C = X.shape
    mx = torch.empty(C, dtype=torch.float32, device=X.device)
    ex = torch.empty(C, dtype=torch.int32, device=X.device)
    flag = torch.zeros(1, dtype=torch.int32, device=X.device)
    check(L.ha_split_absmax(_ptr(X), R, C, X.stride(0), 1, _ptr(mx), _ptr(flag), st), "ha_split_absmax")
    W = torch.empty((4 * R, C), dtype=torch.float16, device=X.device)
    check(L.ha_split3(_ptr(X), R, C, X.stride(0), 1, _ptr(mx), _ptr(W[:R]), _ptr(W[R:2 * R]), _ptr(W[3 * R:]),
                      _ptr(W[2 * R:3 * R]), C, _ptr(ex), st), "ha_split3")
    return W[R:].t(), W[:3 * R], ex, flag


def gemm_f16x3(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 ``a @ b`` on the FP16 matrix cores: both operands split into fp16 hi/lo planes with
    power-of-two row (a) / column (b) scales, ONE fp16-in/fp32-out library GEMM over the tripled
    contraction (hi.hi + hi.lo + lo.hi), exact ldexp unscaling. Accuracy of an fp32 GEMM (errors
    <= ~2^-21 |a||b| per product, fp32 accumulation), ~2.7x its speed on MI355X. Operands holding
    inf/nan go to the fp32 GEMM (one host sync per call for that check). ``out``: a row-major
    fp32 [M, N] tensor (e.g. a row block of a larger result) the GEMM writes directly."""
    def fallback():
        if out is None:
            return torch.matmul(a, b)
        return torch.mm(a, b, out=out)

    if not (a.is_cuda and use_native(a)) or a.dtype != torch.float32 or b.dtype != torch.float32 \
            or a.dim() != 2 or b.dim() != 2:
        return fallback()
    M, K = a.shape
    N = b.shape[1]
    if M == 0 or N == 0 or K == 0:
        return fallback()
    if out is not None and (out.shape != (M, N) or out.dtype != torch.float32 or out.stride(1) != 1):
        raise ValueError("gemm_f16x3: out must be a row-major float32 [M, N] tensor")
    if _is_gram(a, b):
        A3, B3, ea, fa = _split_gram(b)
        eb, fb = ea, fa
    else:
        A3, ea, fa = split_planes(a, 0, "hhl", 1)
        B3, eb, fb = split_planes(b, 1, "hlh", 0)
    if int((fa + fb).item()) != 0:
        return fallback()
    if out is None:
        C = torch.mm(A3, B3, out_dtype=torch.float32)
    else:
        C = torch.mm(A3, B3, out_dtype=torch.float32, out=out)
    check(lib().ha_split_unscale(_ptr(C), M, N, C.stride(0), _ptr(ea), _ptr(eb),
                                 ctypes.c_void_p(stream_ptr(a.device))), "ha_split_unscale")
    return C


# --------------------------------------------------------------------------------------------- selection
_SEL_DTYPES = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.int32: 3, torch.int16: 4,
               torch.int8: 5, torch.uint8: 6, torch.bool: 6}
_KEY_IDENTITY = -(1 << 63)


def argreduce_supported(t: torch.Tensor, max_index: int) -> bool:
    """Whether the packed-key kernels handle ``t`` (device, <= 32-bit dtype, indices < 2^32 - 1)."""
    return t.is_cuda and t.dtype in _SEL_DTYPES and max_index < 0xFFFFFFFF and use_native(t)


def argreduce_keys(t: torch.Tensor, axis: Optional[int], smallest: bool, displ: int = 0,
                   gextent: Optional[int] = None, split: Optional[int] = None) -> torch.Tensor:
    """Packed (value, first index) keys of an arg-reduction of the device tensor ``t``
    (``csrc/select.hip``): int64, the larger key is the winner, so combining partial results -
    across ranks too - is an integer MAX (one RCCL all-reduce).

    axis None: one key over all elements; the index is the GLOBAL flat index when ``t`` is the
    local block of an array split along ``split`` whose extent is ``gextent`` and this block starts
    at ``displ``. axis given: keys of shape ``t.shape`` without ``axis``, indices along ``axis``
    offset by ``displ``."""
    t = t.contiguous()
    if t.dtype == torch.bool:
        t = t.view(torch.uint8)
    shp = list(t.shape)
    L = lib()
    if axis is None:
        s = 0 if split is None else split
        O = int(np.prod(shp[:s])) if shp else 1
        Lx = shp[s] if shp else 1
        I = int(np.prod(shp[s + 1:])) if shp else 1
        gL = gextent if gextent is not None else Lx
        out = torch.full((1,), _KEY_IDENTITY, dtype=torch.int64, device=t.device)
        mode = 0
    else:
        O = int(np.prod(shp[:axis]))
        Lx = shp[axis]
        I = int(np.prod(shp[axis + 1:]))
        gL = Lx
        out = torch.full(shp[:axis] + shp[axis + 1:], _KEY_IDENTITY, dtype=torch.int64, device=t.device)
        mode = 1
    check(L.ha_argreduce(_ptr(t), _SEL_DTYPES[t.dtype], O, Lx, I, gL, displ, mode, int(smallest), _ptr(out),
                         ctypes.c_void_p(stream_ptr(t.device))), "ha_argreduce")
    return out


def argreduce_decode(keys: torch.Tensor) -> torch.Tensor:
    """Indices of packed arg-reduction keys (-1 where no element contributed)."""
    idx = 0xFFFFFFFF - (keys & 0xFFFFFFFF)
    return torch.where(keys == _KEY_IDENTITY, torch.full_like(idx, -1), idx)


def topk_rows(t: torch.Tensor, k: int, dim: int, largest: bool, displ: int = 0):
    """Top-k (k <= 32) along ``dim`` of a device tensor with one wave per row (``csrc/select.hip``):
    values sorted best first, int64 indices (+ ``displ``); ties resolve to the smaller index; NaN
    ranks like torch.topk (largest). None where the kernel does not apply."""
    if not (t.is_cuda and t.dtype in _SEL_DTYPES and t.dtype != torch.bool and 0 < k <= 32
            and t.shape[dim] >= k and t.shape[dim] < 0xFFFFFFFF and use_native(t)):
        return None
    x = t.movedim(dim, -1).contiguous()
    lead = tuple(x.shape[:-1])
    O = int(np.prod(lead)) if lead else 1
    Lr = x.shape[-1]
    vals = torch.empty(lead + (k,), dtype=x.dtype, device=x.device)
    idx = torch.empty(lead + (k,), dtype=torch.int64, device=x.device)
    if O:
        check(lib().ha_topk_rows(_ptr(x), _SEL_DTYPES[x.dtype], O, Lr, displ, k, int(not largest), _ptr(vals),
                                 _ptr(idx), ctypes.c_void_p(stream_ptr(x.device))), "ha_topk_rows")
    return vals.movedim(-1, dim), idx.movedim(-1, dim)


# --------------------------------------------------------------------------------------------- exact fp32 GEMM
def _gemm_operand(t: torch.Tensor, contig_dim: int):
    """(tensor, ld, alt_major) for a 2-D fp32 operand: alt_major False when dim ``contig_dim`` is
    contiguous, True when the other dim is; otherwise a contiguous copy."""
    if t.stride(contig_dim) == 1 and t.stride(1 - contig_dim) >= max(1, t.shape[contig_dim]):
        return t, t.stride(1 - contig_dim), False
    if t.stride(1 - contig_dim) == 1 and t.stride(contig_dim) >= max(1, t.shape[1 - contig_dim]):
        return t, t.stride(contig_dim), True
    t = t.contiguous()
    return t, t.stride(0) if contig_dim == 1 else t.stride(1), contig_dim == 0


_GEMM_BK = int(os.environ.get("HEAT_GEMM_VARIANT", "4"))  # 128-tile exact GEMM block: 2 = 128x128, 4 = 128x256
_SPLITK = os.environ.get("HEAT_GEMM_SPLITK", "1") != "0"
_SPLITK_MIN_K = 1024          # K per slice: the pipeline's prologue / C epilogue amortised over >= 64 k-stages
_SPLITK_MAX_BYTES = 1 << 29   # partial buffer cap


def _splitk_slices(M: int, N: int, K: int, device) -> int:
    """Number of K slices for a 256 x 256-tile GEMM whose output tiles cover less than half the CUs
    (1 = no split): enough slices for one workgroup per CU, each >= _SPLITK_MIN_K deep."""
    if not _SPLITK:
        return 1
    tiles = -(-M // 256) * -(-N // 256)
    ncu = num_cus(device)
    if 2 * tiles > ncu or K < 2 * _SPLITK_MIN_K:
        return 1
    s = min(-(-ncu // tiles), K // _SPLITK_MIN_K, max(1, _SPLITK_MAX_BYTES // (4 * M * N)))
    return max(1, s)
_HA_UNSUPPORTED = 2


def gemm_f32(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
             accumulate: bool = False, alpha: float = 1.0, slices: Optional[int] = None,
             b_upper: bool = False) -> torch.Tensor:
    """Exact fp32 ``alpha * a @ b`` (``+ out`` when ``accumulate``) on the f32-input matrix cores:
    fp32 products and accumulation in k order like any fp32 GEMM, every operand layout
    (row-/column-major views such as ``x.T @ x``) without a copy, 64-bit offsets (no 4 GB operand
    limit). The 256 x 256-tile pipelined kernel (``csrc/gemm_tiled.hip: gemm_f32t``) takes
    16-byte-aligned operands whose contiguous extents are multiples of 4; anything else runs on
    the 128-tile kernel (``csrc/gemm_mfma.hip``). ``out``: a row-major fp32 [M, N] view (e.g. a
    row block of a larger result). ``b_upper``: b is square and upper triangular (the caller's
    guarantee, e.g. an R^-1 factor): output column tile n0 contracts only k < n0 + 256, so the zero
    half of K is never loaded or multiplied (~half the work at K = N = 4096)."""
    if not (a.is_cuda and use_native(a)) or a.dtype != torch.float32 or b.dtype != torch.float32 \
            or a.dim() != 2 or b.dim() != 2:
        res = alpha * (a @ b) if alpha != 1.0 else a @ b
        if out is None:
            return res
        return out.add_(res) if accumulate else out.copy_(res)
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K:
        raise ValueError("gemm_f32: inner dimensions differ: {} vs {}".format(K, b.shape[0]))
    if out is None:
        out = torch.zeros((M, N), dtype=torch.float32, device=a.device) if accumulate else \
            torch.empty((M, N), dtype=torch.float32, device=a.device)
    elif out.shape != (M, N) or out.dtype != torch.float32 or (N > 1 and out.stride(1) != 1):
        raise ValueError("gemm_f32: out must be a row-major float32 [M, N] tensor")
    if M == 0 or N == 0:
        return out
    if K == 0:
        return out if accumulate else out.zero_()
    A, lda, a_km = _gemm_operand(a, 1)      # row-major: k contiguous; k-major: m contiguous
    B, ldb, b_nm = _gemm_operand(b, 1)      # k-major: n contiguous; n-major: k contiguous
    L = lib()
    st = ctypes.c_void_p(stream_ptr(a.device))
    ldc = out.stride(0) if M > 1 else N
    ub = _TG_B_UPPER if (b_upper and K == N) else 0
    if slices is None:
        slices = _splitk_slices(M, N, K, a.device)
    if slices > 1:
        # few 256 x 256 output tiles: split K so the grid fills the CUs, fp32 partial per slice,
        # slices summed in fixed order (fp64) with alpha / accumulate in the same pass
        P = torch.empty(slices * M * N, dtype=torch.float32, device=a.device)
        rc = L.ha_gemm_f32t(_ptr(A), _ptr(B), _ptr(P), M, N, K, lda, ldb, N, int(a_km), int(not b_nm), 1.0, 0, ub,
                            slices, M * N, st)
        if rc == 0:
            check(L.ha_sum_slices32(_ptr(P), L.ha_gemm_tiled_slices(K, slices), M, N, M * N, _ptr(out), ldc,
                                    float(alpha), int(accumulate), st), "ha_sum_slices32")
            return out
    rc = L.ha_gemm_f32t(_ptr(A), _ptr(B), _ptr(out), M, N, K, lda, ldb, ldc, int(a_km), int(not b_nm),
                        float(alpha), int(accumulate), ub, 1, 0, st)
    if rc == _HA_UNSUPPORTED:
        if alpha != 1.0:
            tmp = gemm_f32(a, b)
            return out.add_(tmp, alpha=alpha) if accumulate else torch.mul(tmp, alpha, out=out)
        rc = L.ha_gemm_f32(_ptr(A), _ptr(B), _ptr(out), M, N, K, lda, ldb, ldc, int(a_km), int(b_nm),
                           int(accumulate), _GEMM_BK, st)
    check(rc, "ha_gemm_f32")
    return out


_GEMM_SMALL = os.environ.get("HEAT_GEMM_SMALL", "1") != "0"
# the 128-tile kernel: "mid" (LDS-DMA pipelined, csrc/gemm_mid.hip: gemm_f32m) or "s" (the round-5
# register-staged gemm_f32s, A/B)
_GEMM_MID = os.environ.get("HEAT_GEMM_MID", "1") != "0"
# products with K <= this on the 64 x 64-tile gemm_f32m by default (the Householder in-block
# updates, K = 32: 1.25e6 x 4096 factor + Q 1.346 -> 1.322 s, profiles/gemm_mid_r06.jsonl); 0 = off
_GM64_MAXK = int(os.environ.get("HEAT_GM64_MAXK", "64"))


def gemm_f32_small(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, alpha: float = 1.0,
                   accumulate: bool = False, slices: Optional[int] = None,
                   kernel: Optional[str] = None) -> Optional[torch.Tensor]:
    """Exact fp32 ``alpha * a @ b`` (``+ out`` when ``accumulate``) on a 128 x 128-tile kernel with
    split-K, two workgroups per CU: the products whose 256 x 256 tiles cannot fill the GPU (1024^3
    .. 6144^3) and short-K tall updates (the Householder rank-256 update). ``kernel``: "mid"
    (default: LDS-DMA pipeline, ``csrc/gemm_mid.hip: gemm_f32m``, 256 x 128 tiles where they fill
    the GPU, else 128 x 128; "mid128" / "mid256" / "mid64" / "mid128x64" force a tile) or "s" (register-staged,
    ``csrc/gemm_small.hip: gemm_f32s``; also where gemm_f32m's operand requirements fail). Any
    row-/column-major operand views; None where neither kernel applies (host tensors, unaligned
    operands: the caller picks another GEMM)."""
    if not (_GEMM_SMALL and a.is_cuda and use_native(a)) or a.dtype != torch.float32 or b.dtype != torch.float32 \
            or a.dim() != 2 or b.dim() != 2:
        return None
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K:
        raise ValueError("gemm_f32_small: inner dimensions differ: {} vs {}".format(K, b.shape[0]))
    if out is not None and (out.shape != (M, N) or out.dtype != torch.float32 or (N > 1 and out.stride(1) != 1)):
        raise ValueError("gemm_f32_small: out must be a row-major float32 [M, N] tensor")
    if out is None:
        out = torch.zeros((M, N), dtype=torch.float32, device=a.device) if accumulate else \
            torch.empty((M, N), dtype=torch.float32, device=a.device)
    if M == 0 or N == 0:
        return out
    if K == 0:
        return out if accumulate else out.zero_()
    A, lda, a_km = _gemm_operand(a, 1)
    B, ldb, b_nm = _gemm_operand(b, 1)
    if A.data_ptr() % 16 or B.data_ptr() % 16 or lda % 4 or ldb % 4:
        return None
    L = lib()
    st = ctypes.c_void_p(stream_ptr(a.device))
    ldc = out.stride(0) if M > 1 else N
    tiles = -(-M // 128) * -(-N // 128)
    ncu = num_cus(a.device)
    if slices is None:
        slices = 1
        if tiles < 2 * ncu and K >= 512:   # two workgroups per CU: split K over the missing ones
            slices = max(1, min(-(-2 * ncu // tiles), K // 256, _SPLITK_MAX_BYTES // (4 * M * N)))
    if kernel is None and _GEMM_MID and K <= _GM64_MAXK:
        kernel = "mid64"   # short K: per-tile latency dominates, more (smaller) tiles per CU hide it
    kernel = kernel or ("mid" if _GEMM_MID else "s")
    mid = kernel.startswith("mid")
    tile = {"mid128": 1, "mid256": 2, "mid64": 3, "mid128x64": 4, "mid128g2": 5}.get(kernel, 0)
    if mid and ((M if a_km else K) % 4 or (N if not b_nm else K) % 4 or min(M, N, K) < 4):
        mid = False          # gemm_f32m's operand requirements (contiguous extents multiples of 4)
    if mid:
        used_fn = L.ha_gemm_f32m_slices
        launch = lambda *args: L.ha_gemm_f32m(*args[:-1], tile, args[-1])   # noqa: E731
        bflag = int(not b_nm)            # gemm_f32m takes "B k-major"
    else:
        launch, used_fn = L.ha_gemm_f32s, L.ha_gemm_f32s_slices
        bflag = int(b_nm)                # gemm_f32s takes "B n-major"
    name = "ha_gemm_f32m" if mid else "ha_gemm_f32s"
    if slices > 1:
        used = used_fn(K, slices)
        if used > 1:
            P = torch.empty(used * M * N, dtype=torch.float32, device=a.device)
            check(launch(_ptr(A), _ptr(B), _ptr(P), M, N, K, lda, ldb, N, int(a_km), bflag, 1.0, 0, slices, M * N, st),
                  name)
            check(L.ha_sum_slices32(_ptr(P), used, M, N, M * N, _ptr(out), ldc, float(alpha), int(accumulate), st),
                  "ha_sum_slices32")
            return out
    check(launch(_ptr(A), _ptr(B), _ptr(out), M, N, K, lda, ldb, ldc, int(a_km), bflag, float(alpha),
                 int(accumulate), 1, 0, st), name)
    return out


class H3Planes(NamedTuple):
    """fp16 hi/lo planes of one GEMM operand in the K8-panel layout [Kp/8][Rp][8] (rows = the
    operand's non-contracted dimension, padded to 256; K padded to 16; zero padding), int32
    power-of-two row exponents [Rp], and the device inf/nan flag."""
    hi: torch.Tensor
    lo: torch.Tensor
    ex: torch.Tensor
    flag: torch.Tensor
    rows: int
    Rp: int
    Kp: int


def h3_planes(x: torch.Tensor, contract_dim: int) -> H3Planes:
    """Split a 2-D fp32 GEMM operand for :func:`gemm_h3`: ``contract_dim`` is the dimension summed
    over (1 for the left operand A[M, K], 0 for the right operand B[K, N]); the other dimension
    gets one power-of-two scale per index (``csrc/gemm_tiled.hip: tg_split_rows / tg_split_cols``:
    one read of x, fully coalesced plane writes)."""
    L = lib()
    st = ctypes.c_void_p(stream_ptr(x.device))
    rows_dim = 1 - contract_dim
    R, K = x.shape[rows_dim], x.shape[contract_dim]
    Rp, Kp = max(256, (R + 255) // 256 * 256), max(16, (K + 15) // 16 * 16)
    hi = torch.empty((Kp // 8, Rp, 8), dtype=torch.float16, device=x.device)
    lo = torch.empty_like(hi)
    ex = torch.empty(Rp, dtype=torch.int32, device=x.device)
    flag = torch.zeros(1, dtype=torch.int32, device=x.device)
    # physical layout: rows of the operand contiguous along k ("rows" split) or along rows ("cols")
    if x.stride(contract_dim) == 1 and x.stride(rows_dim) >= max(1, K):
        P = x if contract_dim == 1 else x.t()           # [R][K], unit stride along K
        check(L.ha_h3_split_rows(_ptr(P), R, K, P.stride(0), Rp, Kp, _ptr(hi), _ptr(lo), _ptr(ex), _ptr(flag), st),
              "ha_h3_split_rows")
    else:
        P = x.t() if contract_dim == 1 else x           # [K][R], unit stride along R
        if P.stride(1) != 1 or P.stride(0) < max(1, R):
            P = P.contiguous()
        mx = torch.empty(R, dtype=torch.float32, device=x.device)
        check(L.ha_split_absmax(_ptr(P), K, R, P.stride(0), 1, _ptr(mx), _ptr(flag), st), "ha_split_absmax")
        check(L.ha_h3_split_cols(_ptr(P), K, R, P.stride(0), Rp, Kp, _ptr(mx), _ptr(hi), _ptr(lo), _ptr(ex), st),
              "ha_h3_split_cols")
    return H3Planes(hi, lo, ex, flag, R, Rp, Kp)


_TG_B_UPPER = 2   # gemm_tiled.hip: bit of the ``upper`` argument - B upper triangular, K clipped per column tile


def gemm_h3_planes(pa: H3Planes, pb: H3Planes, out: torch.Tensor, alpha: float = 1.0, accumulate: bool = False,
                   b_upper: bool = False):
    """``out (+)= alpha * A @ B`` from pre-split operands (see :func:`h3_planes`). ``b_upper``: B is
    upper triangular (caller's guarantee), so output column tile n0 contracts only k < n0 + 256."""
    ub = _TG_B_UPPER if b_upper else 0
    if pa.Kp != pb.Kp:
        raise ValueError("gemm_h3_planes: contraction lengths differ")
    M, N = pa.rows, pb.rows
    L = lib()
    st = ctypes.c_void_p(stream_ptr(out.device))
    slices = _splitk_slices(M, N, pa.Kp, out.device)
    if slices > 1:   # few output tiles: split K (see gemm_f32)
        P = torch.empty(slices * M * N, dtype=torch.float32, device=out.device)
        check(L.ha_gemm_h3t(_ptr(pa.hi), _ptr(pa.lo), _ptr(pb.hi), _ptr(pb.lo), _ptr(pa.ex), _ptr(pb.ex), _ptr(P), M,
                            N, pa.Kp, pa.Rp, pb.Rp, N, 1.0, 0, ub, slices, M * N, st), "ha_gemm_h3t")
        check(L.ha_sum_slices32(_ptr(P), L.ha_gemm_tiled_slices(pa.Kp, slices), M, N, M * N, _ptr(out),
                                out.stride(0) if M > 1 else N, float(alpha), int(accumulate), st), "ha_sum_slices32")
        return out
    check(L.ha_gemm_h3t(_ptr(pa.hi), _ptr(pa.lo), _ptr(pb.hi), _ptr(pb.lo), _ptr(pa.ex), _ptr(pb.ex), _ptr(out),
                        M, N, pa.Kp, pa.Rp, pb.Rp, out.stride(0) if M > 1 else N, float(alpha), int(accumulate),
                        ub, 1, 0, st), "ha_gemm_h3t")
    return out


def gemm_h3(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, alpha: float = 1.0,
            accumulate: bool = False, b_upper: bool = False) -> Optional[torch.Tensor]:
    """fp32 ``alpha * a @ b`` (``+ out`` when ``accumulate``) by the fused fp16x3 MFMA kernel
    (``csrc/gemm_tiled.hip: gemm_h3t``): power-of-two scaled fp16 hi/lo planes of both operands,
    one 256 x 256-tile kernel forming hi.hi + hi.lo + lo.hi with fp32 accumulation and the exact
    unscale in its epilogue. Accuracy of an fp32 GEMM (errors <= ~2^-21 |a||b| per product).
    ``x.T @ x`` splits x once. Returns None for non-finite operands (the caller falls back; the
    check is one host sync). ``b_upper``: b is upper triangular (see :func:`gemm_f32`)."""
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        out = torch.zeros((M, N), dtype=torch.float32, device=a.device) if accumulate else \
            torch.empty((M, N), dtype=torch.float32, device=a.device)
    elif out.shape != (M, N) or out.dtype != torch.float32 or (N > 1 and out.stride(1) != 1):
        raise ValueError("gemm_h3: out must be a row-major float32 [M, N] tensor")
    if M == 0 or N == 0:
        return out
    if K == 0:
        return out if accumulate else out.zero_()
    pa = h3_planes(a, 1)
    pb = pa if _is_gram(a, b) else h3_planes(b, 0)
    if int((pa.flag + pb.flag).item()) != 0:
        return None
    return gemm_h3_planes(pa, pb, out, alpha, accumulate, b_upper=b_upper and K == N)


_GRAM_KCHUNK = max(16, int(os.environ.get("HEAT_GRAM_KCHUNK", "4096")) // 16 * 16)
_GRAM_PARTIAL_BYTES = 1 << 30
# K slice of the Gram behind ht.matmul(X.T, X) (fp32 result): 16384 rows per fp32 slice sum, a
# quarter of the partial-sum traffic of CholeskyQR's 4096 (1.25e6 x 4096, tools/r5/gpu_gramk.sh:
# 172 / 166 / 163 / 164 ms at 4096 / 8192 / 16384 / 32768) - still far finer than one fp32 sum
_GRAM_MATMUL_KCHUNK = max(16, int(os.environ.get("HEAT_GRAM_MATMUL_KCHUNK", "16384")) // 16 * 16)


def gram_product(a: torch.Tensor, b: torch.Tensor) -> Optional[torch.Tensor]:
    """``a @ b`` as a symmetric fp32 matrix when it is the Gram product of ONE device fp32 matrix
    X - ``X^T X`` (a the transposed view of a row-major b) or ``X X^T`` (b the transposed view of a
    row-major a) - computed once per upper-triangle tile pair (``gram64``'s upper-tile split-K
    launches, half the MFMA work of the full product) and mirrored, so the result is exactly
    symmetric; None when the operands are not of that form."""
    if not (a.is_cuda and use_native(a)) or a.dtype != torch.float32 or b.dtype != torch.float32:
        return None
    if _is_gram(a, b):
        g = gram64(b, kchunk=_GRAM_MATMUL_KCHUNK)
    elif _is_gram(b, a):
        g = gram64(a, rows=True, kchunk=_GRAM_MATMUL_KCHUNK)
    else:
        return None
    u = torch.triu(g)
    return (u + torch.triu(u, 1).t()).float()


def gram64(x: torch.Tensor, exact: Optional[bool] = None, rows: bool = False,
           kchunk: Optional[int] = None) -> torch.Tensor:
    """Upper triangle (lower triangle zero) of the Gram matrix x^T x of a tall fp32 block as an
    fp64 [n, n] tensor - the CholeskyQR Gram. One 256-tile MFMA launch per group of K slices
    (``csrc/gemm_tiled.hip``: upper-triangle tiles only, split-K over ``HEAT_GRAM_KCHUNK`` = 4096
    rows), fp32 accumulation inside a slice and the slices summed in fp64 in fixed order
    (``ha_sum_slices64``): the accumulation error of one fp32 sum over all 1.25e6 rows (~u sqrt(m) / 3
    = 4e-5 relative on the diagonal at m = 1.25e6) drops to ~u chunk / (3 sqrt(m)) = 7e-8. ``exact``: exact fp32
    products (``gemm_f32t``) instead of the fp16x3 split (``gemm_h3t``); default from
    torch.get_float32_matmul_precision() ("highest" -> exact). Host / fp64: an fp64 GEMM.
    ``rows``: the Gram of the ROWS, x x^T (x [n, m] row-major, contraction along its columns).
    ``kchunk``: rows per fp32 slice (a multiple of 16; default ``HEAT_GRAM_KCHUNK``)."""
    if rows:
        n, m = x.shape
    else:
        m, n = x.shape
    if not (x.is_cuda and use_native(x)) or x.dtype != torch.float32:
        xd = x.double()
        return torch.triu(xd @ xd.T if rows else xd.T @ xd)
    out = torch.zeros((n, n), dtype=torch.float64, device=x.device)
    if m == 0 or n == 0:
        return out
    if exact is None:
        exact = torch.get_float32_matmul_precision() == "highest"
    L = lib()
    st = ctypes.c_void_p(stream_ptr(x.device))
    kc = _GRAM_KCHUNK if kchunk is None else max(16, int(kchunk) // 16 * 16)
    group = max(1, min(-(-m // kc), _GRAM_PARTIAL_BYTES // (4 * n * n)))
    P = torch.empty(group * n * n, dtype=torch.float32, device=x.device)
    pa = None
    if not exact:
        pa = h3_planes(x, 1) if rows else h3_planes(x.t(), 1)
        if int(pa.flag.item()) != 0:
            pa = None
            exact = True
    if exact and rows and (x.stride(1) != 1 or x.stride(0) % 4 or x.data_ptr() % 16):
        x = x.contiguous()
    for k0 in range(0, m, group * kc):
        k1 = min(m, k0 + group * kc)
        slices = -(-(k1 - k0) // kc)
        if exact:
            if rows:   # A = x (row-major, k contiguous), B = x^T (n-major): columns k0..k1 of x
                xs = x[:, k0:k1]
                ok = xs.data_ptr() % 16 == 0 and (k1 - k0) % 4 == 0
                rc = L.ha_gemm_f32t(_ptr(xs), _ptr(xs), _ptr(P), n, n, k1 - k0, xs.stride(0), xs.stride(0), n, 0, 0,
                                    1.0, 0, 1, slices, n * n, st) if ok else _HA_UNSUPPORTED
            else:
                xs = x[k0:k1]
                if xs.stride(1) != 1 or xs.stride(0) % 4 or xs.data_ptr() % 16 or n % 4:
                    xs = xs.contiguous()
                rc = L.ha_gemm_f32t(_ptr(xs), _ptr(xs), _ptr(P), n, n, k1 - k0, xs.stride(0), xs.stride(0), n, 1, 1,
                                    1.0, 0, 1, slices, n * n, st)
            if rc == _HA_UNSUPPORTED:   # tiny / unaligned blocks: the 128-tile kernel, one slice
                res = gemm_f32(xs, xs.t()) if rows else gemm_f32(xs.t(), xs)
                out += torch.triu(res.double())
                continue
            check(rc, "ha_gemm_f32t")
            used = L.ha_gemm_tiled_slices(k1 - k0, slices)
        else:
            kp0 = k0                       # k0 is a multiple of kc (16 | kc): a plane panel boundary
            kp1 = min(pa.Kp, k0 + group * kc) if k1 == m else k1
            off = (kp0 // 8) * pa.Rp * 8 * 2   # bytes into the [Kp/8][Rp][8] fp16 planes
            check(L.ha_gemm_h3t(ctypes.c_void_p(pa.hi.data_ptr() + off), ctypes.c_void_p(pa.lo.data_ptr() + off),
                                ctypes.c_void_p(pa.hi.data_ptr() + off), ctypes.c_void_p(pa.lo.data_ptr() + off),
                                _ptr(pa.ex), _ptr(pa.ex), _ptr(P), n, n, kp1 - kp0, pa.Rp, pa.Rp, n, 1.0, 0, 1,
                                slices, n * n, st), "ha_gemm_h3t")
            used = L.ha_gemm_tiled_slices(kp1 - kp0, slices)
        check(L.ha_sum_slices64(_ptr(P), used, n, n, n * n, _ptr(out), n, 1, 1, st), "ha_sum_slices64")
    return out


def gemm_h3_v1(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """The round-2 128 x 128-tile fused fp16x3 kernel (``csrc/gemm_mfma.hip: gemm_h3``), kept for
    the A/B benchmark (``tools/microbench/gemm_bench.py``)."""
    M, K = a.shape
    N = b.shape[1]
    Kp = (K + 31) // 32 * 32
    A = a if a.stride(-1) == 1 else a.contiguous()
    BT = b.t() if b.stride(0) == 1 else b.t().contiguous()
    ahi, alo, ea, fa = _h3_rows(A, Kp)
    bhi, blo, eb, fb = _h3_rows(BT, Kp)
    if int((fa + fb).item()) != 0:
        return None
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    check(lib().ha_gemm_h3(_ptr(ahi), _ptr(alo), _ptr(bhi), _ptr(blo), _ptr(ea), _ptr(eb), _ptr(out), M, N, Kp,
                           out.stride(0) if M > 1 else N, ctypes.c_void_p(stream_ptr(a.device))), "ha_gemm_h3")
    return out


def gemm_f32_v1(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The round-2 128-tile exact fp32 kernel (``csrc/gemm_mfma.hip: gemm_f32``), for A/B benches."""
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    A, lda, a_km = _gemm_operand(a, 1)
    B, ldb, b_nm = _gemm_operand(b, 1)
    check(lib().ha_gemm_f32(_ptr(A), _ptr(B), _ptr(out), M, N, K, lda, ldb, out.stride(0) if M > 1 else N,
                            int(a_km), int(b_nm), 0, _GEMM_BK, ctypes.c_void_p(stream_ptr(a.device))), "ha_gemm_f32")
    return out


def _h3_rows(X: torch.Tensor, Kp: int):
    """fp16 hi/lo planes [R, Kp] (zero tail) + int32 row exponents of a row-major fp32 matrix X
    [R, K], and the device non-finite flag (the round-2 kernel's row-major plane layout)."""
    R, K = X.shape
    if K % 4 != 0 or X.stride(1) != 1 or X.stride(0) % 4 != 0 or X.data_ptr() % 16 != 0:
        X = F.pad(X.contiguous(), (0, Kp - K)) if K % 4 else X.contiguous()
        K = X.shape[1]
    hi = torch.empty((R, Kp), dtype=torch.float16, device=X.device)
    lo = torch.empty((R, Kp), dtype=torch.float16, device=X.device)
    if Kp > K:
        hi[:, K:].zero_()
        lo[:, K:].zero_()
    ex = torch.empty(R, dtype=torch.int32, device=X.device)
    flag = torch.zeros(1, dtype=torch.int32, device=X.device)
    check(lib().ha_split3_rows(_ptr(X), R, K, X.stride(0), _ptr(hi), _ptr(None), _ptr(lo), Kp, _ptr(ex), _ptr(flag),
                               ctypes.c_void_p(stream_ptr(X.device))), "ha_split3_rows")
    return hi, lo, ex, flag


# --------------------------------------------------------------------------------------------- fp64 factor kernels
def _native64(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.float64 and use_native(t)


def gemm64(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, alpha: float = 1.0,
           beta: float = 0.0, upper: bool = False) -> torch.Tensor:
    """fp64 ``out = beta * out + alpha * a @ b`` on the fp64 matrix cores (``csrc/linalg64.hip:
    gemm64``, v_mfma_f64_16x16x4_f64); any row-/column-major operand views. ``upper``: only the
    entries on or above the diagonal of ``out`` are written. Host tensors: torch."""
    M, K = a.shape
    N = b.shape[1]
    if not _native64(a) or b.dtype != torch.float64:
        res = alpha * (a @ b)
        if out is None:
            out = torch.zeros((M, N), dtype=a.dtype, device=a.device)
        full = res + beta * out if beta != 0.0 else res
        if upper:
            mask = torch.ones((M, N), dtype=torch.bool, device=a.device).triu()
            out.copy_(torch.where(mask, full, out))
        else:
            out.copy_(full)
        return out
    if out is None:
        out = torch.zeros((M, N), dtype=torch.float64, device=a.device)
    A, lda, a_km = _gemm_operand(a, 1)
    B, ldb, b_nm = _gemm_operand(b, 1)
    check(lib().ha_gemm64(_ptr(A), _ptr(B), _ptr(out), M, N, K, lda, ldb, out.stride(0) if M > 1 else N, int(a_km),
                          int(not b_nm), int(upper), 1, 0, 0, 0, float(alpha), float(beta),
                          ctypes.c_void_p(stream_ptr(a.device))), "ha_gemm64")
    return out


def gemv64(m: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """fp64 ``m @ x`` for a matrix [rows, cols] and a vector [cols] (or [cols, 1]): one block per
    row with a fixed-order reduction (``csrc/linalg64.hip: gemv64_rows``) for device fp64 input
    (a row-major view; a transposed view is copied once), torch otherwise."""
    shape1 = x.dim() == 2
    xv = x.reshape(-1)
    if not (_native64(m) and xv.dtype == torch.float64 and m.dim() == 2 and m.shape[1] == xv.numel()):
        return m @ x
    M = m if (m.stride(1) == 1 and (m.shape[0] <= 1 or m.stride(0) >= m.shape[1])) else m.contiguous()
    xc = xv.contiguous()
    y = torch.empty(M.shape[0], dtype=torch.float64, device=m.device)
    check(lib().ha_gemv64(_ptr(M), M.shape[0], M.shape[1], M.stride(0) if M.shape[0] > 1 else M.shape[1], _ptr(xc),
                          _ptr(y), ctypes.c_void_p(stream_ptr(m.device))), "ha_gemv64")
    return y.reshape(-1, 1) if shape1 else y


def cholesky_upper(g: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Upper Cholesky factor R (G = R^T R) of a symmetric positive definite fp64 matrix and a
    device int32 ``info`` (0, or 1 + the first failing column). Device tensors: the blocked
    kernels of ``csrc/linalg64.hip`` (chol_diag / chol_panel / gemm64 trailing update) - no
    rocSOLVER. Host: torch.linalg.cholesky_ex."""
    if not _native64(g):
        r, info = torch.linalg.cholesky_ex(g, upper=True)
        return r, info.to(torch.int32).reshape(1)
    n = g.shape[0]
    R = g.contiguous().clone()
    info = torch.zeros(1, dtype=torch.int32, device=g.device)
    if n:
        check(lib().ha_chol_upper64(_ptr(R), n, R.stride(0), _ptr(info), ctypes.c_void_p(stream_ptr(g.device))),
              "ha_chol_upper64")
    return R.triu_(), info


def tri_inv_upper(r: torch.Tensor) -> torch.Tensor:
    """Inverse of an upper-triangular fp64 matrix (``csrc/linalg64.hip``: 64 x 64 diagonal blocks
    inverted directly, off-diagonal blocks by recursive doubling on gemm64). Host: a triangular
    solve against the identity."""
    n = r.shape[0]
    if not _native64(r):
        return torch.linalg.solve_triangular(r, torch.eye(n, dtype=r.dtype, device=r.device), upper=True)
    R = r.contiguous()
    X = torch.empty((n, n), dtype=torch.float64, device=r.device)
    W = torch.empty((n, n), dtype=torch.float64, device=r.device)
    if n:
        check(lib().ha_trtri_upper64(_ptr(R), n, R.stride(0), _ptr(X), n, _ptr(W),
                                     ctypes.c_void_p(stream_ptr(r.device))), "ha_trtri_upper64")
    return X


# --------------------------------------------------------------------------------------------- Householder QR
def householder_qr(local: torch.Tensor, g0: int, m_total: int, calc_q: bool = True, allreduce=None):
    """Blocked Householder QR of a row block (rows [g0, g0 + m_r) of an m_total x n matrix whose
    other rows live on other ranks) - ``csrc/householder.hip``: one kernel per panel column
    (geqrf panel, fp64 dot products), compact-WY T by ``hh_larft`` and the trailing update
    C -= V (T^T (V^T C)) as two GEMMs. ``allreduce(t)`` sums a device tensor over the ranks in
    place (None: a single block holds all rows). Backward stable for any conditioning.

    Returns (this rank's rows of the reduced Q or None, R [min(m, n), n] replicated), with
    diag(R) >= 0."""
    A, panels = householder_factor(local, g0, m_total, allreduce)
    dev, dt = A.device, A.dtype
    m_r, n = A.shape
    kmax = min(m_total, n)
    red = allreduce or (lambda t: t)
    # R: the upper triangle of global rows [0, kmax), gathered from their owners by the all-reduce
    R = torch.zeros((kmax, n), dtype=dt, device=dev)
    lo, hi = max(g0, 0), min(g0 + m_r, kmax)
    if hi > lo:
        R[lo:hi] = torch.triu(A[lo - g0: hi - g0], diagonal=lo)
    red(R)
    d = torch.sign(torch.diagonal(R))
    d = torch.where(d == 0, torch.ones_like(d), d)
    R = d.unsqueeze(1) * R
    if not calc_q:
        return None, R
    Q = torch.zeros((m_r, kmax), dtype=dt, device=dev)
    if hi > lo:
        Q[lo - g0: hi - g0, lo:hi] = torch.eye(hi - lo, dtype=dt, device=dev)
    householder_apply(A, panels, Q, g0, transpose=False, allreduce=allreduce, identity_start=True)
    return Q * d.unsqueeze(0), R


# HEAT_HH_SKIP=1 (A/B): the column steps skip the panel's finished columns and V^T V is one GEMM
# after the panel. Measured 1.25e6 x 4096 QR: 1.41 s vs 1.29 s for the default (the per-panel
# V^T V launches cost more than the skipped loads save; `profiles/hh_profile_r05.txt`)
_HH_SKIP = os.environ.get("HEAT_HH_SKIP", "0") == "1"


def _hh_outer(native: bool, nb: int) -> int:
    """Width of the aggregated block reflector of the two-level Householder factorisation: the
    trailing matrix is updated once per outer block (W = V^T C on the fp64 matrix cores, then one
    K = 256 GEMM) instead of once per 32-column panel. Env ``HEAT_HH_OUTER`` overrides (a multiple
    of the panel width; = panel width: the one-level algorithm)."""
    env = os.environ.get("HEAT_HH_OUTER")
    w = int(env) if env else (8 * nb if native else 2 * nb)
    return max(nb, w // nb * nb)


def householder_factor(local: torch.Tensor, g0: int = 0, m_total: Optional[int] = None, allreduce=None):
    """The factorisation half of :func:`householder_qr`: returns (A, panels) - A holds R in its
    upper triangle and the reflectors below it (LAPACK geqrf layout, rows [g0, g0 + m_r) of the
    global matrix), ``panels`` the compact-WY blocks as [(k0, nc, T)].

    Two-level blocking (ref ``heat/core/linalg/qr.py`` factors tiles with torch.linalg.qr; this is
    the MI355X design): 32-column panels (``csrc/householder.hip``: one kernel per column with
    fp64 dot products, ``hh_larft`` T factor) update only the rest of their 256-column outer
    block; the outer block is then applied to the trailing matrix as ONE block reflector
    Q_b = I - V T V^T with T = (striu(V^T V) + diag(1/tau))^-1 (``tri_inv_upper``), W = V^T C
    from the fp64 matrix-core kernel (``csrc/linalg64.hip: vtc64``, exact products, split-K in
    fixed order) and C -= V (T^T W) as one fp32 GEMM (``csrc/gemm_mid.hip: gemm_f32m``, see
    ``_HH_UPDATE``). Each 32-column panel is factored in a compact m x 32 copy and its V^T V comes
    from the column sums of the steps (no separate pass)."""
    m_r, n = local.shape
    m_total = m_r if m_total is None else m_total
    native = local.is_cuda and use_native(local)
    L = lib() if native else None
    nb = L.ha_hh_nb() if native else 32
    outer = _hh_outer(native, nb)
    if native and os.environ.get("HEAT_HH_NB"):
        # narrower column panels inside the same outer block (A/B): each column step streams an
        # m x nb panel, so nb = 16 halves the panel traffic for twice the in-block updates
        nb = max(4, min(nb, int(os.environ["HEAT_HH_NB"]) // 4 * 4))
    slen = L.ha_hh_slen() if native else 2 * nb  # replicated accumulators (the host path: one)
    dev = local.device
    dt = local.dtype
    code = 0 if dt == torch.float32 else 1
    kmax = min(m_total, n)
    A = local.contiguous().clone()
    st = ctypes.c_void_p(stream_ptr(dev)) if native else None
    red = allreduce or (lambda t: t)
    rows = torch.arange(g0, g0 + m_r, device=dev).unsqueeze(1)
    if native:
        # per-block partial slots + self-resetting group counters of the fixed-order panel sums
        hpart = torch.empty(max(1, L.ha_hh_part_len(m_r)), dtype=torch.float64, device=dev)
        hcnt = torch.zeros(L.ha_hh_counters(), dtype=torch.int32, device=dev)
    panels = []
    for K0 in range(0, kmax, outer):
        ncol = min(outer, kmax - K0)
        taus, inner = [], []
        for k0 in range(K0, K0 + ncol, nb):
            nc = min(nb, K0 + ncol - k0)
            S = torch.zeros((nc + 1, slen), dtype=torch.float64, device=dev)
            tau = torch.empty(nc, dtype=dt, device=dev)
            Y = torch.zeros((nc, nc), dtype=torch.float64, device=dev)  # V^T V, written by the steps
            if native:
                # the panel in a compact m x nc copy: the nc + 1 passes stream contiguous rows
                # instead of one 128-byte segment per (16 KB) matrix row
                # (always a copy: when the panel spans every column of A, .contiguous() would return A
                # itself and the reflector masking below would overwrite R)
                Pb = A[:, k0: k0 + nc].clone(memory_format=torch.contiguous_format)
                check(L.ha_hh_colsums(_ptr(Pb), code, m_r, nc, g0, 0, nc, k0, _ptr(S[0]), _ptr(hpart),
                                      _ptr(hcnt), st), "ha_hh_colsums")
            else:
                _hh_colsums_host(A, rows, k0, nc, S[0])
            red(S[0])
            for j in range(nc):
                last = j + 1 == nc
                if native:
                    check(L.ha_hh_step(_ptr(Pb), code, m_r, nc, g0, k0, 0, nc, j, _ptr(S[j]),
                                       _ptr(None) if last else _ptr(S[j + 1]), _ptr(tau),
                                       _ptr(None) if _HH_SKIP else _ptr(Y), _ptr(hpart), _ptr(hcnt), st), "ha_hh_step")
                else:
                    _hh_step_host(A, rows, k0, nc, j, S[j], None if last else S[j + 1], tau, Y)
                if not last:
                    red(S[j + 1])
            taus.append(tau)
            if native:
                A[:, k0: k0 + nc] = Pb
                V = _hh_v_fix(Pb, rows, k0, g0)
            else:
                V = _hh_v(A, rows, k0, nc, g0)
            Tm = torch.empty((nc, nc), dtype=dt, device=dev)
            if native and _HH_SKIP:
                # V^T V in one pass over the finished panel (the steps skipped the done columns)
                Y = _vtc(V, V, native, st)
                red(Y)
                Y = Y.contiguous()
            if native:
                check(L.ha_hh_larft(_ptr(Y), _ptr(tau), nc, code, _ptr(Tm), st), "ha_hh_larft")
            else:
                Tm.copy_(_hh_larft_host(Y, tau))
            inner.append(Tm)
            if k0 + nc < K0 + ncol:        # the rest of this outer block
                _hh_block_update(A[:, k0 + nc: K0 + ncol], V, Tm, True, native, st, red)
        V = _hh_v(A, rows, K0, ncol, g0)
        if len(inner) == 1:
            Tb = inner[0].double()
        else:
            Y = _vtc(V, V, native, st)
            red(Y)
            tinv = torch.triu(Y, diagonal=1)
            tinv.diagonal().copy_(1.0 / torch.cat(taus).double())
            Tb = tri_inv_upper(tinv)
        panels.append((K0, ncol, Tb))
        if K0 + ncol < n:
            _hh_block_update(A[:, K0 + ncol:], V, Tb, True, native, st, red)
    return A, panels


def householder_block(t: Optional[torch.Tensor] = None) -> int:
    """Width of the compact-WY blocks :func:`householder_factor` returns for ``t``'s device (the
    outer block: its ``panels`` are [(k0, min(width, kmax - k0), T fp64)] for k0 = 0, width, ...)."""
    native = t is not None and t.is_cuda and use_native(t)
    return _hh_outer(native, lib().ha_hh_nb() if native else 32)


def householder_apply(A: torch.Tensor, panels, C: torch.Tensor, g0: int = 0, transpose: bool = True,
                      allreduce=None, identity_start: bool = False) -> torch.Tensor:
    """Apply the orthogonal factor of a :func:`householder_factor` result to C in place (rows of
    C aligned with the rows of A): Q^T C (``transpose``) or Q C, block by block as
    C -= V (T^T|T (V^T C)) with the V^T C products accumulated in fp64."""
    native = A.is_cuda and use_native(A)
    st = ctypes.c_void_p(stream_ptr(A.device)) if native else None
    red = allreduce or (lambda t: t)
    rows = torch.arange(g0, g0 + A.shape[0], device=A.device).unsqueeze(1)
    for k0, nc, Tm in (panels if transpose else list(reversed(panels))):
        V = _hh_v(A, rows, k0, nc, g0)
        # C = [I; 0] accumulation: columns before k0 are still unit vectors that V (zero above
        # global row k0) does not touch
        Cc = C[:, k0:] if identity_start else C
        _hh_block_update(Cc, V, Tm, transpose, native, st, red)
    return C


# the rank-nc update C -= V X of the Householder QR: small (default: the LDS-DMA 128-tile gemm_f32m,
# csrc/gemm_mid.hip) | blas (hipBLASLt fp32) | f32 (the 256-tile gemm_f32t) | h3 (fp16x3 MFMA). The
# update is a plain fp32 GEMM with a small K (256 outer / 32 inner) and a tall C read and written
# once. Measured at 1.25e6 rows (tools/microbench/gemm_mid.py, profiles/gemm_mid_r06.jsonl):
# K = 256, N = 3840: gemm_f32m 23.05 ms, hipBLASLt 19.75, gemm_f32t 27.6; the whole 1.25e6 x 4096
# factorisation + Q 1.32 s native (K <= 64 products on the 64 x 64 tile) vs 1.28-1.31 s with the
# library update (tools/microbench/hh_update_ab.py) - 1-3 % for a QR with no library GEMM in it. The blas form runs at float32 matmul
# precision "highest" whatever the caller set: under "high" hipBLASLt drops to a reduced-precision
# fp32 path (measured ||Q^T Q - I|| 1.5e-5 instead of 1.2e-7, tools/microbench/hh_prec.py).
_HH_UPDATE = os.environ.get("HEAT_HH_UPDATE", "small")


_PRECISION_LOCK = threading.RLock()


@contextlib.contextmanager
def exact_fp32_library():
    """Library GEMMs inside run with exact fp32 products. torch's float32 matmul precision is
    process-global, so the switch to "highest" and back is serialised under one lock (every
    framework call site that changes it goes through here), and nothing changes when it already
    is "highest"."""
    with _PRECISION_LOCK:
        prev = torch.get_float32_matmul_precision()
        if prev == "highest":
            yield
            return
        torch.set_float32_matmul_precision("highest")
        try:
            yield
        finally:
            torch.set_float32_matmul_precision(prev)


def _exact_addmm_(C: torch.Tensor, A: torch.Tensor, B: torch.Tensor, alpha: float) -> None:
    """C += alpha A B through the library GEMM with exact fp32 products."""
    with exact_fp32_library():
        C.addmm_(A, B, alpha=alpha)


def _hh_block_update(C: torch.Tensor, V: torch.Tensor, Tm: torch.Tensor, transpose: bool, native: bool, st,
                     red) -> None:
    """C -= V op(T) (V^T C) in place: W = V^T C with fp64 accumulation (summed over the ranks by
    ``red``), X = op(T) W in fp64 (``gemm64``), then the rank-nc update (fp32: ``gemm_f32m``, see
    ``_HH_UPDATE``; fp64: ``gemm64``)."""
    if C.shape[1] == 0 or V.shape[1] == 0:
        return
    W = _vtc(V, C, native, st)
    red(W)
    T64 = Tm.double()
    Tt = T64.T if transpose else T64
    if not native:
        _exact_addmm_(C, V, (Tt @ W).to(C.dtype), -1.0)
        return
    X = gemm64(Tt, W)
    if C.dtype == torch.float64:
        gemm64(V, X, out=C, alpha=-1.0, beta=1.0)
        return
    X = X.to(C.dtype)
    if _HH_UPDATE == "small" and C.stride(1) == 1 and gemm_f32_small(V, X, out=C, alpha=-1.0, accumulate=True) is not None:
        pass
    elif C.stride(1) != 1 or _HH_UPDATE == "blas":
        _exact_addmm_(C, V, X, -1.0)
    elif _HH_UPDATE == "h3" and gemm_h3(V, X, out=C, alpha=-1.0, accumulate=True) is not None:
        pass
    else:
        gemm_f32(V, X, out=C, accumulate=True, alpha=-1.0)


def vtc64(V: torch.Tensor, C: torch.Tensor, out: Optional[torch.Tensor] = None,
          accumulate: bool = False) -> torch.Tensor:
    """``V^T C`` ([nc, N] fp64) with exact products and fp64 accumulation over the (long) row
    dimension on the fp64 matrix cores (``csrc/linalg64.hip: vtc64``; split-K partials added in
    fixed order - deterministic). V [m, nc], C [m, N]: fp32 or fp64 device tensors, rows
    contiguous. Host tensors: an fp64 GEMM."""
    nc, N = V.shape[1], C.shape[1]
    if not (V.is_cuda and use_native(V)) or V.dtype not in (torch.float32, torch.float64):
        r = V.double().T @ C.double()
        if out is None:
            return r
        return out.add_(r) if accumulate else out.copy_(r)
    if C.dtype != V.dtype:
        C = C.to(V.dtype)
    if V.stride(-1) != 1 or (nc > 1 and V.stride(0) < nc):
        V = V.contiguous()
    if C.stride(-1) != 1 or (N > 1 and C.stride(0) < N):
        C = C.contiguous()
    if out is None:
        out = torch.zeros((nc, N), dtype=torch.float64, device=V.device) if accumulate else \
            torch.empty((nc, N), dtype=torch.float64, device=V.device)
    elif not out.is_contiguous() or out.shape != (nc, N) or out.dtype != torch.float64:
        raise ValueError("vtc64: out must be a contiguous float64 [nc, N] tensor")
    L = lib()
    m = V.shape[0]
    P = torch.empty(max(1, L.ha_vtc64_splits(m, nc, N) * nc * N), dtype=torch.float64, device=V.device)
    check(L.ha_vtc64(_ptr(V), V.stride(0) if m > 1 else nc, _ptr(C), C.stride(0) if m > 1 else N,
                     0 if V.dtype == torch.float32 else 1, m, nc, N, _ptr(out), _ptr(P), int(accumulate),
                     ctypes.c_void_p(stream_ptr(V.device))), "ha_vtc64")
    return out


# 1024-row slices: on the cond-1e8 test matrix ||QR - A|| is 4.5e-6 (4.2e-6 with exact fp64 V^T C)
# vs 1.3e-5 with 4096-row slices, for 2 % of the QR time (tools/microbench/hh_variants.py, r4t)
_VTC_KCHUNK = max(256, int(os.environ.get("HEAT_VTC_KCHUNK", "1024")) // 256 * 256)
_VTC_WIDE = os.environ.get("HEAT_HH_VTC", "f32s")   # f32s (sliced fp32 MFMA) | f64 (vtc64)


def vtc_f32s(V: torch.Tensor, C: torch.Tensor) -> Optional[torch.Tensor]:
    """``V^T C`` ([nc, N] fp64) of fp32 device blocks on the f32-input matrix cores: the exact-fp32
    256-tile GEMM (``csrc/gemm_tiled.hip: gemm_f32t``) split over K slices of ``HEAT_VTC_KCHUNK``
    = 1024 rows (fp32 accumulation inside a slice, a 256 x 256 tile per workgroup), the slices
    summed in fp64 in fixed order (``ha_sum_slices64``) - the Gram's accumulation scheme
    (:func:`gram64`). Error ~ u sqrt(chunk) / sqrt(m / chunk) |v||c| < 1 u |v||c| at m = 1.25e6,
    below the fp32 rounding of the Householder update that consumes W; ~2.5x the fp64-MFMA rate
    of :func:`vtc64`. Returns None when the operands do not fit the tiled kernel (alignment)."""
    m, nc = V.shape
    N = C.shape[1]
    W = torch.zeros((nc, N), dtype=torch.float64, device=V.device)
    if m == 0 or nc == 0 or N == 0:
        return W
    L = lib()
    st = ctypes.c_void_p(stream_ptr(V.device))
    kc = _VTC_KCHUNK
    group = max(1, min(-(-m // kc), _GRAM_PARTIAL_BYTES // (4 * nc * N)))
    P = torch.empty(group * nc * N, dtype=torch.float32, device=V.device)
    for k0 in range(0, m, group * kc):
        k1 = min(m, k0 + group * kc)
        slices = -(-(k1 - k0) // kc)
        Vs, Cs = V[k0:k1], C[k0:k1]
        # A = V^T: k-major (rows of V contiguous along nc); B = C: k-major (rows contiguous along N)
        rc = L.ha_gemm_f32t(_ptr(Vs), _ptr(Cs), _ptr(P), nc, N, k1 - k0, Vs.stride(0), Cs.stride(0), N, 1, 1,
                            1.0, 0, 0, slices, nc * N, st)
        if rc == _HA_UNSUPPORTED:
            return None
        check(rc, "ha_gemm_f32t")
        used = L.ha_gemm_tiled_slices(k1 - k0, slices)
        check(L.ha_sum_slices64(_ptr(P), used, nc, N, nc * N, _ptr(W), N, 0, 1, st), "ha_sum_slices64")
    return W


def _vtc(V: torch.Tensor, C: torch.Tensor, native: bool, st) -> torch.Tensor:
    """V^T C with fp64 accumulation across the rows: fp32 block reflectors wider than a panel on
    the sliced fp32 matrix-core GEMM (:func:`vtc_f32s`), fp32 panels up to 32 columns on the
    narrow fp64-MFMA kernel ``vtc32`` (:func:`vtc64`; ``HEAT_HH_VTC=f64`` sends the wide ones
    there too); fp64 panels on the VALU kernel ``hh_vtc``; host: an fp64 GEMM."""
    if not native:
        return V.double().T @ C.double()
    nc, N = V.shape[1], C.shape[1]
    if C.stride(1) != 1:
        C = C.contiguous()
    L = lib()
    if V.dtype == torch.float32 and nc > L.ha_hh_nb() and _VTC_WIDE == "f32s":
        if V.stride(1) != 1 or V.stride(0) < nc:
            V = V.contiguous()
        W = vtc_f32s(V, C)
        if W is not None:
            return W
    if nc > L.ha_hh_nb() or V.dtype == torch.float32:  # fp32 panels: the narrow MFMA kernel vtc32
        return vtc64(V, C)
    W = torch.zeros((nc, N), dtype=torch.float64, device=V.device)
    P = torch.empty(max(1, L.ha_hh_vtc_splits(V.shape[0], N) * nc * N), dtype=torch.float64, device=V.device)
    check(L.ha_hh_vtc(_ptr(V), V.stride(0), _ptr(C), C.stride(0), 0 if V.dtype == torch.float32 else 1,
                      V.shape[0], N, nc, _ptr(W), _ptr(P), st), "ha_hh_vtc")
    return W


def _hh_v(A: torch.Tensor, rows: torch.Tensor, k0: int, nc: int, g0: int) -> torch.Tensor:
    """Explicit reflectors of a factorised panel: V[g, c] = A[g, k0 + c] below the diagonal row
    k0 + c, 1 on it, 0 above (a contiguous copy of the columns; only the local rows above global
    row k0 + nc need the mask)."""
    return _hh_v_fix(A[:, k0: k0 + nc].clone(memory_format=torch.contiguous_format), rows, k0, g0)


def _hh_v_fix(P: torch.Tensor, rows: torch.Tensor, k0: int, g0: int) -> torch.Tensor:
    """In place: the rows of a contiguous panel copy P (global rows g0 ...) above global row
    k0 + P.shape[1] become the unit-lower reflector rows (1 on the diagonal, 0 above)."""
    nc = P.shape[1]
    top = min(max(k0 + nc - g0, 0), P.shape[0])
    if top:
        dcol = torch.arange(k0, k0 + nc, device=P.device).unsqueeze(0)
        r = rows[:top]
        P[:top] = torch.where(r > dcol, P[:top], (r == dcol).to(P.dtype))
    return P


# host (CPU) reference of the panel kernels: same math, same buffer conventions (the oracle of the
# tests and the CPU / gloo multi-rank path)
def _hh_colsums_host(A, rows, k0, nc, S):
    below = (rows[:, 0] >= k0)
    P = A[below, k0: k0 + nc].double()
    S[:nc] += P[:, 0] @ P
    own = rows[:, 0] == k0
    if bool(own.any()):
        S[32: 32 + nc] += A[own, k0: k0 + nc].double().reshape(-1)


def _hh_step_host(A, rows, k0, nc, j, Sin, Sout, tau, Y=None):
    d = k0 + j
    alpha = float(Sin[32 + j])
    nrm2 = float(Sin[j])
    sig = nrm2 - alpha * alpha
    beta, tv, scale = alpha, 0.0, 0.0
    if sig > 0.0 and nrm2 > 0.0:
        nx = nrm2 ** 0.5
        beta = -nx if alpha >= 0 else nx
        tv = (beta - alpha) / beta
        scale = 1.0 / (alpha - beta)
    tau[j] = tv
    rd = Sin[32: 32 + nc]
    w = rd + scale * (Sin[:nc] - alpha * rd)
    if Y is not None:  # column j of V^T V from the same sums (see csrc/householder.hip: hh_step)
        Y[:j, j] = w[:j]
        Y[j, j] = 1.0 + scale * scale * sig
    w[: j + 1] = 0.0
    g = rows[:, 0]
    own = g == d
    if bool(own.any()):
        r = A[own, k0: k0 + nc].double()
        r[:, j + 1:] -= tv * w[j + 1:]
        r[:, j] = beta
        A[own, k0: k0 + nc] = r.to(A.dtype)
    below = g > d
    P = A[below, k0: k0 + nc].double()
    v = P[:, j] * scale
    P -= tv * v.unsqueeze(1) * w.unsqueeze(0)
    P[:, j] = v
    A[below, k0: k0 + nc] = P.to(A.dtype)
    if Sout is not None:
        P = A[below, k0: k0 + nc].double()
        Sout[:nc] += P[:, j + 1] @ P
        nxt = g == d + 1
        if bool(nxt.any()):
            Sout[32: 32 + nc] += A[nxt, k0: k0 + nc].double().reshape(-1)


def _hh_larft_host(Y, tau):
    nc = tau.shape[0]
    T = torch.zeros((nc, nc), dtype=torch.float64, device=Y.device)
    for j in range(nc):
        tj = float(tau[j])
        if j:
            T[:j, j] = -tj * (T[:j, :j] @ Y[:j, j])
        T[j, j] = tj
    return T.to(tau.dtype)


_RADIX_DTYPES = {torch.float32: 0, torch.int32: 1}


_RADIX_MIN_ROWS = int(os.environ.get("HEAT_RADIX_MIN_ROWS", "8"))


def radix_sort_supported(t: torch.Tensor, dim: int = -1) -> bool:
    """Device float32 / int32 tensors below 2^31 elements go to the native radix sort when they
    hold at least ``_RADIX_MIN_ROWS`` rows along ``dim``: measured (profiles/radix_sort_bench.jsonl)
    3.9x faster than torch.sort on 64 x 1e6, 1.1-1.6x slower on a single 1e7-1e8 row, where
    rocPRIM's one-sweep sort (torch.sort) keeps the job."""
    if not (t.is_cuda and t.dtype in _RADIX_DTYPES and 0 < t.numel() < (1 << 31) - 1):
        return False
    rows = t.numel() // max(t.shape[dim], 1) if t.dim() else 1
    return rows >= _RADIX_MIN_ROWS and use_native(t)


def sort_rows(x: torch.Tensor, descending: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """Stable sort along the last axis (``csrc/radix.hip``: LSD radix, 8-bit digits, row number
    as the most significant digits of a batch) - ``torch.sort(x, dim=-1, stable=True)``
    semantics: ties keep their order, NaN sorts last (first when descending), -0.0 ties +0.0.
    Returns (values, int64 positions)."""
    shp = x.shape
    rowlen = shp[-1] if x.dim() else 1
    xc = x.contiguous()
    rows = xc.numel() // max(rowlen, 1)
    vals = torch.empty_like(xc)
    idx = torch.empty(shp, dtype=torch.int64, device=x.device)
    if xc.numel() == 0:
        return vals, idx
    L = lib()
    ws = torch.empty(L.ha_radix_workspace_bytes(xc.numel()), dtype=torch.uint8, device=x.device)
    check(L.ha_radix_sort_rows(_ptr(xc), _RADIX_DTYPES[x.dtype], rows, rowlen, int(descending), _ptr(vals), _ptr(idx),
                               _ptr(ws), ctypes.c_void_p(stream_ptr(x.device))), "ha_radix_sort_rows")
    return vals, idx


# --------------------------------------------------------------------------------------------
# block pack / unpack for personalised exchanges (csrc/pack.hip)
# --------------------------------------------------------------------------------------------
def _rows_view(shape, axis):
    O = int(np.prod(shape[:axis])) if axis else 1
    S = int(shape[axis])
    R = int(np.prod(shape[axis + 1:])) if axis + 1 < len(shape) else 1
    return O, S, R


def _block_offsets(counts):
    off = [0]
    for c in counts:
        off.append(off[-1] + int(c))
    return off


def pack_supported(t: torch.Tensor) -> bool:
    """Device tensors of at most 256 blocks go through the native pack kernel."""
    return t.is_cuda and use_native(t) and hasattr(lib(), "ha_rows_permute")


def pack_blocks(t: torch.Tensor, axis: int, counts) -> torch.Tensor:
    """The blocks ``t.narrow(axis, off_q, counts[q])`` one after the other, each in C order, as ONE
    flat tensor (the send buffer of an all-to-all) - a single pass over ``t``."""
    counts = [int(c) for c in counts]
    if not pack_supported(t) or len(counts) > 256:
        parts = [t.narrow(axis, o, c).reshape(-1) for o, c in zip(_block_offsets(counts)[:-1], counts)]
        return torch.cat(parts) if parts else t.new_empty(0)
    src = t.contiguous()
    O, S, R = _rows_view(src.shape, axis)
    assert sum(counts) == S, (counts, S)
    if O == 1:
        return src.reshape(-1)  # blocks along the outermost axis are already back to back
    out = torch.empty(src.numel(), dtype=src.dtype, device=src.device)
    off = np.asarray(_block_offsets(counts), dtype=np.int64)
    check(lib().ha_rows_permute(_ptr(src), _ptr(out), O, S, R * src.element_size(),
                                off.ctypes.data_as(ctypes.c_void_p), len(counts), 0,
                                ctypes.c_void_p(stream_ptr(src.device))), "ha_rows_permute")
    return out


def unpack_blocks(flat: torch.Tensor, shape, axis: int, counts, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Inverse of :func:`pack_blocks`: the tensor of ``shape`` whose blocks along ``axis``
    (``counts[q]`` rows each) arrive one after the other in ``flat`` - a single pass."""
    counts = [int(c) for c in counts]
    shape = tuple(int(s) for s in shape)
    if out is None:
        out = torch.empty(shape, dtype=flat.dtype, device=flat.device)
    if not pack_supported(flat) or len(counts) > 256 or not out.is_contiguous():
        parts, pos = [], 0
        for c in counts:
            sh = list(shape)
            sh[axis] = c
            n = int(np.prod(sh))
            parts.append(flat[pos: pos + n].reshape(sh))
            pos += n
        out.copy_(torch.cat(parts, dim=axis))
        return out
    O, S, R = _rows_view(shape, axis)
    assert sum(counts) == S and flat.numel() == O * S * R, (counts, shape, flat.numel())
    if O == 1:
        out.view(-1).copy_(flat) if out.data_ptr() != flat.data_ptr() else None
        return out
    off = np.asarray(_block_offsets(counts), dtype=np.int64)
    src = flat.contiguous()
    check(lib().ha_rows_permute(_ptr(src), _ptr(out), O, S, R * src.element_size(),
                                off.ctypes.data_as(ctypes.c_void_p), len(counts), 1,
                                ctypes.c_void_p(stream_ptr(src.device))), "ha_rows_permute")
    return out


_FIN_WS = {}


def _finalize_ws(device: torch.device) -> torch.Tensor:
    """Zeroed once per (device, stream): per-block partials + the self-resetting arrival counter of
    ``km_finalize`` (two streams must not share one)."""
    key = (device, stream_ptr(device))
    ws = _FIN_WS.get(key)
    if ws is None:
        ws = torch.zeros(int(lib().ha_km_finalize_workspace()), dtype=torch.uint8, device=device)
        _FIN_WS[key] = ws
    return ws


def kmeans_finalize(packed: Optional[torch.Tensor], C: torch.Tensor, sums: Optional[torch.Tensor] = None,
                    counts: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Lloyd epilogue (``csrc/kmeans_finalize.hip``): from ``packed = [sums (k*f) | counts (k)]``
    (fp64; or fp32 ``sums`` [k, f] and ``counts`` [k] with ``packed=None``) and the current
    centroids C (float32, k x f) return (new centroids, squared shift as a 0-d fp64 tensor); empty
    clusters keep their centroid. One launch on the GPU."""
    k, f = C.shape
    dev_in = packed if packed is not None else sums
    if dev_in.is_cuda and C.dtype == torch.float32 and k * f < 2 ** 31 and use_native(C) and \
            hasattr(lib(), "ha_km_finalize_f32"):
        Cc = C if C.stride(-1) == 1 else C.contiguous()
        newC = torch.empty((k, f), dtype=torch.float32, device=C.device)
        shift = torch.empty((), dtype=torch.float64, device=C.device)
        ws = _finalize_ws(C.device)
        s = ctypes.c_void_p(stream_ptr(C.device))
        if packed is not None:
            pk = packed.contiguous()
            check(lib().ha_km_finalize(_ptr(pk), k, f, _ptr(Cc), Cc.stride(0), _ptr(newC), _ptr(shift), _ptr(ws), s),
                  "ha_km_finalize")
        else:
            sc, cc = sums.float().contiguous(), counts.float().contiguous()
            check(lib().ha_km_finalize_f32(_ptr(sc), _ptr(cc), k, f, _ptr(Cc), Cc.stride(0), _ptr(newC), _ptr(shift),
                                           _ptr(ws), s), "ha_km_finalize_f32")
        return newC, shift
    if packed is None:
        packed = torch.cat([sums.reshape(-1).double(), counts.double()])
    kf = k * f
    gs = packed[:kf].reshape(k, f)
    gc = packed[kf:]
    newC = torch.where(gc.unsqueeze(1) > 0, gs / gc.clamp(min=1).unsqueeze(1), C.double()).to(C.dtype)
    return newC, ((C.double() - newC.double()) ** 2).sum()
