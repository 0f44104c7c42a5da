"""
Linear-algebra basics (reference ``heat/core/linalg/basics.py``: ``dot`` 42, ``matmul`` 108-773,
``matrix_norm`` 779, ``norm`` 907, ``outer`` 1056, ``projection`` 1289, ``trace`` 1313,
``transpose`` 1735, ``tril/triu`` 1875/1898, ``vecdot`` 1920, ``vector_norm`` 1957).

Distributed matmul keeps the reference's output-split rules but replaces its block-broadcast
pipeline and full-size all-reduces:

* ``0 x None``, ``None x 1``: local GEMM, no communication;
* ``0 x 0``, ``0 x 1``, ``1 x 1``: ONE all-gather of the replicated operand's panels (all 7 xGMI
  links in parallel), then ONE local GEMM - fp32 on the hand-written 256 x 256-tile MFMA kernels
  (``ops/csrc/gemm_tiled.hip``: exact f32 MFMA, or the fused fp16x3 kernel when the float32
  matmul precision is "high"), other dtypes on torch;
* ``1 x None``, ``None x 0``, ``1 x 0`` (contraction axis split): local partial GEMM + ONE
  reduce-scatter straight into the split output (half the traffic of an all-reduce and no
  replicated M x N result).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple, Union

import numpy as np
import functools
import os

import torch

from ...parallel import staging as _SD
from ...parallel.ring import ring_pass
import torch.distributed as dist

from .. import _operations, factories, types
from ..communication import MPI
from ..dndarray import DNDarray, _chunk_counts
from ..stride_tricks import sanitize_axis

__all__ = ["dot", "matmul", "matrix_norm", "norm", "outer", "projection", "trace", "transpose", "tril",
           "triu", "vecdot", "vector_norm"]


def transpose(a: DNDarray, axes: Optional[List[int]] = None) -> DNDarray:
    """Permute the dimensions (the split axis follows its data; no communication)."""
    if not isinstance(a, DNDarray):
        raise TypeError("Input must be a DNDarray, is {}".format(type(a)))
    nd = a.ndim
    if axes is None:
        axes = list(reversed(range(nd)))
    else:
        if isinstance(axes, str) or not hasattr(axes, "__iter__"):
            raise TypeError("axes must be an iterable containing ints, got {}".format(type(axes)))
        axes = list(axes)
        if len(axes) != nd:
            raise ValueError("axes do not match tensor shape")
        for i, ax in enumerate(axes):
            if not isinstance(ax, (int, np.integer)):
                raise TypeError("axis must be an integer, but was {}".format(type(ax)))
            if ax < 0:
                axes[i] = ax + nd
    if sorted(axes) != list(range(nd)):
        raise ValueError("axes do not match tensor shape")
    split = axes.index(a.split) if a.split is not None else None
    data = a.larray.permute(*axes)
    gshape = tuple(a.gshape[ax] for ax in axes)
    return DNDarray(data, gshape, a.dtype, split, a.device, a.comm, a.balanced)


DNDarray.transpose = lambda self, axes=None: transpose(self, axes)


def _reduce_scatter(partial: torch.Tensor, comm, axis: int) -> torch.Tensor:
    """Sum ``partial`` (identical global shape on every rank) and keep this rank's chunk along
    ``axis`` (RCCL reduce-scatter, padded to equal chunks)."""
    if comm.size == 1:
        return partial
    n = partial.shape[axis]
    counts = _chunk_counts(n, comm.size)
    mx = max(counts)
    moved = partial.movedim(axis, 0)
    rest = tuple(moved.shape[1:])
    if all(c == mx for c in counts):
        inp = moved.contiguous()
    else:
        inp = moved.new_zeros((mx * comm.size,) + rest)
        off = 0
        for r, c in enumerate(counts):
            inp[r * mx: r * mx + c] = moved[off: off + c]
            off += c
    out = moved.new_empty((mx,) + rest)
    wire_in, wire_out = inp, out
    if inp.dtype == torch.bool:
        wire_in, wire_out = inp.to(torch.uint8), out.to(torch.uint8)
    comm.reduce_scatter_tensor(wire_out, wire_in)  # native stream-ordered RCCL under HEAT_COMM_NATIVE=1
    res = wire_out[: counts[comm.rank]]
    return res.movedim(0, axis).contiguous()


# Largest operand handed to one BLAS call on the device. rocBLAS/hipBLASLt kernels address their
# operands through 32-bit buffer descriptors, so a single GEMM on a >4 GB operand (a 1.25e6 x 4096
# fp32 shard is 20 GB on a 288 GB MI355X) faults; larger library products are split into blocks.
# The hand-written kernels (fp32 on every path below) use 64-bit offsets and take any size.
_BLAS_MAX_BYTES = int(os.environ.get("HEAT_BLAS_MAX_BYTES", str(1 << 31)))
_CHUNK_ON_HOST = False  # tests: exercise the blocking on CPU tensors too

# "native" (default): fp32 device GEMMs on the hand-written MFMA kernels (ops/csrc/gemm_tiled.hip);
# "blas": torch.matmul / the tripled-K library split (A/B comparisons)
_GEMM_BACKEND = os.environ.get("HEAT_GEMM_BACKEND", "native")


# Gram products (X^T X, X X^T) from this size on: the upper-triangle tiles only (ops.gram_product)
_GRAM_MIN_N = int(os.environ.get("HEAT_GRAM_MIN_N", "512"))


def _split_gemm_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """fp32 device GEMMs run as the fused fp16x3 split GEMM (fp32-GEMM accuracy on the FP16 matrix
    cores, ~2.3x faster) when torch's float32 matmul precision is "high" or "medium"
    (``torch.set_float32_matmul_precision``; both allow TF32/bf16-class products, the split is more
    accurate than either). The default "highest" keeps exact fp32 products (f32 MFMA)."""
    return (a.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32
            and torch.get_float32_matmul_precision() != "highest")


def _native_fp32(a: torch.Tensor, b: torch.Tensor) -> bool:
    if _GEMM_BACKEND != "native" or not (a.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32):
        return False
    from ... import ops

    return ops.use_native(a)


_GEMM_PLAN = os.environ.get("HEAT_GEMM_PLAN", "1") != "0"   # 0: the library for the small products


@functools.lru_cache(maxsize=1024)
def _native_plan(M: int, N: int, K: int):
    """(kernel, K slices) for an exact fp32 product that fills the GPU poorly with 256 x 256 tiles.
    Cost model (units of K per output element): time ~ M N (K + s o_k) / (eff_k rate_k) + the
    split-K slice sum, (s + 1) M N 4 bytes at ~4 TB/s, plus one extra launch (~5 us) when s > 1.
    gemm_f32t ("f32t"): 256-tiles, one workgroup per CU, o = 256 k (prologue + C epilogue per
    tile), rate 1; gemm_f32m ("f32s": the 128-tile LDS-DMA kernel behind ops.gemm_f32_small),
    two workgroups per CU, o = 64, rate 0.92; its 64 x 64-tile form ("f32m64"), rate 0.90 - no
    split-K needed where 128-tiles are too few; a workgroup alone on its CU runs at 2 x 0.87 of
    the shared rate, so a last wave of at most one per CU costs 0.575 of a wave. eff = W / (the
    waves' time) for W waves of tiles x slices. Measured (profiles/gemm_mid_r06.jsonl, r6m rows)
    and picked: 1024^3 f32m64 x1 (0.023 ms, 0.88x hipBLASLt), 2048^3 f32m64 x1 (0.141, 1.10x; the
    128-tile form ties; now f32g2, below), 3072^3 f32m64 x1 (0.470, 1.04x), 4096^3 f32t x1 (0.977, 1.04x), 6144^3
    f32s x1 (3.58, 1.17x). Where every 128-tile workgroup has its CU alone (tiles <= CUs, one K slice,
    K a multiple of 32, up to 4096) the form with one barrier per PAIR of 16-k stages ("f32g2", rate fitted to
    2048^3: 0.135 ms = 1.03x hipBLASLt vs 0.144 for f32m64, gemm_mid_r06.jsonl r6v2 rows; 2-3 % slower
    than the per-stage form once two workgroups share a CU, so only there)."""
    from ... import ops

    ncu = ops.num_cus(torch.device("cuda", torch.cuda.current_device())) if torch.cuda.is_available() else 256
    t256 = -(-M // 256) * -(-N // 256)
    t128 = -(-M // 128) * -(-N // 128)
    t64 = -(-M // 64) * -(-N // 64)
    unit = 2.0 * M * N / 140e12           # seconds per unit of K at ~140 TF
    best = None
    for s in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64):
        ks = -(-K // s)
        if s > 1 and (ks < 64 or s * M * N * 4 > (1 << 30)):
            continue
        extra = 0.0 if s == 1 else (s + 1) * M * N * 4 / 4e12 / unit + 5e-6 / unit
        for kern, tiles, slots, o, rate in (("f32t", t256, ncu, 256, 1.0), ("f32s", t128, 2 * ncu, 64, 0.92),
                                            ("f32m64", t64, 2 * ncu, 64, 0.90), ("f32g2", t128, 2 * ncu, 64, 1.09)):
            if kern == "f32g2" and (s > 1 or t128 > ncu or K % 32 or K > 4096):
                continue      # the paired-barrier form: measured where a workgroup has its CU alone
            w = tiles * s / slots
            full, frac = int(w), w - int(w)
            if kern != "f32t" and 0 < frac <= 0.5:
                # a last wave of at most one workgroup per CU runs unshared: 1 / (2 x 0.87) of a wave
                waves = full + 0.575
            else:
                waves = full + (1 if frac > 0 else 0)
            eff = w / waves
            cost = (K + s * o) / (eff * rate) + extra
            if best is None or cost < best[0]:
                best = (cost, kern, s)
    return best[1], best[2]


@functools.lru_cache(maxsize=1024)
def _library_better(M: int, N: int, K: int, exact: bool) -> bool:
    """Plain fp32 GEMMs whose 256 x 256 output tiles fill the 256 CUs poorly go to the library
    (hipBLASLt, exact fp32 products). Measured (``tools/microbench/gemm_small.py``, profiles/README):
    hipBLASLt 0.029 / 0.133 / 0.46 / 3.06 ms vs gemm_f32t 0.27 / 0.30 / 0.74 / 4.44 ms at 1024^3 /
    2048^3 / 3072^3 / 6144^3 (tail waves), and vs the fp16x3 kernel 0.20 / 0.26 ms at 1024^3 /
    2048^3; the hand-written kernels win or tie from ~4 full waves of tiles (8192^3: 7.7 vs 7.2 ms
    exact, 3.3 ms fp16x3; 1.25e6 x 4096^2: 296 vs 283 ms exact without the library's 4 GB
    blocking) and on tiny-output, huge-K products through split-K (512^2 x 1e6: 3.8 vs 5.5 ms)."""
    from ... import ops

    ncu = ops.num_cus(torch.device("cuda", torch.cuda.current_device())) if torch.cuda.is_available() else 256
    tiles = -(-M // 256) * -(-N // 256)
    if tiles <= ncu // 16 and K >= (1 << 18):
        return False            # split-K on the hand-written kernel
    return tiles < (4 * ncu if exact else ncu)


def fgemm(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None, alpha: float = 1.0,
          accumulate: bool = False, b_upper: bool = False) -> torch.Tensor:
    """``alpha * a @ b`` (``+ out`` when ``accumulate``) for 2-D operands: device fp32 on the
    hand-written MFMA kernels - the fused fp16x3 kernel when the float32 matmul precision allows it,
    else the exact f32-MFMA kernel (both 256 x 256 tiles, any operand layout, 64-bit offsets, so no
    blocking) - except products with too few output tiles to fill the GPU, which run on the library
    with exact fp32 products (:func:`_library_better`); other dtypes / host tensors on torch
    (blocked below the library's operand limit). ``b_upper``: b is square upper triangular (the
    caller's guarantee, e.g. CholeskyQR's R^-1): the 256-tile kernels skip its zero half of K."""
    if _native_fp32(a, b) and a.shape[0] == b.shape[1] >= _GRAM_MIN_N and a.shape[1] >= a.shape[0]:
        from ... import ops

        g = ops.gram_product(a, b)   # X^T X / X X^T: upper tiles once + mirror (exactly symmetric)
        if g is not None:
            if alpha != 1.0:
                g.mul_(alpha)
            if out is None:
                return g
            return out.add_(g) if accumulate else out.copy_(g)
    if _native_fp32(a, b) and _library_better(a.shape[0], b.shape[1], a.shape[1], not _split_gemm_ok(a, b)):
        from ...ops import kernels as _kern

        # products whose 256 x 256 tiles do not fill the GPU: the hand-written kernel and K-slice
        # count of the measured cost model (_native_plan); the library only if neither applies
        kern, sl = _native_plan(a.shape[0], b.shape[1], a.shape[1])
        if _GEMM_PLAN and kern in ("f32s", "f32m64", "f32g2"):
            r = _kern.gemm_f32_small(a, b, out=out, alpha=alpha, accumulate=accumulate, slices=sl,
                                     kernel={"f32m64": "mid64", "f32g2": "mid128g2"}.get(kern))
            if r is not None:
                return r
        elif _GEMM_PLAN:
            return _kern.gemm_f32(a, b, out=out, accumulate=accumulate, alpha=alpha, slices=sl)

        with _kern.exact_fp32_library():   # exact fp32 products under any setting
            r = _mm_blocked(a, b)
        if alpha != 1.0:
            r = r * alpha
        if out is None:
            return r
        return out.add_(r) if accumulate else out.copy_(r)
    if _native_fp32(a, b):
        from ... import ops

        if _split_gemm_ok(a, b):
            r = ops.gemm_h3(a, b, out=out, alpha=alpha, accumulate=accumulate, b_upper=b_upper)
            if r is not None:
                return r
        return ops.gemm_f32(a, b, out=out, accumulate=accumulate, alpha=alpha, b_upper=b_upper)
    r = _mm_blocked(a, b)
    if alpha != 1.0:
        r = r * alpha
    if out is None:
        return r
    return out.add_(r) if accumulate else out.copy_(r)


def _leaf_mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    if a.dim() == 2 and b.dim() == 2 and _split_gemm_ok(a, b) and _GEMM_BACKEND != "native":
        from ... import ops

        return ops.gemm_f16x3(a, b)
    return torch.matmul(a, b)


def _mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b``: device fp32 matrices on the hand-written kernels (:func:`fgemm`), everything else
    through :func:`_mm_blocked`."""
    if a.dim() == 2 and b.dim() == 2 and _native_fp32(a, b):
        return fgemm(a, b)
    return _mm_blocked(a, b)


def _mm_blocked(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b`` with every library operand below ``_BLAS_MAX_BYTES`` (blocks along the largest of
    m, k, n; contraction blocks accumulate)."""
    if a.dim() != 2 or b.dim() != 2 or not (a.is_cuda or _CHUNK_ON_HOST):
        return _leaf_mm(a, b)
    m, k = a.shape
    n = b.shape[1]
    es = a.element_size()
    lim = _BLAS_MAX_BYTES
    if max(m * k, k * n, m * n) * es <= lim:
        return _leaf_mm(a, b)
    if k >= m and k >= n and k > 1:
        step = max(1, lim // (max(m, n, 1) * es))
        out = _mm_blocked(a[:, :step], b[:step])
        for k0 in range(step, k, step):
            out += _mm_blocked(a[:, k0: k0 + step], b[k0: k0 + step])
        return out
    out = torch.empty((m, n), dtype=torch.result_type(a, b), device=a.device)
    if m >= n:
        step = max(1, lim // (max(k, n) * es))
        for r0 in range(0, m, step):
            out[r0: r0 + step] = _mm_blocked(a[r0: r0 + step], b)
    else:
        step = max(1, lim // (max(k, m) * es))
        for c0 in range(0, n, step):
            out[:, c0: c0 + step] = _mm_blocked(a, b[:, c0: c0 + step])
    return out


# Distributed operand size (bytes, whole array) from which matmul streams its panels around the
# ring (memory O(local + 2 panels), every transfer overlapped with the previous panel's GEMM)
# instead of all-gathering the whole operand in one collective (lower latency for small operands).
_RING_MIN_BYTES = int(os.environ.get("HEAT_MATMUL_RING_BYTES", str(256 << 20)))


def _stream_panels(x: DNDarray, comm) -> bool:
    return comm.size > 1 and x.gnumel * x.larray.element_size() >= _RING_MIN_BYTES


def _batched_matmul(a: DNDarray, b: DNDarray) -> DNDarray:
    """Stacks of matrices (an extension: the reference's matmul is 2-D only). The batch
    dimensions must match; a split along a batch dimension stays local (one batched GEMM per
    rank), a split matrix dimension is replicated first."""
    from ..manipulations import resplit

    if a.ndim != b.ndim or a.gshape[:-2] != b.gshape[:-2]:
        raise ValueError("batched matmul needs equal batch dimensions, got {} and {}".format(a.gshape, b.gshape))
    if a.gshape[-1] != b.gshape[-2]:
        raise ValueError("If the last dimension of a ({}) is not the same size as the second-to-last dimension "
                         "of b. ({})".format(a.gshape[-1], b.gshape[-2]))
    nb = a.ndim - 2
    split = a.split if a.split is not None and a.split < nb else (b.split if b.split is not None and b.split < nb
                                                                   else None)
    a = a if a.split == split else resplit(a, split)
    b = b if b.split == split else resplit(b, split)
    c_type = types.promote_types(a.dtype, b.dtype)
    tt = c_type.torch_type()
    res = torch.matmul(a.larray.to(tt), b.larray.to(tt))
    gshape = a.gshape[:-1] + (b.gshape[-1],)
    return DNDarray(res, gshape, c_type, split, a.device, a.comm, a.balanced if split is not None else True)


def matmul(a: DNDarray, b: DNDarray, allow_resplit: bool = False) -> DNDarray:
    """Matrix product ``a @ b`` of 1-D/2-D DNDarrays with the reference's split rules.

    Reference ``linalg/basics.py:483-750`` pipelines block broadcasts with one-step lookahead;
    here the operand that must travel is passed around the ring in its natural row/column panels
    (``parallel.ring.ring_pass``: the next panel is in flight while the current one's GEMM runs),
    or, below ``_RING_MIN_BYTES``, all-gathered once. A contraction-split product is local GEMMs
    plus one reduce-scatter."""
    if not isinstance(a, DNDarray) or not isinstance(b, DNDarray):
        raise TypeError("matmul requires two DNDarrays")
    if a.ndim > 2 or b.ndim > 2:
        return _batched_matmul(a, b)
    if a.gshape[-1] != b.gshape[0]:
        raise ValueError("If the last dimension of a ({}) is not the same size as the second-to-last dimension "
                         "of b. ({})".format(a.gshape[-1], b.gshape[-2] if b.ndim > 1 else b.gshape[0]))
    c_type = types.promote_types(a.dtype, b.dtype)
    og_type = c_type
    if a.device.device_type == "gpu":
        # BLAS on the GPU has no integer GEMM: compute in floating point, cast back (reference 180-195)
        if c_type in (types.bool, types.uint8, types.int8, types.int16, types.int32):
            c_type = types.float32
        elif c_type == types.int64:
            c_type = types.float64
    elif c_type is types.bool:
        c_type = types.uint8
    tt = c_type.torch_type()
    comm = a.comm
    dev = a.device

    def finish(t: torch.Tensor, gshape, split, balanced=True):
        t = t.to(og_type.torch_type()) if og_type is not c_type else t
        return DNDarray(t, tuple(gshape), og_type, split, dev, comm, balanced)

    A, B = a.larray.to(tt), b.larray.to(tt)
    # a world of one follows the same split rules (the result keeps the split the reference gives)
    solo = comm.size == 1
    sa = a.split if (a.is_distributed() or solo) else None
    sb = b.split if (b.is_distributed() or solo) else None

    # vector cases ------------------------------------------------------------------------
    if a.ndim == 1 and b.ndim == 1:
        if sa is None and sb is None:
            return finish(A @ B, (), None)
        if sa is not None and sb is not None and a.split_counts() == b.split_counts():
            part = (A @ B).reshape(1)
        else:
            fa = a._gathered().to(tt) if sa is not None else A
            fb = b._gathered().to(tt) if sb is not None else B
            return finish(fa @ fb, (), None)
        comm.Allreduce(MPI.IN_PLACE, part, MPI.SUM)
        return finish(part.reshape(()), (), None)
    vec_a = a.ndim == 1
    vec_b = b.ndim == 1
    if vec_a:
        A = A.unsqueeze(0)
        sa = None if sa is None else 1
    if vec_b:
        B = B.unsqueeze(1)
        sb = None if sb is None else 0
    L = 1 if vec_a else a.gshape[0]
    Q = b.gshape[1] if not vec_b else 1
    out_shape = (L, Q)

    def squeeze_out(t, split, gshape=out_shape, balanced=True):
        if vec_a and vec_b:
            return finish(t.reshape(()), (), None)
        if vec_a:
            gs = (Q,)
            return finish(t.reshape(-1), gs, None if split is None else 0, balanced)
        if vec_b:
            gs = (L,)
            return finish(t.reshape(-1), gs, None if split is None else 0, balanced)
        return finish(t, gshape, split, balanced)

    if sa is None and sb is None:
        if allow_resplit and not vec_a and not vec_b and comm.is_distributed():
            a.resplit_(0)
            return matmul(a, b)
        return squeeze_out(_mm(A, B), None)
    if sa == 0 and sb is None:
        return squeeze_out(_mm(A, B), 0, balanced=a.balanced)
    if sa is None and sb == 1:
        return squeeze_out(_mm(A, B), 1, balanced=b.balanced)
    if sa == 0 and sb == 1:
        counts, displs = b.counts_displs()
        if _stream_panels(b, comm):
            # C[:, cols of q] = A_local @ B_q for every rank's column panel, streamed around the ring
            C = torch.empty((A.shape[0], Q), dtype=tt, device=A.device)

            def panel(blk, q):
                C[:, displs[q]: displs[q] + counts[q]] = _mm(A, blk.t())

            ring_pass(B.t().contiguous(), panel, comm, list(counts))
            return squeeze_out(C, 0, balanced=a.balanced)
        Bf = comm.allgather_tensor(B.contiguous(), 1, b.split_counts())
        return squeeze_out(_mm(A, Bf), 0, balanced=a.balanced)
    if sa == 0 and sb == 0:
        counts, displs = b.counts_displs()
        if _stream_panels(b, comm):
            # C = sum_q A_local[:, rows of q] @ B_q, B's row panels streamed around the ring
            C = torch.zeros((A.shape[0], B.shape[1]), dtype=tt, device=A.device)

            def panel(blk, q):
                if counts[q]:
                    C.add_(_mm(A[:, displs[q]: displs[q] + counts[q]], blk))

            ring_pass(B.contiguous(), panel, comm, list(counts))
            return squeeze_out(C, 0, balanced=a.balanced)
        Bf = comm.allgather_tensor(B.contiguous(), 0, b.split_counts())
        return squeeze_out(_mm(A, Bf), 0, balanced=a.balanced)
    if sa == 1 and sb == 1:
        if not vec_a and _stream_panels(a, comm):
            counts, displs = a.counts_displs()
            # C_local = sum_q A_q @ B_local[rows of q], A's column panels streamed around the ring
            C = torch.zeros((L, B.shape[1]), dtype=tt, device=B.device)

            def panel(blk, q):
                if counts[q]:
                    C.add_(_mm(blk.t(), B[displs[q]: displs[q] + counts[q]]))

            ring_pass(A.t().contiguous(), panel, comm, list(counts))
            return squeeze_out(C, 1, balanced=b.balanced)
        Af = comm.allgather_tensor(A.contiguous(), 1, a.split_counts() if not vec_a else None)
        return squeeze_out(_mm(Af, B), 1, balanced=b.balanced)
    # contraction axis distributed: partial products + reduce-scatter
    if sa == 1 and sb is None:
        counts, displs = a.counts_displs()
        r = comm.rank
        part = _mm(A, B[displs[r]: displs[r] + counts[r]])
        split = 1 if (Q > 1 and not vec_b) else 0
    elif sa is None and sb == 0:
        counts, displs = b.counts_displs()
        r = comm.rank
        part = _mm(A[:, displs[r]: displs[r] + counts[r]], B)
        split = 0 if (L > 1 or vec_a) else 1
        if vec_a:
            split = 1
    elif sa == 1 and sb == 0:
        if a.split_counts() != b.split_counts():
            B = b._exchange_rows(b.split_counts(), a.split_counts()).to(tt)
            if vec_b:
                B = B.unsqueeze(1)
        part = _mm(A, B)
        split = 1 if (Q > 1 and not vec_b) else 0
    else:
        raise NotImplementedError("splits > 1 not implemented")
    if vec_a and vec_b:
        comm.Allreduce(MPI.IN_PLACE, part, MPI.SUM)
        return finish(part.reshape(()), (), None)
    if vec_a:
        full = part.reshape(1, -1)
        loc = _reduce_scatter(full, comm, 1)
        return finish(loc.reshape(-1), (Q,), 0)
    if vec_b:
        full = part.reshape(-1, 1)
        loc = _reduce_scatter(full, comm, 0)
        return finish(loc.reshape(-1), (L,), 0)
    loc = _reduce_scatter(part, comm, split)
    return finish(loc, out_shape, split)


DNDarray.__matmul__ = lambda self, other: matmul(self, other)
DNDarray.__rmatmul__ = lambda self, other: matmul(other, self)


def dot(a, b, out: Optional[DNDarray] = None):
    """Dot product: scalars multiply, 1-D inner product, otherwise matmul."""
    if isinstance(a, (float, int)) or isinstance(b, (float, int)) or a.ndim == 0 or b.ndim == 0:
        ret = a * b
        if out is not None:
            out.larray = ret.larray if isinstance(ret, DNDarray) else torch.as_tensor(ret)
            return out
        return ret
    if a.ndim == 1 and b.ndim == 1:
        if a.gshape[0] != b.gshape[0]:
            raise ValueError("shapes {} and {} not aligned".format(a.gshape, b.gshape))
        ret = matmul(a, b)
        if out is not None:
            out.larray.copy_(ret.larray)
            return out
        return ret
    if a.ndim <= 2 and b.ndim <= 2:
        ret = matmul(a, b)
        if out is not None:
            out.larray = ret.larray.to(out.larray.dtype)
            return out
        return ret
    raise NotImplementedError("ht.dot not implemented for N-D dot M-D arrays")


DNDarray.dot = lambda self, b, out=None: dot(self, b, out)


def outer(a: DNDarray, b: DNDarray, out: Optional[DNDarray] = None, split: Optional[int] = None) -> DNDarray:
    """Outer product of two vectors (one all-gather of the other operand instead of a ring)."""
    if not isinstance(a, DNDarray) or not isinstance(b, DNDarray):
        raise TypeError("a and b must be DNDarrays, got {} and {}".format(type(a), type(b)))
    if a.ndim == 0 or b.ndim == 0:
        raise RuntimeError("outer requires arrays of at least one dimension")
    if out is not None and not isinstance(out, DNDarray):
        raise TypeError("out must be a DNDarray, got {}".format(type(out)))
    if a.ndim > 1:
        a = a.flatten()
    if b.ndim > 1:
        b = b.flatten()
    dtype = types.promote_types(a.dtype, b.dtype)
    tt = dtype.torch_type()
    if split is None:
        split = a.split if a.split is not None else (1 if b.split is not None else None)
    gshape = (a.gshape[0], b.gshape[0])
    comm = a.comm
    if split is None or not comm.is_distributed():
        fa = a._gathered().to(tt)
        fb = b._gathered().to(tt)
        res = torch.outer(fa, fb)
        out_arr = DNDarray(res, gshape, dtype, None, a.device, comm, True)
        if split is not None:
            out_arr = factories.array(res, split=split, device=a.device, comm=comm)
    elif split == 0:
        la = a.larray.to(tt) if a.split == 0 else factories.array(a._gathered(), split=0, comm=comm).larray.to(tt)
        fb = b._gathered().to(tt)
        out_arr = DNDarray(torch.outer(la, fb), gshape, dtype, 0, a.device, comm,
                           a.balanced if a.split == 0 else True)
    else:
        fa = a._gathered().to(tt)
        lb = b.larray.to(tt) if b.split == 0 else factories.array(b._gathered(), split=0, comm=comm).larray.to(tt)
        out_arr = DNDarray(torch.outer(fa, lb), gshape, dtype, 1, a.device, comm,
                           b.balanced if b.split == 0 else True)
    if out is not None:
        if out.gshape != out_arr.gshape:
            raise ValueError("out must have shape {}, got {}".format(out_arr.gshape, out.gshape))
        if split is not None and out.split != split:
            raise ValueError("out must have split {}, got {}".format(split, out.split))
        if out.split != out_arr.split:
            from ..manipulations import resplit

            out_arr = resplit(out_arr, out.split)
        out.larray = out_arr.larray.to(out.larray.dtype)
        return out
    return out_arr


def projection(a: DNDarray, b: DNDarray) -> DNDarray:
    """Projection of vector a onto vector b."""
    if not isinstance(a, DNDarray) or not isinstance(b, DNDarray):
        raise TypeError("a, b must be of type ht.DNDarray, but were {}, {}".format(type(a), type(b)))
    if a.ndim != 1 or b.ndim != 1:
        raise RuntimeError("a, b must be vectors of length 1, but were {}, {}".format(a.ndim, b.ndim))
    return (dot(a, b) / dot(b, b)) * b


def trace(a: DNDarray, offset: int = 0, axis1: int = 0, axis2: int = 1, dtype=None, out=None):
    """Sum along a diagonal (a Python scalar for 2-D input, like the reference)."""
    from .. import arithmetics, manipulations

    if not isinstance(a, DNDarray):
        if isinstance(a, (list, tuple)):
            a = factories.array(a)
        else:
            raise TypeError("`a` must be a DNDarray, list or tuple, is {}".format(type(a)))
    if a.ndim < 2:
        raise ValueError("`a` must contain at least 2 dimensions")
    for v, name in ((axis1, "axis1"), (axis2, "axis2"), (offset, "offset")):
        if not isinstance(v, (int, np.integer)) or isinstance(v, bool):
            raise TypeError("{} must be an integer, got {}".format(name, type(v)))
    if out is not None and not isinstance(out, DNDarray):
        raise TypeError("out must be a DNDarray, got {}".format(type(out)))
    if isinstance(dtype, str):
        raise ValueError("dtype must be a heat or torch type, not the string {!r}".format(dtype))
    d = manipulations.diagonal(a, offset=offset, dim1=axis1, dim2=axis2)
    if dtype is not None:
        d = d.astype(dtype)
    s = arithmetics.sum(d, axis=-1)
    if out is not None:
        if a.ndim == 2:
            raise ValueError("the trace of a 2-D array is a scalar: out= is only for n-D input")
        if out.gshape != s.gshape:
            raise ValueError("out must have shape {}, got {}".format(s.gshape, out.gshape))
        if out.split != s.split:
            s = manipulations.resplit(s, out.split)
        out.larray = s.larray.to(out.larray.dtype)
        return out
    if a.ndim == 2:
        return s.item()
    return s


DNDarray.trace = lambda self, offset=0, axis1=0, axis2=1, dtype=None, out=None: trace(self, offset, axis1, axis2, dtype, out)


def _tri(m: DNDarray, k: int, op) -> DNDarray:
    if not isinstance(m, DNDarray):
        raise TypeError("Expected m to be a tensor but was {}".format(type(m)))
    if not isinstance(k, int):
        raise TypeError("Expected k to be integral, but was {}".format(type(k)))
    if m.ndim < 1:
        return m.copy()
    if m.ndim == 1:
        # NumPy: a vector is broadcast to a square matrix first
        n = m.gshape[0]
        full = m._gathered().expand(n, n)
        res = op(full, k)
        out = DNDarray(res.contiguous(), (n, n), m.dtype, None, m.device, m.comm, True)
        if m.split is not None:
            from .. import manipulations

            out = manipulations.resplit(out, 0 if m.split == 0 else 1) if m.comm.is_distributed() else \
                DNDarray(out.larray, (n, n), m.dtype, m.split, m.device, m.comm, True)
        return out
    t = m.larray
    if not m.is_distributed() or m.split < m.ndim - 2:
        return DNDarray(op(t, k), m.gshape, m.dtype, m.split, m.device, m.comm, m.balanced)
    counts, displs = m.counts_displs()
    off = displs[m.comm.rank]
    if m.split == m.ndim - 2:
        kk = k + off  # local row i is global row i+off
    else:
        kk = k - off
    return DNDarray(op(t, kk), m.gshape, m.dtype, m.split, m.device, m.comm, m.balanced)


def tril(m: DNDarray, k: int = 0) -> DNDarray:
    """Lower triangle (elements above the k-th diagonal zeroed)."""
    return _tri(m, k, torch.tril)


def triu(m: DNDarray, k: int = 0) -> DNDarray:
    """Upper triangle (elements below the k-th diagonal zeroed)."""
    return _tri(m, k, torch.triu)


DNDarray.tril = lambda self, k=0: tril(self, k)
DNDarray.triu = lambda self, k=0: triu(self, k)


def vecdot(x1: DNDarray, x2: DNDarray, axis: Optional[int] = None, keepdim: Optional[bool] = None) -> DNDarray:
    """Vector dot product along ``axis`` (default: last)."""
    from .. import arithmetics

    m = arithmetics.mul(x1, x2)
    if axis is None:
        axis = m.ndim - 1
    return arithmetics.sum(m, axis=axis, keepdim=bool(keepdim))


def vector_norm(x: DNDarray, axis=None, keepdims: bool = False, ord=None) -> DNDarray:
    """Vector p-norm over ``axis`` (all elements if None)."""
    from .. import arithmetics, exponential, rounding, statistics

    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a DNDarray, but was {}".format(type(x)))
    if axis is not None and not isinstance(axis, (int, tuple, list)):
        raise TypeError("axis must be an int or a tuple, is {}".format(type(axis)))
    if isinstance(ord, str):
        raise ValueError("Invalid norm order for vectors: {}".format(ord))
    ax = tuple(axis) if isinstance(axis, list) else axis
    xa = rounding.abs(x) if not types.heat_type_is_complexfloating(x.dtype) else _operations.local_op(torch.abs, x, no_cast=True)
    if not types.heat_type_is_inexact(xa.dtype):
        xa = xa.astype(types.promote_types(xa.dtype, types.float32))
    if ord == math.inf or ord == float("inf"):
        return statistics.max(xa, axis=ax, keepdim=keepdims)
    if ord == -math.inf or ord == -float("inf"):
        return statistics.min(xa, axis=ax, keepdim=keepdims)
    if ord == 0:
        return arithmetics.sum(xa != 0, axis=ax, keepdim=keepdims).astype(xa.dtype)
    if ord is None or ord == 2:
        if types.heat_type_is_complexfloating(x.dtype):
            # |z|^2 = re^2 + im^2 without the rounding of a sqrt followed by a square
            sq = _operations.local_op(lambda t: torch.view_as_real(t).square().sum(-1), x, no_cast=True)
            return exponential.sqrt(arithmetics.sum(sq, axis=ax, keepdim=keepdims))
        return exponential.sqrt(arithmetics.sum(xa * xa, axis=ax, keepdim=keepdims))
    if ord == 1:
        return arithmetics.sum(xa, axis=ax, keepdim=keepdims)
    return arithmetics.pow(arithmetics.sum(arithmetics.pow(xa, ord), axis=ax, keepdim=keepdims), 1.0 / ord)


def matrix_norm(x: DNDarray, axis: Optional[Tuple[int, int]] = None, keepdims: bool = False, ord=None) -> DNDarray:
    """Matrix norm ('fro', 'nuc', +-1, +-2, +-inf) over two axes."""
    from .. import arithmetics, exponential, rounding, statistics

    if x.ndim < 2:
        raise ValueError("Input must be a matrix (ndim >= 2)")
    if axis is None:
        if x.ndim > 2:
            raise ValueError("axis must be given for arrays of more than 2 dimensions")
        axis = (0, 1)
    if not isinstance(axis, (tuple, list)) or len(axis) != 2:
        raise TypeError("axis must be a 2-tuple")
    row, col = sanitize_axis(x.gshape, tuple(axis))
    if row == col:
        raise ValueError("Duplicate axes given")
    xa = rounding.abs(x)
    if not types.heat_type_is_inexact(xa.dtype):
        xa = xa.astype(types.promote_types(xa.dtype, types.float32))
    if ord is None or ord == "fro":
        return exponential.sqrt(arithmetics.sum(xa * xa, axis=(row, col), keepdim=keepdims))
    if ord in (1, -1):
        s = arithmetics.sum(xa, axis=row, keepdim=True)
        r = statistics.max(s, axis=col, keepdim=True) if ord == 1 else statistics.min(s, axis=col, keepdim=True)
    elif ord in (math.inf, -math.inf):
        s = arithmetics.sum(xa, axis=col, keepdim=True)
        r = statistics.max(s, axis=row, keepdim=True) if ord > 0 else statistics.min(s, axis=row, keepdim=True)
    elif ord in ("nuc", 2, -2):
        sv = None
        if x.ndim == 2 and x.is_distributed():
            # singular values of a distributed matrix = those of its n x n R factor (tall, split 0)
            # or of R of the transpose (wide, split 1): one TSQR, no gather of the m x n matrix
            from .qr import qr as _qr

            m_, n_ = x.gshape
            src = None
            if x.split == 0 and m_ >= n_:
                src = x if (row, col) == (0, 1) else transpose(x)
            elif x.split == 1 and n_ >= m_:
                src = transpose(x) if (row, col) == (0, 1) else x
            if src is not None and src.split == 0 and src.gshape[0] >= src.gshape[1]:
                R = _qr(src.astype(xa.dtype) if src.dtype != xa.dtype else src, calc_q=False, mode="reduced").R
                Rl = R._gathered() if R.is_distributed() else R.larray
                sv = torch.linalg.svdvals(Rl.to(xa.larray.dtype))
        if sv is None:
            full = x._gathered().to(xa.larray.dtype)
            fm = full.movedim((row, col), (-2, -1))
            sv = torch.linalg.svdvals(fm)
        val = sv.sum(-1) if ord == "nuc" else (sv.max(-1).values if ord == 2 else sv.min(-1).values)
        if keepdims:
            val = val.unsqueeze(-1).unsqueeze(-1).movedim((-2, -1), (row, col))
        return DNDarray(val, tuple(val.shape), types.canonical_heat_type(val.dtype), None, x.device, x.comm, True)
    else:
        raise ValueError("Invalid norm order for matrices: {}".format(ord))
    if not keepdims:
        from .. import manipulations

        r = manipulations.squeeze(r, axis=(row, col))
    return r


def norm(x: DNDarray, axis=None, keepdims: bool = False, ord=None) -> DNDarray:
    """Matrix or vector norm (NumPy semantics)."""
    if not isinstance(x, DNDarray):
        raise TypeError("'x' must be a DNDarray, but is {}".format(type(x)))
    if axis is None:
        if ord is None:
            return vector_norm(x, axis=None, keepdims=keepdims)
        if x.ndim == 2:
            return matrix_norm(x, keepdims=keepdims, ord=ord)
        if x.ndim == 1:
            return vector_norm(x, keepdims=keepdims, ord=ord)
        raise ValueError("Improper number of dimensions to norm.")
    if isinstance(axis, int) or (isinstance(axis, (tuple, list)) and len(axis) == 1):
        ax = axis if isinstance(axis, int) else axis[0]
        return vector_norm(x, axis=ax, keepdims=keepdims, ord=ord)
    if isinstance(axis, (tuple, list)) and len(axis) == 2:
        return matrix_norm(x, axis=tuple(axis), keepdims=keepdims, ord=ord)
    raise ValueError("Improper number of dimensions to norm.")


DNDarray.norm = lambda self: norm(self)
