// Block pack / unpack for personalised all-to-all exchanges (resplit, Alltoallv).
//
// A tensor is viewed as rows: (O, S, R) with S the axis that is cut into p blocks (block q = rows
// [off[q], off[q+1]) of S) and R the contiguous bytes of one row. The wire format of an
// all-to-all is the blocks one after the other, each in C order: block q = (O, off[q+1]-off[q], R).
//   pack:   wire[O*off[q] + o*c_q + (s - off[q])] = tensor[o*S + s]
//   unpack: tensor[o*S + s] = wire[O*off[q] + o*c_q + (s - off[q])]
// One pass over the data replaces p strided narrow().contiguous() copies plus a torch.cat on the
// send side and p copies plus a cat on the receive side (reference: MPI derived datatypes,
// communication.py:242-437). Every thread moves one W-byte word (W = 16 when the row size and
// both base pointers allow it); the block of a row is found by a binary search over p+1 offsets
// held in the kernel argument segment.
#include "common.h"

namespace {

constexpr int kMaxBlocks = 256;

struct BlockOffsets {
  int64_t off[kMaxBlocks + 1];
  int p;
};

template <typename W>
__global__ __launch_bounds__(256) void rows_permute(const W* __restrict__ src, W* __restrict__ dst, int64_t O,
                                                    int64_t S, int64_t nw, BlockOffsets bo, int unpack) {
  const int64_t total = O * S * nw;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t row = i / nw;
    const int64_t c = i - row * nw;
    const int64_t o = row / S;
    const int64_t s = row - o * S;
    // block of s: the last q with off[q] <= s (empty blocks have off[q] == off[q+1])
    int lo = 0, hi = bo.p;  // invariant: off[lo] <= s < off[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (bo.off[mid] <= s) lo = mid; else hi = mid;
    }
    const int64_t c_q = bo.off[lo + 1] - bo.off[lo];
    const int64_t wrow = O * bo.off[lo] + o * c_q + (s - bo.off[lo]);
    if (unpack) dst[row * nw + c] = src[wrow * nw + c];
    else dst[wrow * nw + c] = src[row * nw + c];
  }
}

template <typename W>
int launch(const void* src, void* dst, int64_t O, int64_t S, int64_t row_bytes, const BlockOffsets& bo, int unpack,
           hipStream_t stream) {
  const int64_t nw = row_bytes / (int64_t)sizeof(W);
  const int64_t total = O * S * nw;
  if (total <= 0) return HA_OK;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;  // grid-stride beyond 32 waves per CU
  hipLaunchKernelGGL(rows_permute<W>, dim3((unsigned)blocks), dim3(256), 0, stream, (const W*)src, (W*)dst, O, S, nw,
                     bo, unpack);
  return ha_launch_status();
}

}  // namespace

// offsets: p+1 prefix offsets along S (offsets[0] == 0, offsets[p] == S), p <= 256.
HA_EXPORT int ha_rows_permute(const void* src, void* dst, int64_t O, int64_t S, int64_t row_bytes,
                              const int64_t* offsets, int p, int unpack, void* stream) {
  if (p < 1 || p > kMaxBlocks || O < 0 || S < 0 || row_bytes < 0) return HA_BAD_ARG;
  if (offsets[0] != 0 || offsets[p] != S) return HA_BAD_ARG;
  BlockOffsets bo;
  bo.p = p;
  for (int q = 0; q <= p; ++q) {
    if (q && offsets[q] < offsets[q - 1]) return HA_BAD_ARG;
    bo.off[q] = offsets[q];
  }
  for (int q = p + 1; q <= kMaxBlocks; ++q) bo.off[q] = S;
  hipStream_t s = (hipStream_t)stream;
  const uintptr_t a = (uintptr_t)src | (uintptr_t)dst | (uintptr_t)row_bytes;
  if ((a & 15) == 0) return launch<uint4>(src, dst, O, S, row_bytes, bo, unpack, s);
  if ((a & 7) == 0) return launch<uint2>(src, dst, O, S, row_bytes, bo, unpack, s);
  if ((a & 3) == 0) return launch<uint32_t>(src, dst, O, S, row_bytes, bo, unpack, s);
  if ((a & 1) == 0) return launch<uint16_t>(src, dst, O, S, row_bytes, bo, unpack, s);
  return launch<uint8_t>(src, dst, O, S, row_bytes, bo, unpack, s);
}
