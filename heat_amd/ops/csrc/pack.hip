// Block pack / unpack for personalised all-to-all exchanges (resplit, Alltoallv).
//
// A tensor is viewed as rows: (O, S, R) with S the axis that is cut into p blocks (block q = rows
// [off[q], off[q+1]) of S) and R the contiguous bytes of one row. The wire format of an
// all-to-all is the blocks one after the other, each in C order: block q = (O, off[q+1]-off[q], R).
//   pack:   wire[O*off[q] + o*c_q + (s - off[q])] = tensor[o*S + s]
//   unpack: tensor[o*S + s] = wire[O*off[q] + o*c_q + (s - off[q])]
// One pass over the data replaces p strided narrow().contiguous() copies plus a torch.cat on the
// send side and p copies plus a cat on the receive side (reference: MPI derived datatypes,
// communication.py:242-437). Each block of one outer index is ONE contiguous run on both sides,
// so threads walk the wire buffer linearly and every access is coalesced; each thread moves one
// W-byte word (W = 16 when the base pointers and every block boundary in bytes allow it, so even
// 4-byte rows of a 1-D split move as 16-byte words). The block of a word is found by a binary
// search over p+1 offsets held in the kernel argument segment.
#include "common.h"

namespace {

constexpr int kMaxBlocks = 256;

// offsets in W-byte words along the flattened (S x R) row of one outer index
struct BlockOffsets {
  int64_t off[kMaxBlocks + 1];  // block starts within a row of Sw words (off[p] == Sw)
  int p;
};

// One W-byte word per thread, indexed by its position j in the WIRE buffer, so that consecutive
// threads touch consecutive words on both sides (a block of one outer index is one contiguous run
// in the tensor AND in the wire). The block of j is found by binary search over O * off[q].
template <typename W>
__global__ __launch_bounds__(256) void runs_permute(const W* __restrict__ src, W* __restrict__ dst, int64_t O,
                                                    int64_t Sw, BlockOffsets bo, int unpack) {
  const int64_t total = O * Sw;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += stride) {
    int lo = 0, hi = bo.p;  // invariant: O*off[lo] <= j < O*off[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (O * bo.off[mid] <= j) lo = mid; else hi = mid;
    }
    const int64_t cw = bo.off[lo + 1] - bo.off[lo];
    const int64_t local = j - O * bo.off[lo];
    const int64_t o = local / cw;
    const int64_t t = o * Sw + bo.off[lo] + (local - o * cw);
    if (unpack) dst[t] = src[j];
    else dst[j] = src[t];
  }
}

template <typename W>
int launch(const void* src, void* dst, int64_t O, int64_t S, int64_t row_bytes, const int64_t* offsets, int p,
           int unpack, hipStream_t stream) {
  BlockOffsets bo;
  bo.p = p;
  const int64_t rw = (int64_t)sizeof(W);
  for (int q = 0; q <= p; ++q) bo.off[q] = offsets[q] * row_bytes / rw;
  for (int q = p + 1; q <= kMaxBlocks; ++q) bo.off[q] = bo.off[p];
  const int64_t Sw = S * row_bytes / rw;
  const int64_t total = O * Sw;
  if (total <= 0) return HA_OK;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;  // grid-stride beyond 32 waves per CU
  hipLaunchKernelGGL(runs_permute<W>, dim3((unsigned)blocks), dim3(256), 0, stream, (const W*)src, (W*)dst, O, Sw,
                     bo, unpack);
  return ha_launch_status();
}

}  // namespace

// offsets: p+1 prefix offsets along S (offsets[0] == 0, offsets[p] == S), p <= 256.
HA_EXPORT int ha_rows_permute(const void* src, void* dst, int64_t O, int64_t S, int64_t row_bytes,
                              const int64_t* offsets, int p, int unpack, void* stream) {
  if (p < 1 || p > kMaxBlocks || O < 0 || S < 0 || row_bytes < 0) return HA_BAD_ARG;
  if (offsets[0] != 0 || offsets[p] != S) return HA_BAD_ARG;
  // the word: the largest power of two <= 16 dividing both base addresses and every block
  // boundary in bytes (then every run starts and ends on a word on both sides)
  uint64_t a = (uintptr_t)src | (uintptr_t)dst | (uint64_t)(S * row_bytes);
  for (int q = 0; q <= p; ++q) {
    if (q && offsets[q] < offsets[q - 1]) return HA_BAD_ARG;
    a |= (uint64_t)(offsets[q] * row_bytes);
  }
  hipStream_t s = (hipStream_t)stream;
  if ((a & 15) == 0) return launch<uint4>(src, dst, O, S, row_bytes, offsets, p, unpack, s);
  if ((a & 7) == 0) return launch<uint2>(src, dst, O, S, row_bytes, offsets, p, unpack, s);
  if ((a & 3) == 0) return launch<uint32_t>(src, dst, O, S, row_bytes, offsets, p, unpack, s);
  if ((a & 1) == 0) return launch<uint16_t>(src, dst, O, S, row_bytes, offsets, p, unpack, s);
  return launch<uint8_t>(src, dst, O, S, row_bytes, offsets, p, unpack, s);
}
