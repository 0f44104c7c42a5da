// Intra-node collectives over peer (xGMI) mappings of hipIpc-shared buffers: a
// one-shot all-reduce (small messages: the k-means k*f+k sums, moment triples, argmin packs,
// metadata maps, where RCCL's ring/tree start-up dominates), a two-shot reduce-scatter +
// all-gather all-reduce for larger payloads and a direct W-peer all-gather (ipc_allreduce2,
// ipc_allgather below).
//
// Every rank owns one data buffer (two slots, alternating by call parity) and one signal buffer,
// both exported with hipIpcGetMemHandle and mapped by every peer. One call = one kernel:
//   block b copies its slice S_b of the input into its own slot, releases at system scope and
//   writes the call's epoch into slot [b][rank] of every peer's signal buffer; it then waits until
//   all peers' epochs for block b have arrived in its own signal buffer, acquires, and sums S_b of
//   every rank's slot in rank order (bitwise identical results on all ranks) into the output.
// The barrier is per block, so a block only waits for the peers' copies of ITS slice: no grid-wide
// synchronisation and no dependence on which blocks are co-resident. Slot reuse is safe with two
// slots: a rank writes a slot again two calls later, after a barrier for which every peer's block b
// already finished reading it (kernels of one stream are ordered). Epochs only grow, and waits use
// ">=", so a fast peer announcing the next epoch cannot starve a slow waiter.
// Spins are bounded: on timeout the block records an error word in its own signal buffer, fills
// its output slice with NaN (floating types; the stale sum is never returned silently) and exits
// (no hang). ha_ipc_error_async copies the word into pinned host memory behind every call; the
// host raises at the next call (or at an explicit check) and the communicator is poisoned, since
// the two-slot reuse argument no longer holds after a missed barrier.
//
// Coherence of the data slots. The slots are ordinary coarse-grained hipMalloc memory (only the
// signal words are uncached): a rank writes only its OWN slot, with plain stores that may sit
// dirty in its L2, and peers read it over xGMI, possibly through lines of THEIR L2. Both sides
// are covered by the system-scope fences of ipc_block_barrier: on gfx950 the release fence is
// `buffer_wbl2 sc0 sc1` (every dirty L2 line of the writer written back to HBM before its epoch
// is stored) and the acquire fence `buffer_inv sc0 sc1` (the reader's L2 invalidated at system
// scope after it saw every peer's epoch, so no stale line of a previous call's slot survives).
// tests/test_ipc_coherence.py compiles this file for gfx950 and checks that every IPC kernel
// carries that write-back / invalidate pair, so a compiler or scope change cannot drop it
// silently. The MALL sits on the memory side and is coherent for all agents.
#include "common.h"

#include <cstring>
#include <limits>
#include <type_traits>

namespace {

constexpr int IPC_MAX_RANKS = 8;
constexpr int IPC_MAX_BLOCKS = 64;
constexpr int IPC_PHASES = 2;  // barriers per call (two-shot: after the copy, after the reduction)
constexpr int IPC_ERR_WORD = IPC_PHASES * IPC_MAX_BLOCKS * IPC_MAX_RANKS;  // uint32 index of the error word

struct PeerPtrs {
  void* data[IPC_MAX_RANKS];
  unsigned* sig[IPC_MAX_RANKS];
};

template <typename T>
__device__ __forceinline__ T poison() {
  if constexpr (std::is_integral<T>::value) return std::numeric_limits<T>::min();  // an implausible sum
  else return std::numeric_limits<T>::quiet_NaN();
}

// Per-block barrier among the W ranks for phase ph of the call with this epoch: threads 0..W-1
// release this block's writes and announce them to peer threadIdx.x, then wait for that peer's
// announcement. Returns false (and records the error word) when a peer misses it.
template <int W>
__device__ bool ipc_block_barrier(const PeerPtrs& pp, int rank, int ph, unsigned epoch, int64_t max_spins,
                                  int* timed_out) {
  __syncthreads();
  const int b = blockIdx.x;
  if (threadIdx.x < W) {
    const int slotw = (ph * IPC_MAX_BLOCKS + b) * IPC_MAX_RANKS;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(pp.sig[threadIdx.x] + slotw + rank, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* flag = pp.sig[rank] + slotw + threadIdx.x;
    int64_t spins = 0;
    while ((int)(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (++spins > max_spins) {
        __hip_atomic_store(pp.sig[rank] + IPC_ERR_WORD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        *timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  return *timed_out == 0;
}

template <typename T, int W>
__global__ __launch_bounds__(256) void ipc_allreduce(PeerPtrs pp, int rank, T* __restrict__ buf, int64_t n,
                                                     int64_t chunk, int64_t slot_off, unsigned epoch,
                                                     int64_t max_spins) {
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __syncthreads();
  const int b = blockIdx.x;
  const int64_t lo = (int64_t)b * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  T* mine = reinterpret_cast<T*>(pp.data[rank]) + slot_off;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = buf[i];
  if (!ipc_block_barrier<W>(pp, rank, 0, epoch, max_spins, &timed_out)) {
    // a peer never arrived: poison this block's output instead of summing stale slots
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) buf[i] = poison<T>();
    return;
  }
  const T* src[W];
#pragma unroll
  for (int r = 0; r < W; ++r) src[r] = reinterpret_cast<const T*>(pp.data[r]) + slot_off;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    T v[W];
#pragma unroll
    for (int r = 0; r < W; ++r) v[r] = src[r][i];  // all loads in flight before the sum
    T s = v[0];
#pragma unroll
    for (int r = 1; r < W; ++r) s += v[r];
    buf[i] = s;
  }
}

// Two-shot all-reduce for larger payloads: the input is cut into W segments; after the copy
// barrier rank r sums segment r of every slot (rank order) back into its own slot, and after the
// second barrier every rank gathers the W reduced segments from their owners' slots. Each rank
// moves 2 (W-1)/W n elements over the links instead of the one-shot's (W-1) n. Block b handles
// sub-chunk b of every segment, so both barriers stay per block.
template <typename T, int W>
__global__ __launch_bounds__(256) void ipc_allreduce2(PeerPtrs pp, int rank, T* __restrict__ buf, int64_t n,
                                                      int64_t slot_off, unsigned epoch, int64_t max_spins) {
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  const int64_t seg = (n + W - 1) / W;
  const int64_t sc = (seg + gridDim.x - 1) / gridDim.x;
  const int64_t o0 = (int64_t)blockIdx.x * sc;
  T* mine = reinterpret_cast<T*>(pp.data[rank]) + slot_off;
#pragma unroll
  for (int q = 0; q < W; ++q) {
    const int64_t lo = q * seg + o0, hi = min(min(lo + sc, (q + 1) * seg), n);
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = buf[i];
  }
  bool ok = ipc_block_barrier<W>(pp, rank, 0, epoch, max_spins, &timed_out);
  if (ok) {
    const T* src[W];
#pragma unroll
    for (int r = 0; r < W; ++r) src[r] = reinterpret_cast<const T*>(pp.data[r]) + slot_off;
    const int64_t lo = rank * seg + o0, hi = min(min(lo + sc, (rank + 1) * seg), n);
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
      T v[W];
#pragma unroll
      for (int r = 0; r < W; ++r) v[r] = src[r][i];
      T acc = v[0];
#pragma unroll
      for (int r = 1; r < W; ++r) acc += v[r];
      mine[i] = acc;  // only this rank reads segment `rank` of its own slot
    }
    ok = ipc_block_barrier<W>(pp, rank, 1, epoch, max_spins, &timed_out);
  } else {
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < W; ++q) {
    const T* sq = reinterpret_cast<const T*>(pp.data[q]) + slot_off;
    const int64_t lo = q * seg + o0, hi = min(min(lo + sc, (q + 1) * seg), n);
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) buf[i] = ok ? sq[i] : poison<T>();
  }
}

// Direct all-gather: every rank copies its block (count[rank] 32-bit words) into its slot; after
// the barrier it pulls every peer's block straight from the peer's slot into out + displ[q] - W-1
// concurrent reads over the point-to-point xGMI links instead of a ring's W-1 dependent steps.
struct GatherLayout {
  int64_t count[IPC_MAX_RANKS];
  int64_t displ[IPC_MAX_RANKS];
};

template <int W>
__global__ __launch_bounds__(256) void ipc_allgather(PeerPtrs pp, int rank, const unsigned* __restrict__ in,
                                                     unsigned* __restrict__ out, GatherLayout gl, int64_t slot_off,
                                                     unsigned epoch, int64_t max_spins) {
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  unsigned* mine = reinterpret_cast<unsigned*>(pp.data[rank]) + slot_off;
  {
    const int64_t c = gl.count[rank], sc = (c + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * sc, hi = min(lo + sc, c);
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = in[i];
  }
  const bool ok = ipc_block_barrier<W>(pp, rank, 0, epoch, max_spins, &timed_out);
#pragma unroll
  for (int q = 0; q < W; ++q) {
    const unsigned* sq = reinterpret_cast<const unsigned*>(pp.data[q]) + slot_off;
    const int64_t c = gl.count[q], sc = (c + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * sc, hi = min(lo + sc, c);
    unsigned* o = out + gl.displ[q];
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) o[i] = ok ? sq[i] : 0xFFFFFFFFu;
  }
}

template <typename T>
int launch(const PeerPtrs& pp, int world, int rank, T* buf, int64_t n, int64_t slot_off, unsigned epoch,
           int blocks, int64_t max_spins, int two_shot, hipStream_t s) {
  const int64_t chunk = (n + blocks - 1) / blocks;
  const int grid = (int)((n + chunk - 1) / chunk);
#define HA_IPC(WN)                                                                                          \
  case WN:                                                                                                  \
    if (two_shot)                                                                                           \
      hipLaunchKernelGGL((ipc_allreduce2<T, WN>), dim3(blocks), dim3(256), 0, s, pp, rank, buf, n, slot_off, \
                         epoch, max_spins);                                                                 \
    else                                                                                                    \
      hipLaunchKernelGGL((ipc_allreduce<T, WN>), dim3(grid), dim3(256), 0, s, pp, rank, buf, n, chunk,      \
                         slot_off, epoch, max_spins);                                                       \
    break;
  switch (world) {
    HA_IPC(2) HA_IPC(3) HA_IPC(4) HA_IPC(5) HA_IPC(6) HA_IPC(7) HA_IPC(8)
    default: return HA_UNSUPPORTED;
  }
#undef HA_IPC
  return ha_launch_status();
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI
HA_EXPORT int ha_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }
HA_EXPORT int ha_ipc_max_ranks() { return IPC_MAX_RANKS; }
HA_EXPORT int ha_ipc_max_blocks() { return IPC_MAX_BLOCKS; }
HA_EXPORT int64_t ha_ipc_signal_bytes() { return (int64_t)(IPC_ERR_WORD + 64) * 4; }

// Allocate an exportable device buffer (uncached when ``signal``, zero-filled) and its IPC handle.
HA_EXPORT int ha_ipc_alloc(int64_t bytes, int signal, void** ptr, void* handle) {
  if (bytes <= 0 || !ptr || !handle) return HA_BAD_ARG;
  hipError_t e = signal ? hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached)
                        : hipMalloc(ptr, (size_t)bytes);
  if (e != hipSuccess && signal) e = hipMalloc(ptr, (size_t)bytes);
  if (e != hipSuccess) return HA_LAUNCH;
  if (hipMemset(*ptr, 0, (size_t)bytes) != hipSuccess) return HA_LAUNCH;
  if (hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), *ptr) != hipSuccess) return HA_LAUNCH;
  return HA_OK;
}

HA_EXPORT int ha_ipc_free(void* ptr) { return hipFree(ptr) == hipSuccess ? HA_OK : HA_LAUNCH; }

HA_EXPORT int ha_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? HA_OK : HA_LAUNCH;
}

HA_EXPORT int ha_ipc_close(void* ptr) { return hipIpcCloseMemHandle(ptr) == hipSuccess ? HA_OK : HA_LAUNCH; }

// In-place SUM of ``buf`` (n elements, dtype 0 = float32, 1 = float64, 2 = int64) over ``world``
// ranks. data/sig: the world's mapped buffer pointers (own ones included), slot_elems: elements
// per slot; ``epoch`` must grow by one per call on every rank.
HA_EXPORT int ha_ipc_allreduce(void* const* data, void* const* sig, int world, int rank, void* buf, int64_t n,
                               int dtype, int64_t slot_elems, unsigned epoch, int blocks, int64_t max_spins,
                               int two_shot, void* stream) {
  if (world < 2 || world > IPC_MAX_RANKS || rank < 0 || rank >= world || n < 0 || n > slot_elems) return HA_BAD_ARG;
  if (n == 0) return HA_OK;
  blocks = blocks < 1 ? 1 : blocks > IPC_MAX_BLOCKS ? IPC_MAX_BLOCKS : blocks;
  PeerPtrs pp{};
  for (int r = 0; r < world; ++r) {
    pp.data[r] = data[r];
    pp.sig[r] = reinterpret_cast<unsigned*>(sig[r]);
  }
  const int64_t slot_off = (epoch & 1u) ? slot_elems : 0;
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case 0: return launch<float>(pp, world, rank, (float*)buf, n, slot_off, epoch, blocks, max_spins, two_shot, s);
    case 1: return launch<double>(pp, world, rank, (double*)buf, n, slot_off, epoch, blocks, max_spins, two_shot, s);
    case 2:
      return launch<int64_t>(pp, world, rank, (int64_t*)buf, n, slot_off, epoch, blocks, max_spins, two_shot, s);
    default: return HA_UNSUPPORTED;
  }
}

// All-gather of 32-bit words: ``in`` holds counts[rank] words, ``out`` receives every rank's block
// at displs[q] (words). slot_words: words per slot (>= every count). Same epoch rule as above.
HA_EXPORT int ha_ipc_allgather(void* const* data, void* const* sig, int world, int rank, const void* in, void* out,
                               const int64_t* counts, const int64_t* displs, int64_t slot_words, unsigned epoch,
                               int blocks, int64_t max_spins, void* stream) {
  if (world < 2 || world > IPC_MAX_RANKS || rank < 0 || rank >= world) return HA_BAD_ARG;
  GatherLayout gl{};
  int64_t total = 0;
  for (int r = 0; r < world; ++r) {
    if (counts[r] < 0 || counts[r] > slot_words) return HA_BAD_ARG;
    gl.count[r] = counts[r];
    gl.displ[r] = displs[r];
    total += counts[r];
  }
  if (total == 0) return HA_OK;
  blocks = blocks < 1 ? 1 : blocks > IPC_MAX_BLOCKS ? IPC_MAX_BLOCKS : blocks;
  PeerPtrs pp{};
  for (int r = 0; r < world; ++r) {
    pp.data[r] = data[r];
    pp.sig[r] = reinterpret_cast<unsigned*>(sig[r]);
  }
  const int64_t slot_off = (epoch & 1u) ? slot_words : 0;
  hipStream_t s = (hipStream_t)stream;
#define HA_AG(WN)                                                                                           \
  case WN:                                                                                                  \
    hipLaunchKernelGGL((ipc_allgather<WN>), dim3(blocks), dim3(256), 0, s, pp, rank, (const unsigned*)in,    \
                       (unsigned*)out, gl, slot_off, epoch, max_spins);                                     \
    break;
  switch (world) {
    HA_AG(2) HA_AG(3) HA_AG(4) HA_AG(5) HA_AG(6) HA_AG(7) HA_AG(8)
    default: return HA_UNSUPPORTED;
  }
#undef HA_AG
  return ha_launch_status();
}

// Stream-ordered copy of the error word into host memory (pinned, or any host pointer the runtime
// can DMA to) behind the calls already on ``stream``.
HA_EXPORT int ha_ipc_error_async(void* sig, void* host, void* stream) {
  unsigned* w = reinterpret_cast<unsigned*>(sig) + IPC_ERR_WORD;
  return hipMemcpyAsync(host, w, 4, hipMemcpyDeviceToHost, (hipStream_t)stream) == hipSuccess ? HA_OK : HA_LAUNCH;
}

// Error word of this rank's signal buffer (1 after a barrier timed out); reset with clear != 0.
HA_EXPORT int ha_ipc_error(void* sig, int clear) {
  unsigned v = 0;
  unsigned* w = reinterpret_cast<unsigned*>(sig) + IPC_ERR_WORD;
  if (hipMemcpy(&v, w, 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (clear && hipMemset(w, 0, 4) != hipSuccess) return -1;
  return (int)v;
}
