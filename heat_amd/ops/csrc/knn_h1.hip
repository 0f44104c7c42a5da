// hipcc-flags: -fno-slp-vectorize
// Certified one-term kNN top-k (h1_topk, see its comment) on the FP16 matrix cores: the screening
// pass of ops.knn_topk; uncertain points go back through h3_topk_p (knn_f16x3.hip). Split from
// knn_f16x3.hip so that the two kernel families compile in parallel.
#include "h3_common.h"

namespace {

// s_waitcnt vmcnt(N), expcnt / lgkmcnt left alone (gfx9 encoding: vmcnt bits 3:0 and 15:14,
// expcnt 6:4, lgkmcnt 11:8)
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4; LDS address = lds + 16 lane) issued
// through inline asm: for the builtin the compiler's wait-count pass cannot tell which LDS bytes
// the transfer writes and puts s_waitcnt vmcnt(0) before the next LDS read - i.e. it waits for
// the prefetched chunks too. The asm form is invisible to that pass (its own vmcnt waits only
// become more conservative); the kernel waits for its transfers with counted vm_wait<N>().
// M0 (the LDS address of the transfer) is saved and restored around it: the compiler treats M0 as
// reserved and would not see a clobber.
// The LDS address is wave-uniform; readfirstlane pins it to an SGPR (inside a lane-divergent
// branch the compiler may otherwise hand the "s" operand a VGPR).
__device__ __forceinline__ void lds_dma16(const void* g, unsigned lds) {
  unsigned saved;
  const unsigned base = __builtin_amdgcn_readfirstlane(lds);
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(saved)
               : "v"(g), "s"(base)
               : "memory");
}

// Sorted insertion into a descending list with the eviction recorded in rej (the caller has
// checked v > tv[KP - 1]). Slot s keeps median(tv[s - 1], v, tv[s]) - one v_med3_f32 instead of
// two selects - and the index follows with two selects on the shared compares.
template <int KP>
__device__ __forceinline__ void topk_insert_ev(float (&tv)[KP], int (&ti)[KP], float v, int id, float& rej) {
  rej = fmaxf(rej, tv[KP - 1]);  // the evicted last entry (-inf while the list is not full)
#pragma unroll
  for (int s = KP - 1; s >= 1; --s) {
    const bool ap = v > tv[s - 1];
    const bool ac = v > tv[s];
    ti[s] = ap ? ti[s - 1] : (ac ? id : ti[s]);
    tv[s] = __builtin_amdgcn_fmed3f(tv[s - 1], v, tv[s]);
  }
  ti[0] = v > tv[0] ? id : ti[0];
  tv[0] = fmaxf(tv[0], v);
}

// Uniform centroid scale for h1_topk: r_c = 2^e for EVERY live row, e from max_c max_i |c_i|
// (meta[1], posted by h3_cscale), and the rank-1 fragments -u_c / r_c re-split to match. Then a
// tile's accumulator is the score / r, the same r for all rows: the kernel's epilogue compares
// raw accumulators (no per-row multiply, no r staging) and scales its lists once at the end.
// The h1 error bound E is unchanged: it is already stated with the global c_max, and the fp16
// subnormal range (components below 2^-14 of the largest) adds at most f 2^-25 r |x_s|_inf <=
// 2^-17 c_max, inside E's 2^-15 c_max term.
template <int FPAD>
__global__ __launch_bounds__(256) void h3_uniform_r(int k, float* __restrict__ ur, const float* __restrict__ meta,
                                                    unsigned* __restrict__ vimg) {
  constexpr int CB = H3Cfg<FPAD>::CB;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= k) return;
  const float mx = meta[1];
  int e = 0;
  if (mx > 0.f && mx < __builtin_huge_valf()) frexpf(mx, &e);
  float* urc = ur + (int64_t)(c / CB) * 2 * CB + c % CB;
  urc[CB] = ldexpf(1.f, e);
  const float y = -ldexpf(urc[0], -e);  // -u_c / r, split into hi + mid + lo bf16 (24 bits)
  const unsigned hi = h3_bf16_rn(y);
  const float r1 = y - h3_bf16_f(hi);
  const unsigned mid = h3_bf16_rn(r1);
  const unsigned lo = h3_bf16_rn(r1 - h3_bf16_f(mid));
  unsigned* vc = vimg + ((int64_t)(c / 32) * 64 + c % 32) * 2;
  vc[0] = hi | (mid << 16);
  vc[1] = lo;
}

// Certified one-term top-k ("h1"), the kNN form of h1_filter: scores from hi_c . hi_x only (ONE
// MFMA per k-step instead of three) plus the exact rank-1 u term, each within E of the fp32 score
// (E: h1_filter's bound). A lane keeps its KH best approximate scores and `rej`, an upper bound
// of every score it let go (rejected or evicted). After the halves merge, a point is CERTIFIED when
//     rej < a_kn - 2 E          (a_kn = the kn-th best approximate score in the list):
// then every candidate outside the list is, exactly, below kn candidates inside it, so the true
// top-kn is a subset of the KO-list, which the caller rescores exactly. Uncertain points are
// flagged (cert = 0) and re-run through the 3-term kernel by the caller.
// Output per point: KO approximate squared distances (ascending) and int32 indices, cert flag.
//
// Round 5 structure (round 4: 31-35 % MFMA-busy at 2 waves / SIMD; its ISA shows every A
// fragment read from LDS into the SAME registers right before its MFMA - 256 VGPRs in use, so
// the LDS latency was exposed 8 times per tile - and the epilogue in a branch of its own):
//  * one workgroup of 4 waves per CU, 512 registers per wave, 2 x 32 points per wave (NPB = 2:
//    each A fragment read feeds two MFMAs, 256 points per workgroup as before per CU);
//  * the next tile's A fragments are read while the current tile's MFMAs run;
//  * chunks of 4 tiles staged by LDS-DMA into a ring of 4 buffers, 3 chunks in flight, one
//    barrier per chunk (the ring slot refilled is the one every wave finished before it);
//  * uniform centroid scale (h3_uniform_r): the epilogue is a max3 tree, one med3 for rej and a
//    compare per 16 scores, branch-free so it fills the MFMA gaps;
//  * selection through a per-lane queue of Q candidates above the threshold: the sorted insertion
//    (the expensive part: a wave runs the union of its lanes' insertions) runs only when some
//    lane's queue is full, for Q candidates of every lane at once.
// rej bookkeeping: the epilogue sets rej = med3(rej, m, thr) = max(rej, min(m, thr)) with m the
// tile max and thr the list's last entry (rej <= thr always holds): it covers every score of the
// tile that is not queued. Queued scores that no longer beat the list at merge time go to rej
// exactly; evictions too.
template <int FPAD, int KH, int KO, int NPB, int TPI, int MINB, int WAVES = 4, int GRP = 1>
__global__ __launch_bounds__(64 * WAVES, MINB) void h1_topk(const _Float16* __restrict__ planes, const float* __restrict__ sxv,
                                                  int64_t n, const _Float16* __restrict__ image,
                                                  const float* __restrict__ u, const float* __restrict__ meta,
                                                  int nch, int kn, float* __restrict__ dist, int* __restrict__ idx,
                                                  unsigned char* __restrict__ cert, int dbg) {
  using K = H3Cfg<FPAD, NPB>;
  constexpr int F2 = K::F2, KS = K::KS;
  // NPB: 32-point blocks per wave; TPI: 32-centroid tiles per staged chunk; MINB: workgroups / CU
  constexpr int PIECES = TPI * KS;        // 1 KB hi-fragment pieces per chunk (piece q <- image piece 2q)
  constexpr int BUF = PIECES * 1024 + TPI * 512;  // + rank-1 fragments (512 B per tile)
  // chunks in flight, ring slots. GRP > 1: one barrier per GROUP of GRP chunks (all landed), chunk
  // ch + GRP issued during chunk ch into a 2 GRP-slot ring (the barrier waits were a quarter of a
  // chunk's time: stamps). GRP = 1: a barrier per chunk, 3 (2) chunks in flight.
  constexpr int AHEAD = GRP > 1 ? GRP : TPI >= 3 ? 2 : 3, NB = GRP > 1 ? 2 * GRP : AHEAD + 1;
  constexpr int IMGW = PIECES / WAVES;    // image pieces per wave per chunk
  constexpr int PTS_PER_WG = WAVES * NPB * 32;
  constexpr int Q = 4;                    // queue slots per list
  constexpr float NINF = -__builtin_huge_valf();
  static_assert(PIECES % WAVES == 0 && (TPI + 1) / 2 <= WAVES, "pieces per wave");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, h = lane >> 5;
  const int64_t pbase = (int64_t)blockIdx.x * PTS_PER_WG + (int64_t)wave * (NPB * 32);

  halfx8 bhi[NPB][KS];
  bf16x8 bsx[NPB];
  float sx[NPB], hsq[NPB], xsq[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int64_t pi = pbase + pb * 32 + j;
    const int64_t row = pi < n ? pi : n - 1;
    const _Float16* pr = planes + row * (2 * FPAD) + h * F2;
    float q = 0.f, q3 = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bhi[pb][ks] = *reinterpret_cast<const halfx8*>(pr + 8 * ks);
      const halfx8 lo = *reinterpret_cast<const halfx8*>(pr + FPAD + 8 * ks);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float hv = (float)bhi[pb][ks][i];
        q = fmaf(hv, hv, q);
        const float xv = hv + (float)lo[i];
        q3 = fmaf(xv, xv, q3);
      }
    }
    sx[pb] = sxv[row];
    hsq[pb] = q;
    xsq[pb] = q3;
    const unsigned sb = __float_as_uint(sx[pb]) >> 16;
    const u32x4 bw = {h ? 0u : (sb | (sb << 16)), h ? 0u : sb, 0u, 0u};
    bsx[pb] = __builtin_bit_cast(bf16x8, bw);
  }
  float tv[NPB][KH], rej[NPB], thr0[NPB], qv[NPB][Q];
  int ti[NPB][KH], qi[NPB][Q], qn[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    rej[pb] = NINF;
    thr0[pb] = NINF;
    qn[pb] = 0;
#pragma unroll
    for (int s = 0; s < KH; ++s) {
      tv[pb][s] = NINF;
      ti[pb][s] = -1;
    }
#pragma unroll
    for (int s = 0; s < Q; ++s) {
      qv[pb][s] = NINF;
      qi[pb][s] = -1;
    }
  }
  // accumulators: [tile parity][pb]; the "previous tile" of the first one scores -inf everywhere
  floatx16 acc[2][NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    acc[0][pb] = (floatx16)(NINF);
    acc[1][pb] = (floatx16)(NINF);
  }
  bool need = false;
  int ptile = 0;
  // branch-free epilogue of a finished tile: per list, tile max -> threshold test, rej
  auto epilogue = [&](const floatx16 (&ac)[NPB]) __attribute__((always_inline)) {
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      float m = fmaxf(fmaxf(ac[pb][0], ac[pb][1]), ac[pb][2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) m = fmaxf(fmaxf(m, ac[pb][r]), ac[pb][r + 1]);
      m = fmaxf(m, ac[pb][15]);
      const float thr = tv[pb][KH - 1];
      thr0[pb] = thr;
      rej[pb] = __builtin_amdgcn_fmed3f(rej[pb], m, thr);
      need |= m > thr;
    }
  };
  // merge a full queue into the sorted list - branch-free (a rejected or empty slot inserts -inf,
  // which leaves the list as it is): no divergent blocks, so no copies of the lists at joins
  auto merge = [&](int pb) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < Q; ++s) {
      const float v = qv[pb][s];
      const bool has = s < qn[pb];
      const bool ins = has && v > tv[pb][KH - 1];
      rej[pb] = ins ? fmaxf(rej[pb], tv[pb][KH - 1]) : (has ? fmaxf(rej[pb], v) : rej[pb]);
      const float ve = ins ? v : NINF;
      const int id = qi[pb][s];
#pragma unroll
      for (int t = KH - 1; t >= 1; --t) {
        const bool ap = ve > tv[pb][t - 1];
        const bool ac = ve > tv[pb][t];
        ti[pb][t] = ap ? ti[pb][t - 1] : (ac ? id : ti[pb][t]);
        tv[pb][t] = __builtin_amdgcn_fmed3f(tv[pb][t - 1], ve, tv[pb][t]);
      }
      ti[pb][0] = ve > tv[pb][0] ? id : ti[pb][0];
      tv[pb][0] = fmaxf(tv[pb][0], ve);
    }
    qn[pb] = 0;
  };
  // queue the scores of a finished tile that beat the threshold seen by its epilogue. Compact on
  // purpose (the loop body is unrolled 4 tiles deep): one ballot per position builds the
  // wave-uniform mask of positions holding a candidate in SOME lane, and a scalar loop visits only
  // those; the score of a visited position comes out through a select chain (no indexed registers).
  // A full queue (some lane at Q) is merged into the sorted lists right away.
  auto select = [&](const floatx16 (&ac)[NPB], int tile) __attribute__((always_inline)) {
    if (__builtin_amdgcn_ballot_w64(need) == 0ull || (dbg & 1)) return;
    need = false;
    const int tbase = tile * 32 + 4 * h;
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb) {
      unsigned rmask = 0;
#pragma unroll
      for (int r = 0; r < 16; ++r) rmask |= (__builtin_amdgcn_ballot_w64(ac[pb][r] > thr0[pb]) != 0ull ? 1u : 0u) << r;
      while (rmask) {
        const int r = __builtin_ctz(rmask);
        rmask &= rmask - 1;
        float v = ac[pb][0];
#pragma unroll
        for (int q = 1; q < 16; ++q) v = r == q ? ac[pb][q] : v;
        const bool a = v > thr0[pb];
        const int id = tbase + (r & 3) + 8 * (r >> 2);
#pragma unroll
        for (int s = Q - 1; s >= 1; --s) {
          qv[pb][s] = a ? qv[pb][s - 1] : qv[pb][s];
          qi[pb][s] = a ? qi[pb][s - 1] : qi[pb][s];
        }
        qv[pb][0] = a ? v : qv[pb][0];
        qi[pb][0] = a ? id : qi[pb][0];
        qn[pb] += a ? 1 : 0;
        if (__builtin_amdgcn_ballot_w64(qn[pb] == Q) != 0ull) merge(pb);
      }
    }
  };

#ifdef HEAT_H1_STAMPS
  // measurement build only (tools/probes/h1_stamps.py): s_memtime per phase of chunks
  // [H1S_CH0, H1S_CH0 + H1S_NCH) of the waves of workgroups 0..7, into `idx` (not written then)
  constexpr int H1S_CH0 = 2000, H1S_NCH = 64, H1S_NPH = 8;
  unsigned* h1s_out = reinterpret_cast<unsigned*>(idx);
  auto stamp = [&](int ch, int ph) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned t = (unsigned)__builtin_amdgcn_s_memtime();
    if (blockIdx.x < 8 && ch >= H1S_CH0 && ch < H1S_CH0 + H1S_NCH && lane == 0)
      h1s_out[(((int)blockIdx.x * WAVES + wave) * H1S_NCH + (ch - H1S_CH0)) * H1S_NPH + ph] = t;
    __builtin_amdgcn_sched_barrier(0);
  };
#else
  auto stamp = [](int, int) {};
#endif
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem);
  const char* gimg = reinterpret_cast<const char*>(image) + lane * 16;
  const char* gv = reinterpret_cast<const char*>(meta + 4) + lane * 16;
  // this wave's DMA instructions per chunk: image pieces wave, wave + WAVES, ...; rank-1 piece
  // `wave` (1 KB = 2 tiles; a half-wave instruction for the last tile of an odd TPI)
  constexpr int VP = (TPI + 1) / 2;
  const bool vw = wave < VP;
  // the DMA of chunk ch, part tt of TPI (image pieces pc = tt, tt + TPI, ... of this wave; its
  // rank-1 piece with part 0): spread over the tiles of the chunk being computed so the issue
  // cost (tens of cycles per piece) sits in MFMA gaps instead of stalling at the chunk start
  auto issue_part = [&](int ch, int tt) __attribute__((always_inline)) {
    const unsigned dst = lds0 + (ch % NB) * BUF;
#pragma unroll
    for (int pc = tt; pc < IMGW; pc += TPI) {
      const int q = wave + WAVES * pc;
      lds_dma16(gimg + ((int64_t)ch * PIECES + q) * 2048, dst + q * 1024);
    }
    if (tt == 0 && vw && (2 * wave + 1 < TPI || lane < 32))
      lds_dma16(gv + ((int64_t)ch * TPI + 2 * wave) * 512, dst + PIECES * 1024 + 2 * wave * 512);
  };
  auto issue = [&](int ch) __attribute__((always_inline)) {
#pragma unroll
    for (int tt = 0; tt < TPI; ++tt) issue_part(ch, tt);
  };
  // the point fragments are in registers before the ring starts: otherwise the compiler's waits
  // for them land inside the loop (first use), where they would also wait for the DMA in flight
  vm_wait<0>();
#pragma unroll
  for (int c = 0; c < AHEAD; ++c)
    if (c < nch) issue(c);
  for (int ch = 0; ch < nch; ++ch) {
    __builtin_amdgcn_sched_barrier(0);
    stamp(ch, 0);
    // this wave's pieces of chunk ch have landed once at most the later chunks' are outstanding
    const int later = min(nch - 1 - ch, AHEAD - 1);
    if (GRP > 1) {
      if (ch % GRP == 0) vm_wait<0>();   // chunks ch .. ch + GRP - 1: everything outstanding
    } else if (later >= 2) {
      if (vw) vm_wait<2 * IMGW + 2>();
      else vm_wait<2 * IMGW>();
    } else if (later == 1) {
      if (vw) vm_wait<IMGW + 1>();
      else vm_wait<IMGW>();
    } else {
      vm_wait<0>();
    }
    // a raw barrier: __syncthreads() would add s_waitcnt vmcnt(0), i.e. wait for the prefetch too.
    // Past it every wave has finished chunk ch - 1, whose slot the next DMA refills.
    stamp(ch, 1);
    if (!(dbg & 2) && ch % GRP == 0) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp(ch, 2);
    const bool refill = ch + AHEAD < nch && !(dbg & 4);
    const unsigned char* buf = smem + (ch % NB) * BUF;
    // A fragments of the current tile; fragment ks is replaced by the next tile's as soon as its
    // two MFMAs are issued, so every read has about a tile of MFMA time to land
    halfx8 af[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[ks] = *reinterpret_cast<const halfx8*>(buf + ks * 1024 + lane * 16);
#pragma unroll
    for (int tt = 0; tt < TPI; ++tt) {
      const int cur = tt & 1;
      const uint2 vv = *reinterpret_cast<const uint2*>(buf + PIECES * 1024 + tt * 512 + lane * 8);
      const u32x4 aw = {vv.x, vv.y, 0u, 0u};
      const bf16x8 av = __builtin_bit_cast(bf16x8, aw);
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb) acc[cur][pb] = (floatx16)(0.f);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
          acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[ks], bhi[pb][ks], acc[cur][pb], 0, 0, 0);
        if (tt + 1 < TPI) af[ks] = *reinterpret_cast<const halfx8*>(buf + ((tt + 1) * KS + ks) * 1024 + lane * 16);
        // this tile's share of the refill DMA (ring slot of chunk ch - 1: free past the barrier)
        if (ks == (KS > 1 ? 1 : 0) && refill) issue_part(ch + AHEAD, tt);
      }
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb)
        acc[cur][pb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bsx[pb], acc[cur][pb], 0, 0, 0);
      epilogue(acc[cur ^ 1]);
#pragma unroll
      for (int i = 0; i < (KS + 1) * NPB; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // then up to 2 VALU
      }
      stamp(ch, 3 + 2 * tt);
      select(acc[cur ^ 1], ptile);
      stamp(ch, 4 + 2 * tt);
      ptile = ch * TPI + tt;
    }
  }
  // the last tile, then whatever the queues still hold
  epilogue(acc[(TPI - 1) & 1]);
  select(acc[(TPI - 1) & 1], ptile);
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb)
    if (__builtin_amdgcn_ballot_w64(qn[pb] > 0) != 0ull) merge(pb);
  // lists are in accumulator units (score / r, one r for every row): back to scores
  const float R = u[K::CB];
  const float umax = meta[2];
  const float cmax = sqrtf(2.f * umax);
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
#pragma unroll
    for (int s = 0; s < KH; ++s) tv[pb][s] *= R;
    rej[pb] *= R;
    // merge the two half lists (disjoint candidates) into the output list of KO: whatever the
    // merge lets go raises rej
    float mv[KO];
    int mi[KO];
#pragma unroll
    for (int s2 = 0; s2 < KO; ++s2) {
      mv[s2] = s2 < KH ? tv[pb][s2 < KH ? s2 : 0] : NINF;
      mi[s2] = s2 < KH ? ti[pb][s2 < KH ? s2 : 0] : -1;
    }
#pragma unroll
    for (int s2 = KO; s2 < KH; ++s2) rej[pb] = fmaxf(rej[pb], tv[pb][s2]);
    float orj = __shfl_xor(rej[pb], 32, 64);
#pragma unroll
    for (int s2 = 0; s2 < KH; ++s2) {
      const float ov = __shfl_xor(tv[pb][s2], 32, 64);
      const int oi = __shfl_xor(ti[pb][s2], 32, 64);
      if (h == 0) {
        if (ov > mv[KO - 1]) topk_insert_ev<KO>(mv, mi, ov, oi, rej[pb]);
        else orj = fmaxf(orj, ov);
      }
    }
    rej[pb] = fmaxf(rej[pb], orj);
    const float xn = sqrtf(hsq[pb] + __shfl_xor(hsq[pb], 32, 64)) * (1.f + 0x1p-10f);
    const float xs = xsq[pb] + __shfl_xor(xsq[pb], 32, 64);
    const float xc = xn * cmax;
    const float E = 1.01f * 0x1p-10f * xc + 0x1p-16f * (xc + sx[pb] * umax) + 0x1p-15f * cmax;
    // the kn-th best entry (kn is a runtime argument: a select chain, no indexed registers)
    float akn = mv[0];
    int ikn = mi[0];
#pragma unroll
    for (int s2 = 1; s2 < KO; ++s2) {
      akn = s2 == kn - 1 ? mv[s2] : akn;
      ikn = s2 == kn - 1 ? mi[s2] : ikn;
    }
    const int64_t pi = pbase + pb * 32 + j;
    if (h == 0 && pi < n) {
      const float isx = 1.f / sx[pb];
#pragma unroll
      for (int s2 = 0; s2 < KO; ++s2) {
        const bool ok = mi[s2] >= 0;
        dist[pi * KO + s2] = ok ? fmaxf(xs * isx * isx - 2.f * mv[s2] * isx, 0.f) : __builtin_huge_valf();
#ifndef HEAT_H1_STAMPS
        idx[pi * KO + s2] = mi[s2];
#endif
      }
      cert[pi] = (ikn >= 0 && rej[pb] < akn - 2.f * E) ? 1 : 0;
    }
  }
}

}  // namespace

// Rows of C padded for h1_topk: whole chunks of 2, 3 or 4 tiles (384 rows).
static inline int64_t h1_kpad(int m) { return ((int64_t)m + 383) / 384 * 384; }

// Workspace of ha_h1_topk (>= ha_h3_workspace_bytes(m, f): the same layout over 384-row padding).
HA_EXPORT int64_t ha_h1_workspace_bytes(int m, int f) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || m <= 0) return -1;
  const int64_t kpad = h1_kpad(m);
  return kpad * fpad * 2 * 2 + kpad * 8 + 16 + kpad * 16;
}

// Certified one-term k nearest rows of C (see h1_topk): dist / idx [n, kp] approximate squared
// distances ascending + int32 row indices (the caller rescores them exactly), cert [n] uint8 (1 =
// the true kn nearest are among the kp). kn <= 8 with kp = 16 or 32. workspace: ha_h1_workspace_bytes.
HA_EXPORT int ha_h1_topk(const void* planes, const float* sx, int64_t n, int f, const float* C, int m, int64_t ldc,
                         void* workspace, int kn, int kp, float* dist, int* idx, unsigned char* cert, void* stream) {
  const int fpad = h3_fpad(f);
  if (fpad < 0 || m <= 0 || kn < 1 || kn > 8 || (kp != 16 && kp != 32)) return HA_UNSUPPORTED;
  if (n <= 0) return HA_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t kpad64 = h1_kpad(m);
  if (kpad64 > (int64_t)1 << 30) return HA_UNSUPPORTED;
  const int kpad = (int)kpad64;
  _Float16* image = (_Float16*)workspace;
  float* u = (float*)((char*)workspace + (int64_t)kpad * fpad * 4);
  float* meta = u + 2 * kpad;
  const _Float16* p = (const _Float16*)planes;
  // HEAT_H1_DEBUG (measurement only, results invalid): 1 = no selection, 2 = no chunk barrier,
  // 4 = no refill DMA (the ring keeps its first chunks)
  static const int dbg = getenv("HEAT_H1_DEBUG") ? atoi(getenv("HEAT_H1_DEBUG")) : 0;
  // the error bound and the uniform scale need max |c| and max u (atomicMax into zeroed words)
  if (hipMemsetAsync(meta, 0, 16, s) != hipSuccess) return HA_LAUNCH;
  // HEAT_H1_CFG=a (A/B): one workgroup per CU of 4 waves x 64 points, 4-tile chunks
  static const bool cfg_a = getenv("HEAT_H1_CFG") && getenv("HEAT_H1_CFG")[0] == 'a';
  // HEAT_H1_CFG=w8 (A/B): one workgroup per CU of 8 waves x 32 points (half the image reads per point)
  static const bool cfg_w8 = getenv("HEAT_H1_CFG") && getenv("HEAT_H1_CFG")[0] == 'w';
  // HEAT_H1_CFG=b (A/B): one barrier per chunk instead of per pair of chunks
  static const bool cfg_b = getenv("HEAT_H1_CFG") && getenv("HEAT_H1_CFG")[0] == 'b';
  // HEAT_H1_CFG=q (A/B): one barrier per 4 chunks (8-slot ring, 73.7 KB of LDS per workgroup):
  // 368-370 vs 297 ms for the pair form on one box (knn_h1_ab_r05.jsonl)
  static const bool cfg_q = getenv("HEAT_H1_CFG") && getenv("HEAT_H1_CFG")[0] == 'q';
  // HEAT_H1_CFG=p (A/B): the f = 128 default with one barrier per pair of chunks (8-wave workgroup)
  static const bool cfg_p = getenv("HEAT_H1_CFG") && getenv("HEAT_H1_CFG")[0] == 'p';
  // HEAT_H1_CFG=o (A/B): the round-5 f = 128 form, two workgroups per CU of 4 waves x 32 points, one
  // barrier per pair of chunks
  static const bool cfg_o = getenv("HEAT_H1_CFG") && getenv("HEAT_H1_CFG")[0] == 'o';
#define HA_H1TK_LAUNCH_K(FP, KH, KO, NPB, TPI, MINB, WV, PB)                                                    \
  do {                                                                                                         \
    using KC = H3Cfg<FP, NPB>;                                                                                 \
    const size_t lds = (PB > 1 ? 2 * PB : TPI >= 3 ? 3 : 4) * ((size_t)TPI * KC::KS * 1024 + TPI * 512); /* slots */ \
    const int ppw = WV * NPB * 32;                                                                             \
    const unsigned blocks = (unsigned)((n + ppw - 1) / ppw);                                                   \
    hipFuncSetAttribute(reinterpret_cast<const void*>(h1_topk<FP, KH, KO, NPB, TPI, MINB, WV, PB>),             \
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                                  \
    hipLaunchKernelGGL((h1_topk<FP, KH, KO, NPB, TPI, MINB, WV, PB>), dim3(blocks), dim3(64 * WV), lds, s, p,   \
                       sx, n, image, u, meta, kpad / (TPI * 32), kn, dist, idx, cert, dbg);                     \
  } while (0)
#define HA_H1TK_LAUNCH_X(FP, KO, NPB, TPI, MINB, WV, PB) HA_H1TK_LAUNCH_K(FP, 16, KO, NPB, TPI, MINB, WV, PB)
#define HA_H1TK_LAUNCH(FP, KO, NPB, TPI, MINB, WV) HA_H1TK_LAUNCH_X(FP, KO, NPB, TPI, MINB, WV, 1)
#define HA_H1TK(FP)                                                                                              \
  case FP: {                                                                                                     \
    hipLaunchKernelGGL(h3_cscale<FP>, dim3(h3_cscale_grid(kpad, FP / 8)), dim3(256), 0, s, C, m, f, ldc, kpad, u,  \
                       meta, (unsigned*)(meta + 4));                                                             \
    hipLaunchKernelGGL(h3_uniform_r<FP>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m, u, meta,         \
                       (unsigned*)(meta + 4));                                                                   \
    hipLaunchKernelGGL(h3_pack_centroids<FP>, dim3((unsigned)(((int64_t)kpad * (FP / 8) + 255) / 256)),       \
                       dim3(256), 0, s, C, m, f, ldc, kpad, image, u);                                           \
    /* 2-tile chunks, one barrier per pair of chunks, chunk ch + 2 issued during ch (4-tile chunks, one */   \
    /* barrier each, 3 in flight for f = 16: whole 1 KB image pieces per wave). Measured at f = 128 */            \
    /* (tools/microbench/h1_ab.py, one box): pair 309-310 ms, per-chunk barrier (HEAT_H1_CFG=b) 313-315; */     \
    /* 3-tile chunks / 2 in flight +2%; one workgroup of 4 x 64 points per CU (HEAT_H1_CFG=a) +30%. */          \
    /* f = 128 (round 6, bench.py --workload knn, one box, knn_h1_ab_r06.jsonl): ONE workgroup per CU of */       \
    /* 8 waves x 32 points, one barrier per 4 chunks (8-slot ring, 136 KB): every staged chunk feeds 256 */        \
    /* points (half the DMA instructions and L2 reads per point) and a quarter of the barriers: 277-279 */        \
    /* vs 295-298 ms (round-5 form, HEAT_H1_CFG=o); a barrier per pair (p) 282-283. f = 64: 189-191 vs */      \
    /* 191-192 ms (f = 32 / 16 have fewer image pieces per chunk than 8 waves). 12-entry half lists */         \
    /* (fewer queued candidates) re-check 2 % of the queries instead of 0.05 %: 284 vs 279 ms */               \
    constexpr int TPB = FP >= 32 ? 2 : 4;                                                                        \
    constexpr int PAIR = TPB == 2 ? 2 : 1;                                                                       \
    if (FP == 128 && cfg_a && kp == 32) {                                                                        \
      HA_H1TK_LAUNCH(128, 32, 2, 4, 1, 4);                                                                       \
    } else if (FP == 128 && cfg_w8 && kp == 32) {                                                                \
      HA_H1TK_LAUNCH(128, 32, 1, 2, 1, 8);                                                                       \
    } else if (FP == 128 && cfg_p && kp == 32) {                                                                 \
      HA_H1TK_LAUNCH_X(128, 32, 1, 2, 1, 8, 2);                                                                  \
    } else if (FP == 128 && cfg_q && kp == 32) {                                                                 \
      HA_H1TK_LAUNCH_X(128, 32, 1, 2, 2, 4, 4);                                                                  \
    } else if (FP >= 64 && !cfg_o && !cfg_b) {                                                                   \
      if constexpr (FP >= 64) { /* 8 waves need >= 8 image pieces per chunk */                                   \
        if (kp == 32) HA_H1TK_LAUNCH_X(FP, 32, 1, 2, 1, 8, 4);                                                   \
        else HA_H1TK_LAUNCH_X(FP, 16, 1, 2, 1, 8, 4);                                                            \
      }                                                                                                          \
    } else if (cfg_b && kp == 32) {                                                                              \
      HA_H1TK_LAUNCH(FP, 32, 1, TPB, 2, 4);                                                                      \
    } else if (kp == 32) {                                                                                       \
      HA_H1TK_LAUNCH_X(FP, 32, 1, TPB, 2, 4, PAIR);                                                              \
    } else {                                                                                                     \
      HA_H1TK_LAUNCH_X(FP, 16, 1, TPB, 2, 4, PAIR);                                                              \
    }                                                                                                            \
    break;                                                                                                       \
  }
  switch (fpad) {
    HA_H1TK(16)
    HA_H1TK(32)
    HA_H1TK(64)
    HA_H1TK(128)
    default:
      return HA_UNSUPPORTED;
  }
#undef HA_H1TK
#undef HA_H1TK_LAUNCH
#undef HA_H1TK_LAUNCH_X
  return ha_launch_status();
}
