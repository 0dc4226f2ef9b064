// query.hip -- batched hot-path kernels for gfx950.
//
//  k_lf          one backward-search (LF) step per row: the loop body of
//                index.py:109-112 / fm_index.cpp:67-97, L dependent levels of
//                two 64-B rank-block reads each.
//  k_search      get_range over CSR patterns with the reference's early exit.
//  k_mask        allowed-next-token mask: the distinct symbols of BWT[lo, hi)
//                (fm_index.cpp:119-144 + index.py:161-174) scattered into a
//                (rows x vocab) bool / bit row.  Narrow ranges stream the plain
//                BWT; wide ranges OR precomputed range bitmaps and stream only
//                their two partial ends.  Each workgroup owns one vocab slice of
//                one row, so every output byte is written exactly once, coalesced.
//  k_distinct    interval_symbols with counts ([sdsl] wt_int::interval_symbols)
//                as a level-synchronous BFS of the wavelet matrix, one
//                workgroup per row, ascending symbol order.
//  k_step_raw / k_raw_multi: the scalar SWIG entry points with sdsl's unsigned
//                arithmetic (fm_index.cpp:55-97).
#include "fmidx_internal.h"

#include <algorithm>
#include <cstdlib>

namespace fmidx {

namespace {

constexpr int kLfThreads = 256;
#ifndef FMIDX_MASK_THREADS
#define FMIDX_MASK_THREADS 256
#endif
constexpr int kMaskThreads = FMIDX_MASK_THREADS;
constexpr int kMaxPlan = 160;           // >= 6 * kMaxBmLevels
constexpr uint32_t kMaxSliceTokens = 32768;
constexpr int kWinWords = kMaxSliceTokens / 32 + 12;
constexpr uint64_t kEarlyZeroWidth = 64;   // default: rows this narrow get their zeros written up front

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup
// release/acquire, which on gfx950 also drains every wave's outstanding
// global stores (s_waitcnt vmcnt(0)) -- measured as several us behind the
// early zero-fill of the mask rows.  Nothing crossing these barriers is
// global data, so only LDS (lgkmcnt) is drained.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// ------------------------------------------------------------------ LF
// 16 lanes per row (kLfThreads / 16 rows per block).
__global__ void __launch_bounds__(kLfThreads) k_lf(DevView v, const int64_t* __restrict__ tok,
                                                  int64_t shift, int64_t reset_below,
                                                  const uint64_t* lo_in, const uint64_t* hi_in,
                                                  uint64_t* lo_out, uint64_t* hi_out, uint64_t m) {
  const uint64_t i = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 4;
  const uint32_t lane16 = threadIdx.x & 15u;
  if (i >= m) return;
  const int64_t t = tok[i];
  uint64_t l = lo_in[i], h = hi_in[i];
  if (t < reset_below) {
    l = 0;
    h = v.n;
  } else {
    lf_step16(v, t + shift, l, h, lane16);
  }
  if (lane16 == 0) {
    lo_out[i] = l;
    hi_out[i] = h;
  }
}

__global__ void __launch_bounds__(kLfThreads) k_search(DevView v, const int64_t* __restrict__ tok,
                                                      const int64_t* __restrict__ off, uint64_t m,
                                                      int64_t shift, const uint64_t* lo_in,
                                                      const uint64_t* hi_in, uint64_t* lo_out,
                                                      uint64_t* hi_out) {
  const uint64_t i = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 4;
  const uint32_t lane16 = threadIdx.x & 15u;
  if (i >= m) return;
  uint64_t l = lo_in ? lo_in[i] : 0;
  uint64_t h = hi_in ? hi_in[i] : v.n;
  const int64_t a = off[i], b = off[i + 1];
  for (int64_t j = a; j < b; ++j) {
    lf_step16(v, tok[j] + shift, l, h, lane16);
    if (l == 0 && h == 0) break;       // index.py:111-112
  }
  if (lane16 == 0) {
    lo_out[i] = l;
    hi_out[i] = h;
  }
}

// [sdsl] backward_search on an inclusive range with unsigned wrap-around.
__device__ void sdsl_backward_search(const DevView& v, uint64_t c, uint64_t l, uint64_t r,
                                     uint64_t& lr, uint64_t& rr) {
  const bool unknown = c > v.max_sym || (c > 0 && v.C[c + 1] == v.C[c]);
  if (unknown) {
    lr = 1;
    rr = 0;
    return;
  }
  uint64_t pl = l > v.n ? v.n : l;
  uint64_t pr = r + 1;
  if (pr > v.n) pr = v.n;
  descend_full(v, (uint32_t)c, pl, pr);
  const int64_t d = v.D[c];
  lr = (uint64_t)((int64_t)pl + d);
  rr = (uint64_t)((int64_t)pr + d) - 1;
}

__global__ void k_step_raw(DevView v, uint64_t sym, uint64_t low, uint64_t high, uint64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (high >= v.n) high = v.n - 1;      // fm_index.cpp:74-76
  if (low > high) {                      // :77-82
    out[0] = 0;
    out[1] = 0;
    return;
  }
  uint64_t lr, rr;
  sdsl_backward_search(v, sym, low, high, lr, rr);
  if (lr > rr) {                         // :87-92
    out[0] = 0;
    out[1] = 0;
    return;
  }
  out[0] = lr;
  out[1] = rr + 1;
}

__global__ void k_raw_multi(DevView v, const uint64_t* q, uint64_t len, uint64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t l = 0, r = v.n - 1;           // fm_index.cpp:58-59
  for (uint64_t i = 0; i < len; ++i) sdsl_backward_search(v, q[i], l, r, l, r);
  out[0] = l;
  out[1] = r + 1;
}

// ------------------------------------------------------------------ mask
struct Plan {
  uint64_t a0, b0, a1, b1;   // streamed row ranges
  uint32_t nb;               // bitmaps to OR
  uint64_t off[kMaxPlan];    // word offsets of those bitmaps
};

// Canonical decomposition of [lo, hi) into two streamed partial ends plus the
// maximal aligned bitmap blocks (B0*4^j rows at level j), computed by wave 0
// with one lane per bitmap level: with a_j / b_j = x / y rounded up / down to
// level-j alignment and `top` the highest level holding a whole block, level
// j < top contributes [a_j, a_{j+1}) and [b_{j+1}, b_j), level top [a_top,
// b_top) -- the same set the greedy left-to-right cover produces (<= 6 per level).
__device__ void plan_range_wave(const DevView& v, uint64_t lo, uint64_t hi, int64_t follow, Plan& p) {
  const uint32_t lane = threadIdx.x;   // called by the 64 lanes of wave 0
  const uint32_t* one = nullptr;
  if (lo == 0 && hi == v.n && v.bm_full)
    one = v.bm_full;                                    // the whole BWT
  else if (follow >= 0 && v.bm_follow)
    one = v.bm_follow + (uint64_t)follow * v.bm_words;  // C-block of symbol `follow`
  if (one) {                                            // one precomputed bitmap
    if (lane == 0) {
      p.a0 = p.b0 = p.a1 = p.b1 = 0;
      p.nb = 1;
      p.off[0] = (uint64_t)(one - v.bm);
    }
    return;
  }
  const uint32_t lg = v.bm_log2;
  const uint64_t B0 = 1ull << lg;
  bool split = v.bm_levels > 0 && hi - lo > B0;
  uint64_t x = 0, y = 0;
  if (split) {
    x = (lo + B0 - 1) >> lg;
    y = hi >> lg;
    split = x < y;
  }
  if (lane == 0) {
    p.a0 = lo;
    p.b0 = split ? (x << lg) : hi;
    p.a1 = split ? (y << lg) : 0;
    p.b1 = split ? hi : 0;
    p.nb = 0;
  }
  if (!split) return;
  const uint32_t J = v.bm_levels;
  const uint32_t j = lane;
  uint64_t aj = 0, bj = 0, aj1 = 0, bj1 = 0;
  bool valid = false;
  if (j < J) {
    const uint64_t s0 = 1ull << (2 * j), s1 = 1ull << (2 * (j + 1));
    aj = (x + s0 - 1) & ~(s0 - 1);
    bj = y & ~(s0 - 1);
    aj1 = (x + s1 - 1) & ~(s1 - 1);
    bj1 = y & ~(s1 - 1);
    valid = aj < bj;
  }
  const uint64_t vb = __ballot(valid);
  const uint32_t top = 63u - (uint32_t)__clzll(vb);
  uint32_t cnt = 0;
  if (j < top)
    cnt = (uint32_t)(((aj1 - aj) + (bj - bj1)) >> (2 * j));
  else if (j == top)
    cnt = (uint32_t)((bj - aj) >> (2 * j));
  uint32_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += t;
  }
  const uint32_t start = incl - cnt;
  if (cnt) {
    uint64_t off = 0;
    for (uint32_t i = 0; i < j; ++i) off += (v.bm_count[0] >> (2 * i)) * (uint64_t)v.bm_words;
    const uint64_t s0 = 1ull << (2 * j);
    uint32_t k = start;
    if (j < top) {
      for (uint64_t pos = aj; pos < aj1; pos += s0) p.off[k++] = off + (pos >> (2 * j)) * v.bm_words;
      for (uint64_t pos = bj1; pos < bj; pos += s0) p.off[k++] = off + (pos >> (2 * j)) * v.bm_words;
    } else {
      for (uint64_t pos = aj; pos < bj; pos += s0) p.off[k++] = off + (pos >> (2 * j)) * v.bm_words;
    }
  }
  if (j == top) p.nb = start + cnt;
}

// The streamed parts of plan_range_wave, derivable by every thread.
__device__ __forceinline__ void stream_parts(const DevView& v, uint64_t lo, uint64_t hi, int64_t follow,
                                             uint64_t& a0, uint64_t& b0, uint64_t& a1, uint64_t& b1) {
  a0 = b0 = a1 = b1 = 0;
  if ((lo == 0 && hi == v.n && v.bm_full) || (follow >= 0 && v.bm_follow)) return;
  a0 = lo;
  b0 = hi;
  if (v.bm_levels == 0) return;
  const uint32_t lg = v.bm_log2;
  const uint64_t B0 = 1ull << lg;
  if (hi - lo <= B0) return;
  const uint64_t x = (lo + B0 - 1) >> lg, y = hi >> lg;
  if (x >= y) return;
  b0 = x << lg;
  a1 = y << lg;
  b1 = hi;
}

__device__ __forceinline__ int64_t floor_div32(int64_t x) { return x >= 0 ? x / 32 : -((-x + 31) / 32); }

__device__ __forceinline__ void set_bit(uint32_t* win, uint32_t sym, int64_t base_bit, int64_t lim) {
  const int64_t rel = (int64_t)sym - base_bit;
  if (rel >= 0 && rel < lim) atomicOr(&win[rel >> 5], 1u << (rel & 31));
}

// Streamed parts of a range: BWT[a0, b0) and BWT[a1, b1).  Each part is an
// unaligned head (< 4 symbols), a 16-B aligned middle read as uint4, and an
// unaligned tail.  The loads of the first round -- every head/tail symbol
// (threads 0..11) and kUnroll uint4 per thread of the concatenated middles --
// are all issued before any is consumed, together with the caller's first
// batch of bitmap loads, so a partial end of up to 8K symbols costs one memory
// round trip.
constexpr int kUnroll = 8;
struct StreamParts {
  uint64_t q0, n0, q1, n1;       // uint4 middles: [q0, q0+n0) and [q1, q1+n1)
  uint64_t piece[4];             // head/tail start positions
  uint32_t plen[4];              // head/tail lengths (0..3)
};

__device__ __forceinline__ void split_part(uint64_t a, uint64_t b, uint64_t& q, uint64_t& nq, uint64_t& h,
                                           uint32_t& hl, uint64_t& t, uint32_t& tl) {
  hl = tl = 0;
  q = nq = 0;
  h = t = 0;
  if (a >= b) return;
  const uint64_t a4 = (a + 3) & ~3ull, b4 = b & ~3ull;
  if (a4 >= b4) {            // fewer than one aligned uint4: up to 6 symbols as head+tail
    h = a;
    hl = (uint32_t)min((uint64_t)3, b - a);
    t = a + hl;
    tl = (uint32_t)(b - t);
    return;
  }
  h = a;
  hl = (uint32_t)(a4 - a);
  t = b4;
  tl = (uint32_t)(b - b4);
  q = a4 / 4;
  nq = (b4 - a4) / 4;
}

__device__ __forceinline__ StreamParts make_parts(uint64_t a0, uint64_t b0, uint64_t a1, uint64_t b1) {
  StreamParts p;
  split_part(a0, b0, p.q0, p.n0, p.piece[0], p.plen[0], p.piece[1], p.plen[1]);
  split_part(a1, b1, p.q1, p.n1, p.piece[2], p.plen[2], p.piece[3], p.plen[3]);
  return p;
}

__device__ __forceinline__ uint4 part_u4(const uint4* src, const StreamParts& p, uint64_t j) {
  return src[j < p.n0 ? p.q0 + j : p.q1 + (j - p.n0)];
}

__device__ __forceinline__ void set_u4(uint32_t* win, const uint4& q, int64_t base_bit, int64_t lim) {
  set_bit(win, q.x, base_bit, lim);
  set_bit(win, q.y, base_bit, lim);
  set_bit(win, q.z, base_bit, lim);
  set_bit(win, q.w, base_bit, lim);
}

__device__ void stream_symbols2(const uint32_t* __restrict__ bwt, const StreamParts& sp, int64_t base_bit,
                                int64_t lim, uint32_t* win) {
  const uint64_t ntot = sp.n0 + sp.n1;
  const uint4* src = reinterpret_cast<const uint4*>(bwt);
  uint32_t hsym = ~0u;          // head/tail symbols: threads 0..11, loaded with the first round
  if (threadIdx.x < 12) {
    const uint32_t pc = threadIdx.x / 3, k = threadIdx.x % 3;
    if (k < sp.plen[pc]) hsym = bwt[sp.piece[pc] + k];
  }
  for (uint64_t base = threadIdx.x; base < ntot; base += (uint64_t)kMaskThreads * kUnroll) {
    uint4 q[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t j = base + (uint64_t)u * kMaskThreads;
      q[u] = (j < ntot) ? part_u4(src, sp, j) : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      if (q[u].x != ~0u) set_u4(win, q[u], base_bit, lim);
  }
  if (hsym != ~0u) set_bit(win, hsym, base_bit, lim);
}

// blockIdx -> (row, slice).  Blocks b and b+8 share an XCD under round-robin
// dispatch, so the S slices of a row are given blockIdx values congruent mod 8:
// their redundant reads of the row's rank blocks / BWT / bitmaps share one L2.
// Speed only; any placement is correct.
__device__ __forceinline__ void map_block(uint32_t b, uint32_t S, uint64_t& row, uint32_t& slice) {
  const uint32_t per = 8u * S;
  const uint32_t r = b % per;
  row = (uint64_t)(b / per) * 8 + (r & 7u);
  slice = r >> 3;
}

// One workgroup = one vocab slice of one row.  With DO_LF the row's LF step
// (or restart) is computed first by thread 0 (redundantly per slice; slice 0
// publishes the new state), otherwise [lo_in, hi_in) is the range to mask.
template <bool PACKED, bool DO_LF>
__global__ void __launch_bounds__(kMaskThreads) k_decode(DevView v, const int64_t* __restrict__ tok,
                                                        int64_t shift, int64_t reset_below,
                                                        const uint64_t* __restrict__ lo_in,
                                                        const uint64_t* __restrict__ hi_in,
                                                        uint64_t* __restrict__ lo_out,
                                                        uint64_t* __restrict__ hi_out, uint64_t m,
                                                        uint8_t* __restrict__ mask, uint64_t ld,
                                                        uint64_t vocab, uint32_t S, uint32_t SW,
                                                        uint64_t early_width) {
  __shared__ Plan plan;
  __shared__ uint64_t s_lohi[2];
  __shared__ int64_t s_follow;
  __shared__ __attribute__((aligned(16))) uint32_t win[kWinWords];
  FM_STAMP(v, 0);
  // Materialise every kernel-argument field used later now, so their scalar
  // loads issue together at entry instead of one cache-missing round trip
  // per first use deep inside the dependent chain.
  asm volatile("" ::"s"(v.n), "s"(v.nblk), "s"(v.nsb), "s"(v.wm), "s"(v.sb), "s"(v.Z), "s"(v.D), "s"(v.C));
  asm volatile("" ::"s"(v.bwt), "s"(v.bm), "s"(v.bm_full), "s"(v.bm_follow), "s"(v.bm_count[0]),
               "s"(v.L), "s"(v.NL), "s"(v.max_sym), "s"(v.bm_words), "s"(v.bm_levels), "s"(v.bm_log2));
  uint64_t row;
  uint32_t slice;
  map_block(blockIdx.x, S, row, slice);
  if (row >= m) return;
  const uint64_t t0 = (uint64_t)slice * SW;
  if (t0 >= vocab) return;
  const uint64_t t1 = min(vocab, t0 + SW);
  // Rows whose incoming range is narrow stay narrow after the LF step (it
  // can only shrink a range), so their slice is zero-filled right away --
  // the stores overlap the LF chain -- and the final pass rewrites only the
  // chunks holding an allowed token.  Each 32-token chunk is owned by the same
  // thread in both passes, so program order keeps the final value.
  uint8_t* out_row = mask + row * ld;
  const uint64_t ntok = t1 - t0;
  bool early_zero;
  {
    const uint64_t l0 = lo_in[row], h0 = min(hi_in[row], v.n);
    const bool reset = DO_LF && tok[row] < reset_below;
    early_zero = !reset && (l0 >= h0 || h0 - l0 <= early_width);
  }
  FM_STAMP(v, 1);
  // Zero-fill by waves 1.. only: loads and stores share vmcnt in issue order,
  // so a wave with stores in flight cannot wait on a load without also
  // waiting for them -- wave 0 (LF + plan) must stay store-free.
  if (early_zero && threadIdx.x >= 64) {
    for (uint64_t k = threadIdx.x - 64; k * 32 < ntok; k += kMaskThreads - 64) {
      const uint64_t t = t0 + k * 32;
      const uint64_t cnt = min((uint64_t)32, t1 - t);
      if (PACKED) {
        reinterpret_cast<uint32_t*>(out_row)[t / 32] = 0u;
      } else {
        uint8_t* dst = out_row + t;
        if (cnt == 32 && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
          reinterpret_cast<uint4*>(dst)[0] = make_uint4(0, 0, 0, 0);
          reinterpret_cast<uint4*>(dst)[1] = make_uint4(0, 0, 0, 0);
        } else {
          for (uint64_t j = 0; j < cnt; ++j) dst[j] = 0;
        }
      }
    }
  }
  FM_STAMP(v, 2);
  // Wave 0: the LF step (lanes 0-15), then the bitmap plan of the new range
  // (all 64 lanes), published with the range by a single barrier.
  if (threadIdx.x < 64) {
    uint64_t l = 0, h = 0;
    int64_t follow = -1;
    if (threadIdx.x < 16) {
      l = lo_in[row];
      h = hi_in[row];
      if (DO_LF) {
        const int64_t t = tok[row];
        if (t < reset_below) {
          l = 0;
          h = v.n;
        } else {
          // from the full range the LF step lands on symbol c's C-block, whose
          // allowed set is c's precomputed follow-set bitmap
          if (l == 0 && h >= v.n) follow = t + shift;
          lf_step16(v, t + shift, l, h, threadIdx.x);
          if (l >= h) follow = -1;
        }
        if (slice == 0 && threadIdx.x == 0) {
          lo_out[row] = l;
          hi_out[row] = h;
        }
      }
    }
    l = __shfl(l, 0, 64);
    h = __shfl(h, 0, 64);
    follow = __shfl(follow, 0, 64);
    if (h > v.n) h = v.n;
    if (threadIdx.x == 0) {
      s_lohi[0] = l;
      s_lohi[1] = h;
      s_follow = follow;
    }
    if (l < h) plan_range_wave(v, l, h, follow, plan);
  }
  // LDS window over symbol space, 128-bit aligned: words [w_lo, w_lo + nwin)
  const int64_t w_lo = floor_div32((int64_t)t0 + shift) & ~(int64_t)3;
  const int64_t sym_end = (int64_t)t1 + shift + 64;
  const uint32_t nwin = (uint32_t)(((sym_end - w_lo * 32 + 31) / 32 + 3) & ~3ll);
  for (uint32_t w = threadIdx.x; w < nwin; w += kMaskThreads) win[w] = 0;
  lds_barrier();
  const uint64_t lo = s_lohi[0], hi = s_lohi[1];
  const bool live = lo < hi;
  FM_STAMP(v, 3);
  if (live) {
    // streamed partial ends, then bitmap ORs; one barrier after
    const int64_t base_bit = w_lo * 32;
    const int64_t lim = (int64_t)nwin * 32;
    uint64_t a0, b0, a1, b1;
    stream_parts(v, lo, hi, s_follow, a0, b0, a1, b1);
    stream_symbols2(v.bwt, make_parts(a0, b0, a1, b1), base_bit, lim, win);
    FM_STAMP(v, 4);
    const uint32_t nb = plan.nb;
    if (nb) {
      // G thread groups split the bitmaps, each thread owns one uint4 of the
      // window; partial ORs merge with LDS atomics.
      const uint32_t nw4 = nwin / 4;
      const uint32_t G = max(1u, (uint32_t)kMaskThreads / nw4);
      const uint32_t g = threadIdx.x / nw4;
      for (uint32_t w4b = threadIdx.x % nw4; g < G && w4b < nw4; w4b += kMaskThreads) {
        const int64_t gwb = w_lo + 4 * (int64_t)w4b;
        if (!(gwb >= 0 && gwb + 4 <= (int64_t)v.bm_words)) continue;
        uint4 acc = make_uint4(0, 0, 0, 0);
        for (uint32_t q = g; q < nb; q += G * 8) {
          uint4 x[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const uint32_t qq = q + (uint32_t)u * G;
            x[u] = qq < nb ? *reinterpret_cast<const uint4*>(v.bm + plan.off[qq] + gwb) : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            acc.x |= x[u].x;
            acc.y |= x[u].y;
            acc.z |= x[u].z;
            acc.w |= x[u].w;
          }
        }
        if (acc.x) atomicOr(&win[4 * w4b + 0], acc.x);
        if (acc.y) atomicOr(&win[4 * w4b + 1], acc.y);
        if (acc.z) atomicOr(&win[4 * w4b + 2], acc.z);
        if (acc.w) atomicOr(&win[4 * w4b + 3], acc.w);
      }
    }
    FM_STAMP(v, 5);
    lds_barrier();
  }
  FM_STAMP(v, 6);
  // the final stores to an early-zeroed chunk must land after its zero store
  // (same thread, same address): drain this wave's outstanding stores first
  if (early_zero) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // emit: 32 tokens per thread per iteration (early-zeroed rows: by the same
  // thread that zeroed the chunk)
  const int64_t rel0 = (int64_t)t0 + shift - w_lo * 32;   // >= 0
  const uint32_t e_first = early_zero ? 64u : 0u;
  if (threadIdx.x >= e_first)
  for (uint64_t k = threadIdx.x - e_first; k * 32 < ntok; k += kMaskThreads - e_first) {
    const int64_t rel = rel0 + (int64_t)k * 32;
    const uint32_t wi = (uint32_t)(rel >> 5);
    const uint32_t o = (uint32_t)(rel & 31);
    uint32_t bits = o ? ((win[wi] >> o) | (win[wi + 1] << (32 - o))) : win[wi];
    const uint64_t t = t0 + k * 32;
    const uint64_t cnt = min((uint64_t)32, t1 - t);
    if (cnt < 32) bits &= (1u << cnt) - 1u;
    if (early_zero && bits == 0) continue;
    if (PACKED) {
      reinterpret_cast<uint32_t*>(out_row)[t / 32] = bits;   // t is a multiple of 32
    } else {
      uint8_t* dst = out_row + t;
      if (cnt == 32 && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
        uint32_t q[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = (((bits >> (4 * j)) & 0xFu) * 0x204081u) & 0x01010101u;
        reinterpret_cast<uint4*>(dst)[0] = make_uint4(q[0], q[1], q[2], q[3]);
        reinterpret_cast<uint4*>(dst)[1] = make_uint4(q[4], q[5], q[6], q[7]);
      } else {
        for (uint64_t j = 0; j < cnt; ++j) dst[j] = (uint8_t)((bits >> j) & 1u);
      }
    }
  }
  FM_STAMP(v, 7);
}

// ------------------------------------------------------------------ distinct
struct Frontier {
  uint64_t* lo[2];
  uint64_t* hi[2];
  uint32_t* pre[2];
};

// per-digit counts before position i at level lev (16 values, one thread)
__device__ __forceinline__ void digit_counts(const DevView& v, uint32_t lev, uint64_t i, uint64_t* out) {
  const uint64_t b = i / kBlkDigits;
  const uint32_t k = (uint32_t)(i - b * kBlkDigits);
  const uint4* blk = rank_block(v, lev, b);
  const uint64_t* sbr = sb_row(v, lev, b);
  uint4 x[kBlkU4];
#pragma unroll
  for (int q = 0; q < kBlkU4; ++q) x[q] = blk[q];
#pragma unroll
  for (uint32_t d = 0; d < 16; ++d) {
    uint64_t c = sbr[d];
#pragma unroll
    for (uint32_t q = 0; q < kBlkU4; ++q) c += block_part(x[q], q, d, k);
    out[d] = c;
  }
}

__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t* lds /*[4]*/, uint32_t& total) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) lds[wave] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t t = lds[w];
    if ((uint32_t)w < wave) base += t;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}

// interval_symbols with counts: level-synchronous BFS over the 16-ary
// wavelet matrix, one workgroup per row; children are appended in digit
// order so the final frontier is in ascending symbol order.
__global__ void __launch_bounds__(256) k_distinct(DevView v, const uint64_t* __restrict__ lo_a,
                                                 const uint64_t* __restrict__ hi_a, uint64_t m,
                                                 const uint64_t* __restrict__ cap_off,
                                                 uint64_t* __restrict__ syms,
                                                 uint64_t* __restrict__ counts,
                                                 uint64_t* __restrict__ k_out, Frontier fr) {
  __shared__ uint32_t wave_tot[4];
  const uint64_t row = blockIdx.x;
  if (row >= m) return;
  uint64_t lo = lo_a[row], hi = hi_a[row];
  const uint64_t base = cap_off[row];
  const uint64_t cap = cap_off[row + 1] - base;
  // fm_index.cpp:127-133
  bool empty = (lo == hi);
  if (hi > v.n) hi = v.n;
  if (lo >= hi) empty = true;
  if (empty || cap == 0) {
    if (threadIdx.x == 0) k_out[row] = empty ? 0 : ~0ull;
    return;
  }
  uint64_t* alo = fr.lo[0] + base;
  uint64_t* ahi = fr.hi[0] + base;
  uint32_t* apre = fr.pre[0] + base;
  uint64_t* blo = fr.lo[1] + base;
  uint64_t* bhi = fr.hi[1] + base;
  uint32_t* bpre = fr.pre[1] + base;
  if (threadIdx.x == 0) {
    alo[0] = lo;
    ahi[0] = hi;
    apre[0] = 0;
  }
  __syncthreads();
  uint64_t fc = 1;
  bool overflow = false;
  for (uint32_t lev = 0; lev < v.NL; ++lev) {
    const uint64_t* Z = v.Z + lev * kRadix;
    uint64_t out = 0;
    for (uint64_t t0 = 0; t0 < fc; t0 += 256) {
      const uint64_t i = t0 + threadIdx.x;
      uint64_t cl[16], ch[16];
      uint32_t p = 0, nchild = 0;
      if (i < fc) {
        p = apre[i];
        digit_counts(v, lev, alo[i], cl);
        digit_counts(v, lev, ahi[i], ch);
#pragma unroll
        for (int d = 0; d < 16; ++d) nchild += (ch[d] > cl[d]) ? 1u : 0u;
      }
      uint32_t tot;
      const uint64_t pos0 = out + block_scan_u32(nchild, wave_tot, tot);
      if (nchild) {
        uint64_t pos = pos0;
#pragma unroll
        for (uint32_t d = 0; d < 16; ++d) {
          if (ch[d] > cl[d]) {
            if (pos < cap) {
              blo[pos] = Z[d] + cl[d];
              bhi[pos] = Z[d] + ch[d];
              bpre[pos] = (p << 4) | d;
            }
            ++pos;
          }
        }
      }
      out += tot;
    }
    __syncthreads();
    if (out > cap) {
      overflow = true;
      break;
    }
    fc = out;
    uint64_t* t;
    uint32_t* tp;
    t = alo; alo = blo; blo = t;
    t = ahi; ahi = bhi; bhi = t;
    tp = apre; apre = bpre; bpre = tp;
  }
  if (overflow) {
    if (threadIdx.x == 0) k_out[row] = ~0ull;
    return;
  }
  for (uint64_t i = threadIdx.x; i < fc; i += 256) {
    syms[base + i] = apre[i];
    counts[base + i] = ahi[i] - alo[i];
  }
  if (threadIdx.x == 0) k_out[row] = fc;
}

uint32_t env_u32(const char* name, uint32_t dflt) {
  const char* s = std::getenv(name);
  if (!s || !*s) return dflt;
  return (uint32_t)std::strtoul(s, nullptr, 10);
}

}  // namespace

// ------------------------------------------------------------------ launchers
int launch_lf_step(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                   const uint64_t* lo, const uint64_t* hi, uint64_t* lo_out, uint64_t* hi_out,
                   uint64_t m, hipStream_t s) {
  if (m == 0) return 0;
  const unsigned g = (unsigned)((m * 16 + kLfThreads - 1) / kLfThreads);
  k_lf<<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_search(const DevView& v, const int64_t* tok, const int64_t* off, uint64_t m,
                  int64_t shift, const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out,
                  uint64_t* hi_out, hipStream_t s) {
  if (m == 0) return 0;
  const unsigned g = (unsigned)((m * 16 + kLfThreads - 1) / kLfThreads);
  k_search<<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_step_raw(const DevView& v, uint64_t sym, uint64_t low, uint64_t high, uint64_t* out2,
                    hipStream_t s) {
  k_step_raw<<<1, 64, 0, s>>>(v, sym, low, high, out2);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_raw_multi(const DevView& v, const uint64_t* q, uint64_t len, uint64_t* out2,
                     hipStream_t s) {
  k_raw_multi<<<1, 64, 0, s>>>(v, q, len, out2);
  FM_HIP(hipGetLastError());
  return 0;
}

// Slice geometry.  Measured on MI355X (tools/sweep_stamps.sh): this kernel
// keeps at most ~16 waves resident per CU, and a launch of more waves than
// that (4096 over 256 CUs) dispatches its tail only as earlier workgroups
// retire -- a ~1 workgroup-lifetime stall.  So the slices per row are chosen
// to keep rows * S * (threads / 64) within that budget, slices a multiple of
// 32 tokens, at most kMaxSliceTokens.
static void mask_geometry(uint64_t m, uint64_t vocab, uint32_t& S, uint32_t& SW) {
  uint32_t sw = env_u32("FMIDX_MASK_SW", 0);
  if (sw == 0) {
    const uint64_t rows = (m + 7) / 8 * 8;
    const uint64_t waves_per_wg = kMaskThreads / 64;
    const uint64_t budget = env_u32("FMIDX_WAVE_BUDGET", 4096);
    const uint64_t want = std::max<uint64_t>(1, budget / (rows * waves_per_wg));
    const uint64_t max_s = std::max<uint64_t>(1, (vocab + 1023) / 1024);
    const uint64_t s = std::min(want, max_s);
    sw = (uint32_t)((vocab + s - 1) / s);
  }
  sw = (sw + 31) & ~31u;
  if (sw > kMaxSliceTokens) sw = kMaxSliceTokens;
  if (sw < 32) sw = 32;
  SW = sw;
  S = (uint32_t)((vocab + sw - 1) / sw);
}

static int launch_decode_kernel(const DevView& v, const int64_t* tok, int64_t shift,
                                int64_t reset_below, const uint64_t* lo_in, const uint64_t* hi_in,
                                uint64_t* lo_out, uint64_t* hi_out, uint64_t m, uint8_t* mask,
                                uint64_t ld, uint64_t vocab, int64_t mshift, int packed, bool do_lf,
                                hipStream_t s) {
  if (packed && (ld % 4 != 0 || ld < 4 * ((vocab + 31) / 32) ||
                 (reinterpret_cast<uintptr_t>(mask) & 3))) {
    set_error("packed mask needs 4-byte aligned rows with ld >= 4*ceil(vocab/32)");
    return -1;
  }
  if (!packed && ld < vocab) {
    set_error("mask leading dimension %llu < vocab %llu", (unsigned long long)ld,
              (unsigned long long)vocab);
    return -1;
  }
  uint32_t S, SW;
  mask_geometry(m, vocab, S, SW);
  const uint64_t grid = (m + 7) / 8 * 8 * S;
  if (grid > 0x7fffffffull) {
    set_error("too many rows for one launch");
    return -1;
  }
  const unsigned g = (unsigned)grid;
  (void)mshift;
  static const uint64_t ew = [] {
    const char* e = std::getenv("FMIDX_EARLY_ZERO_WIDTH");
    return (e && *e) ? (uint64_t)std::strtoull(e, nullptr, 10) : kEarlyZeroWidth;
  }();
  if (do_lf) {
    if (packed)
      k_decode<true, true><<<g, kMaskThreads, 0, s>>>(v, tok, shift, reset_below, lo_in, hi_in, lo_out, hi_out,
                                                      m, mask, ld, vocab, S, SW, ew);
    else
      k_decode<false, true><<<g, kMaskThreads, 0, s>>>(v, tok, shift, reset_below, lo_in, hi_in, lo_out, hi_out,
                                                       m, mask, ld, vocab, S, SW, ew);
  } else {
    if (packed)
      k_decode<true, false><<<g, kMaskThreads, 0, s>>>(v, tok, shift, reset_below, lo_in, hi_in, lo_out, hi_out,
                                                       m, mask, ld, vocab, S, SW, ew);
    else
      k_decode<false, false><<<g, kMaskThreads, 0, s>>>(v, tok, shift, reset_below, lo_in, hi_in, lo_out,
                                                        hi_out, m, mask, ld, vocab, S, SW, ew);
  }
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_mask(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                uint8_t* mask, uint64_t ld, uint64_t vocab, int64_t shift, int packed,
                hipStream_t s) {
  if (m == 0 || vocab == 0) return 0;
  return launch_decode_kernel(v, nullptr, shift, 0, lo, hi, nullptr, nullptr, m, mask, ld, vocab, shift,
                              packed, false, s);
}

// Follow-set bitmaps: row c = packed mask (symbol space, shift 0) of the
// C-block [C[c], C[c+1]) -- exactly the bitmap layout plan_range_wave reads.
int launch_follow_bitmaps(const DevView& v, const uint64_t* C, uint64_t nsym, uint32_t* out,
                          hipStream_t s) {
  const uint64_t ld = (uint64_t)v.bm_words * 4;
  const uint64_t chunk = 32768;   // rows per launch
  for (uint64_t c0 = 0; c0 < nsym; c0 += chunk) {
    const uint64_t m = std::min(chunk, nsym - c0);
    if (launch_decode_kernel(v, nullptr, 0, 0, C + c0, C + c0 + 1, nullptr, nullptr, m,
                             reinterpret_cast<uint8_t*>(out + c0 * v.bm_words), ld,
                             (uint64_t)v.bm_words * 32, 0, 1, false, s))
      return -1;
  }
  return 0;
}

int launch_decode(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                  const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out, uint64_t* hi_out,
                  uint64_t m, uint8_t* mask, uint64_t ld, uint64_t vocab, int packed, hipStream_t s) {
  if (m == 0) return 0;
  if (vocab == 0)   // LF only: the per-row kernel is safe in place
    return launch_lf_step(v, tok, shift, reset_below, lo_in, hi_in, lo_out, hi_out, m, s);
  if (lo_in == lo_out || hi_in == hi_out) {
    set_error("fused decode step: state in/out buffers must not alias (ping-pong them)");
    return -1;
  }
  return launch_decode_kernel(v, tok, shift, reset_below, lo_in, hi_in, lo_out, hi_out, m, mask, ld, vocab,
                              shift, packed, true, s);
}

size_t distinct_ws_bytes(uint64_t total_cap) { return (size_t)total_cap * 40 + 256; }

int launch_distinct(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                    const uint64_t* cap_off, uint64_t* syms, uint64_t* counts, uint64_t* k,
                    void* ws, uint64_t total_cap, hipStream_t s) {
  if (m == 0) return 0;
  Frontier fr;
  char* p = reinterpret_cast<char*>(ws);
  const uint64_t T = total_cap ? total_cap : 1;
  fr.lo[0] = reinterpret_cast<uint64_t*>(p);
  fr.hi[0] = fr.lo[0] + T;
  fr.lo[1] = fr.hi[0] + T;
  fr.hi[1] = fr.lo[1] + T;
  fr.pre[0] = reinterpret_cast<uint32_t*>(fr.hi[1] + T);
  fr.pre[1] = fr.pre[0] + T;
  k_distinct<<<(unsigned)m, 256, 0, s>>>(v, lo, hi, m, cap_off, syms, counts, k, fr);
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
