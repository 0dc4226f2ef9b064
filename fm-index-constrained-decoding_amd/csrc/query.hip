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

constexpr int kLfThreads = 64;
constexpr int kMaskThreads = 256;
constexpr int kMaxPlan = 160;           // >= 6 * kMaxBmLevels
constexpr uint32_t kMaxSliceTokens = 32768;
constexpr int kWinWords = kMaxSliceTokens / 32 + 12;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// ------------------------------------------------------------------ LF
__global__ void __launch_bounds__(kLfThreads) k_lf(DevView v, const int64_t* __restrict__ tok,
                                                  int64_t shift, int64_t reset_below,
                                                  const uint64_t* lo_in, const uint64_t* hi_in,
                                                  uint64_t* lo_out, uint64_t* hi_out, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * kLfThreads + threadIdx.x;
  if (i >= m) return;
  const int64_t t = tok[i];
  uint64_t l = lo_in[i], h = hi_in[i];
  if (t < reset_below) {
    l = 0;
    h = v.n;
  } else {
    lf_step(v, t + shift, l, h);
  }
  lo_out[i] = l;
  hi_out[i] = h;
}

__global__ void __launch_bounds__(kLfThreads) k_search(DevView v, const int64_t* __restrict__ tok,
                                                      const int64_t* __restrict__ off, uint64_t m,
                                                      int64_t shift, const uint64_t* lo_in,
                                                      const uint64_t* hi_in, uint64_t* lo_out,
                                                      uint64_t* hi_out) {
  const uint64_t i = (uint64_t)blockIdx.x * kLfThreads + threadIdx.x;
  if (i >= m) return;
  uint64_t l = lo_in ? lo_in[i] : 0;
  uint64_t h = hi_in ? hi_in[i] : v.n;
  const int64_t a = off[i], b = off[i + 1];
  for (int64_t j = a; j < b; ++j) {
    lf_step(v, tok[j] + shift, l, h);
    if (l == 0 && h == 0) break;       // index.py:111-112
  }
  lo_out[i] = l;
  hi_out[i] = h;
}

// Full L-level descent of both endpoints (no early exit), positions <= n.
__device__ void descend_full(const DevView& v, uint32_t c, uint64_t& l, uint64_t& r) {
  for (uint32_t lev = 0; lev < v.L; ++lev) {
    const uint64_t r1l = rank1(v, lev, l);
    const uint64_t r1r = rank1(v, lev, r);
    if ((c >> (v.L - 1 - lev)) & 1u) {
      l = v.zeros[lev] + r1l;
      r = v.zeros[lev] + r1r;
    } else {
      l -= r1l;
      r -= r1r;
    }
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

// Canonical decomposition of [lo, hi): two streamed partial ends plus aligned
// bitmap blocks of size B0*4^j, largest first.
__device__ void plan_range(const DevView& v, uint64_t lo, uint64_t hi, Plan& p) {
  p.a0 = lo;
  p.b0 = hi;
  p.a1 = p.b1 = 0;
  p.nb = 0;
  if (v.bm_levels == 0) return;
  const uint32_t lg = v.bm_log2;
  const uint64_t B0 = 1ull << lg;
  if (hi - lo <= B0) return;
  uint64_t x = (lo + B0 - 1) >> lg;
  const uint64_t y = hi >> lg;
  if (x >= y) return;
  p.b0 = x << lg;
  p.a1 = y << lg;
  p.b1 = hi;
  while (x < y && p.nb < (uint32_t)kMaxPlan) {
    uint32_t j = 0;
    while (j + 1 < v.bm_levels) {
      const uint64_t span = 1ull << (2 * (j + 1));
      if ((x & (span - 1)) != 0 || x + span > y) break;
      ++j;
    }
    p.off[p.nb++] = v.bm_off[j] + (x >> (2 * j)) * (uint64_t)v.bm_words;
    x += 1ull << (2 * j);
  }
}

__device__ __forceinline__ int64_t floor_div32(int64_t x) { return x >= 0 ? x / 32 : -((-x + 31) / 32); }

__device__ __forceinline__ void set_bit(uint32_t* win, uint32_t sym, int64_t base_bit, int64_t lim) {
  const int64_t rel = (int64_t)sym - base_bit;
  if (rel >= 0 && rel < lim) atomicOr(&win[rel >> 5], 1u << (rel & 31));
}

// OR the symbols of BWT[a, b) into the LDS window.  The 16-B aligned middle is
// read as uint4 with kUnroll loads in flight per thread before any LDS atomic.
constexpr int kUnroll = 4;
__device__ void stream_symbols(const uint32_t* __restrict__ bwt, uint64_t a, uint64_t b, int64_t base_bit,
                               int64_t lim, uint32_t* win) {
  const uint64_t a4 = (a + 3) & ~3ull;
  const uint64_t b4 = b & ~3ull;
  if (a4 >= b4) {
    for (uint64_t i = a + threadIdx.x; i < b; i += kMaskThreads) set_bit(win, bwt[i], base_bit, lim);
    return;
  }
  if (threadIdx.x < a4 - a) set_bit(win, bwt[a + threadIdx.x], base_bit, lim);
  if (threadIdx.x < b - b4) set_bit(win, bwt[b4 + threadIdx.x], base_bit, lim);
  const uint4* src = reinterpret_cast<const uint4*>(bwt);
  const uint64_t q0 = a4 / 4, q1 = b4 / 4;
  for (uint64_t base = q0 + threadIdx.x; base < q1; base += (uint64_t)kMaskThreads * kUnroll) {
    uint4 q[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t j = base + (uint64_t)u * kMaskThreads;
      q[u] = (j < q1) ? src[j] : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (q[u].x == ~0u) continue;
      set_bit(win, q[u].x, base_bit, lim);
      set_bit(win, q[u].y, base_bit, lim);
      set_bit(win, q[u].z, base_bit, lim);
      set_bit(win, q[u].w, base_bit, lim);
    }
  }
}

template <bool PACKED>
__global__ void __launch_bounds__(kMaskThreads) k_mask(DevView v, const uint64_t* __restrict__ lo_a,
                                                      const uint64_t* __restrict__ hi_a, uint64_t m,
                                                      uint8_t* __restrict__ mask, uint64_t ld,
                                                      uint64_t vocab, int64_t shift, uint32_t S,
                                                      uint32_t SW) {
  __shared__ Plan plan;
  __shared__ __attribute__((aligned(16))) uint32_t win[kWinWords];
  const uint64_t row = blockIdx.x / S;
  const uint32_t slice = blockIdx.x % S;
  if (row >= m) return;
  const uint64_t t0 = (uint64_t)slice * SW;
  if (t0 >= vocab) return;
  const uint64_t t1 = min(vocab, t0 + SW);
  // LDS window over symbol space, 128-bit aligned: words [w_lo, w_lo + nwin)
  const int64_t w_lo = floor_div32((int64_t)t0 + shift) & ~(int64_t)3;
  const int64_t sym_end = (int64_t)t1 + shift + 64;
  const uint32_t nwin = (uint32_t)(((sym_end - w_lo * 32 + 31) / 32 + 3) & ~3ll);
  for (uint32_t w = threadIdx.x; w < nwin; w += kMaskThreads) win[w] = 0;
  uint64_t lo = lo_a[row];
  uint64_t hi = hi_a[row];
  if (hi > v.n) hi = v.n;
  const bool live = lo < hi;
  if (live && threadIdx.x == 0) plan_range(v, lo, hi, plan);
  __syncthreads();
  if (live) {
    const int64_t base_bit = w_lo * 32;
    const int64_t lim = (int64_t)nwin * 32;
    for (int part = 0; part < 2; ++part) {
      const uint64_t a = part ? plan.a1 : plan.a0;
      const uint64_t b = part ? plan.b1 : plan.b0;
      if (a >= b) continue;
      stream_symbols(v.bwt, a, b, base_bit, lim, win);
    }
    __syncthreads();
    const uint32_t nb = plan.nb;
    if (nb) {
      uint4* win4 = reinterpret_cast<uint4*>(win);
      for (uint32_t w4 = threadIdx.x; w4 < nwin / 4; w4 += kMaskThreads) {
        const int64_t gw = w_lo + 4 * (int64_t)w4;
        if (gw < 0 || gw + 4 > (int64_t)v.bm_words) continue;
        uint4 acc = win4[w4];
        uint32_t q = 0;
        for (; q + 4 <= nb; q += 4) {
          const uint4 x0 = *reinterpret_cast<const uint4*>(v.bm + plan.off[q + 0] + gw);
          const uint4 x1 = *reinterpret_cast<const uint4*>(v.bm + plan.off[q + 1] + gw);
          const uint4 x2 = *reinterpret_cast<const uint4*>(v.bm + plan.off[q + 2] + gw);
          const uint4 x3 = *reinterpret_cast<const uint4*>(v.bm + plan.off[q + 3] + gw);
          acc.x |= x0.x | x1.x | x2.x | x3.x;
          acc.y |= x0.y | x1.y | x2.y | x3.y;
          acc.z |= x0.z | x1.z | x2.z | x3.z;
          acc.w |= x0.w | x1.w | x2.w | x3.w;
        }
        for (; q < nb; ++q) {
          const uint4 x0 = *reinterpret_cast<const uint4*>(v.bm + plan.off[q] + gw);
          acc.x |= x0.x;
          acc.y |= x0.y;
          acc.z |= x0.z;
          acc.w |= x0.w;
        }
        win4[w4] = acc;
      }
    }
    __syncthreads();
  }
  // emit: 32 tokens per thread per iteration
  uint8_t* out_row = mask + row * ld;
  const uint64_t ntok = t1 - t0;
  const int64_t rel0 = (int64_t)t0 + shift - w_lo * 32;   // >= 0
  for (uint64_t k = threadIdx.x; k * 32 < ntok; k += kMaskThreads) {
    const int64_t rel = rel0 + (int64_t)k * 32;
    const uint32_t wi = (uint32_t)(rel >> 5);
    const uint32_t o = (uint32_t)(rel & 31);
    uint32_t bits = o ? ((win[wi] >> o) | (win[wi + 1] << (32 - o))) : win[wi];
    const uint64_t t = t0 + k * 32;
    const uint64_t cnt = min((uint64_t)32, t1 - t);
    if (cnt < 32) bits &= (1u << cnt) - 1u;
    if (PACKED) {
      // t is a multiple of 32 -> whole uint32 word
      reinterpret_cast<uint32_t*>(out_row)[t / 32] = bits;
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
}

// ------------------------------------------------------------------ distinct
struct Frontier {
  uint64_t* lo[2];
  uint64_t* hi[2];
  uint32_t* pre[2];
};

__global__ void __launch_bounds__(256) k_distinct(DevView v, const uint64_t* __restrict__ lo_a,
                                                 const uint64_t* __restrict__ hi_a, uint64_t m,
                                                 const uint64_t* __restrict__ cap_off,
                                                 uint64_t* __restrict__ syms,
                                                 uint64_t* __restrict__ counts,
                                                 uint64_t* __restrict__ k_out, Frontier fr) {
  __shared__ uint32_t wave_cnt[4];
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
  const uint32_t lane = lane_id();
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint64_t fc = 1;
  bool overflow = false;
  for (uint32_t lev = 0; lev < v.L; ++lev) {
    const uint64_t z = v.zeros[lev];
    uint64_t out = 0;
    for (uint64_t t0 = 0; t0 < fc; t0 += 256) {
      const uint64_t i = t0 + threadIdx.x;
      bool h0 = false, h1 = false;
      uint64_t z0 = 0, z1 = 0, o0 = 0, o1 = 0;
      uint32_t p = 0;
      if (i < fc) {
        const uint64_t l = alo[i], h = ahi[i];
        p = apre[i];
        const uint64_t r1l = rank1(v, lev, l);
        const uint64_t r1h = rank1(v, lev, h);
        z0 = l - r1l;
        z1 = h - r1h;
        o0 = z + r1l;
        o1 = z + r1h;
        h0 = z0 < z1;
        h1 = o0 < o1;
      }
      const uint64_t b0 = __ballot(h0);
      const uint64_t b1 = __ballot(h1);
      const uint32_t pos_w = __popcll(b0 & below) + __popcll(b1 & below);
      if (lane == 0) wave_cnt[wave] = __popcll(b0) + __popcll(b1);
      __syncthreads();
      uint32_t wbase = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t c = wave_cnt[w];
        if ((uint32_t)w < wave) wbase += c;
        tot += c;
      }
      const uint64_t pos = out + wbase + pos_w;
      if (h0 && pos < cap) {
        blo[pos] = z0;
        bhi[pos] = z1;
        bpre[pos] = p << 1;
      }
      if (h1 && pos + h0 < cap) {
        blo[pos + h0] = o0;
        bhi[pos + h0] = o1;
        bpre[pos + h0] = (p << 1) | 1u;
      }
      out += tot;
      __syncthreads();
    }
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
  const unsigned g = (unsigned)((m + kLfThreads - 1) / kLfThreads);
  k_lf<<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_search(const DevView& v, const int64_t* tok, const int64_t* off, uint64_t m,
                  int64_t shift, const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out,
                  uint64_t* hi_out, hipStream_t s) {
  if (m == 0) return 0;
  const unsigned g = (unsigned)((m + kLfThreads - 1) / kLfThreads);
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

// Slice width: enough workgroups to cover the chip (>= ~2048), slices a
// multiple of 32 tokens, at most kMaxSliceTokens.
static void mask_geometry(uint64_t m, uint64_t vocab, uint32_t& S, uint32_t& SW) {
  uint32_t sw = env_u32("FMIDX_MASK_SW", 0);
  if (sw == 0) {
    const uint64_t want = (2048 + m - 1) / m;
    const uint64_t max_s = std::max<uint64_t>(1, (vocab + 1023) / 1024);
    const uint64_t s = std::min<uint64_t>(std::max<uint64_t>(1, want), max_s);
    sw = (uint32_t)((vocab + s - 1) / s);
  }
  sw = (sw + 31) & ~31u;
  if (sw > kMaxSliceTokens) sw = kMaxSliceTokens;
  if (sw < 32) sw = 32;
  SW = sw;
  S = (uint32_t)((vocab + sw - 1) / sw);
}

int launch_mask(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                uint8_t* mask, uint64_t ld, uint64_t vocab, int64_t shift, int packed,
                hipStream_t s) {
  if (m == 0 || vocab == 0) return 0;
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
  const uint64_t grid = m * S;
  if (grid > 0x7fffffffull) {
    set_error("too many rows for one launch");
    return -1;
  }
  if (packed)
    k_mask<true><<<(unsigned)grid, kMaskThreads, 0, s>>>(v, lo, hi, m, mask, ld, vocab, shift, S, SW);
  else
    k_mask<false><<<(unsigned)grid, kMaskThreads, 0, s>>>(v, lo, hi, m, mask, ld, vocab, shift, S, SW);
  FM_HIP(hipGetLastError());
  return 0;
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
