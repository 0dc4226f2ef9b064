// build.hip -- device-side construction of the HBM index from a BWT.
//
// Replaces the structure-building half of sdsl ``construct`` for
// ``csa_wt_int<>`` (reference cpp_modules_linux/fm_index.cpp:37,44): given the
// BWT (uint32 symbols, one sentinel 0), build
//   * the wavelet matrix (L levels of 64-B rank blocks) by L rounds of
//     ballot-pack + block scan + stable partition,
//   * C / D tables from the final wavelet order (no histogram atomics),
//   * the range-presence bitmap hierarchy.
// Every pass is a coalesced stream over n symbols.
#include "fmidx_internal.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace fmidx {

double build_clock() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void build_phase(const char* name, double t0, hipStream_t s) {
  static const bool on = [] {
    const char* e = std::getenv("FMIDX_BUILD_TIMES");
    return e && *e && *e != '0';
  }();
  if (!on) return;
  (void)hipStreamSynchronize(s);
  std::fprintf(stderr, "[fmidx] build: %s %.2f s\n", name, build_clock() - t0);
}

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// Exclusive scan of a per-thread uint64 over a 256-thread block.
__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* total, uint64_t* lds /*[kWaves]*/) {
  const uint32_t lane = lane_id();
  const uint32_t wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) lds[wave] = x;
  __syncthreads();
  uint64_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    const uint64_t t = lds[w];
    if ((uint32_t)w < wave) base += t;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

__global__ void __launch_bounds__(kThreads) k_chunk_sums(const uint64_t* __restrict__ in, uint64_t n,
                                                        uint64_t* __restrict__ sums) {
  __shared__ uint64_t lds[kWaves];
  const uint64_t base = (uint64_t)blockIdx.x * (kThreads * 4) + threadIdx.x * 4;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + k < n) s += in[base + k];
  uint64_t tot;
  block_exclusive_scan(s, &tot, lds);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kThreads) k_chunk_scan(const uint64_t* __restrict__ in, uint64_t n,
                                                        const uint64_t* __restrict__ offs,
                                                        uint64_t* __restrict__ out,
                                                        uint64_t* __restrict__ total) {
  __shared__ uint64_t lds[kWaves];
  const uint64_t base = (uint64_t)blockIdx.x * (kThreads * 4) + threadIdx.x * 4;
  uint64_t v[4];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = (base + k < n) ? in[base + k] : 0;
    s += v[k];
  }
  uint64_t tot;
  uint64_t ex = block_exclusive_scan(s, &tot, lds) + (offs ? offs[blockIdx.x] : 0);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (base + k < n) out[base + k] = ex;
    ex += v[k];
  }
  if (total && blockIdx.x == gridDim.x - 1 && threadIdx.x == kThreads - 1) *total = ex;
}

__global__ void k_max_sym(const uint32_t* __restrict__ a, uint64_t n, uint32_t* __restrict__ out) {
  uint32_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    m = max(m, a[i]);
  for (int d = 32; d > 0; d >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, d, 64));
  if (lane_id() == 0) atomicMax(out, m);
}

__global__ void k_count_zero(const uint32_t* __restrict__ a, uint64_t n, unsigned long long* out) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    c += (a[i] == 0u);
  if (c) atomicAdd(out, c);
}

// Symbol runs of the final wavelet order: S[c] = first row, E[c] = one past.
// Grid-stride: a dispatch holds at most 2^32 work-items per dimension, so a
// one-thread-per-row grid would silently cover only part of n > 2^32.
__global__ void k_bounds(const uint32_t* __restrict__ fin, uint64_t n, uint64_t* __restrict__ S,
                         uint64_t* __restrict__ E) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = fin[i];
    if (i == 0 || fin[i - 1] != c) S[c] = i;
    if (i + 1 == n || fin[i + 1] != c) E[c] = i + 1;
  }
}

__global__ void k_counts(const uint64_t* __restrict__ S, const uint64_t* __restrict__ E, uint64_t K,
                         uint64_t* __restrict__ cnt, unsigned long long* __restrict__ sigma) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= K) return;
  const uint64_t k = E[c] - S[c];
  cnt[c] = k;
  if (k) atomicAdd(sigma, 1ull);
}

__global__ void k_dtable(const uint64_t* __restrict__ C, const uint64_t* __restrict__ S, uint64_t K,
                         int64_t* __restrict__ D) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= K) return;
  D[c] = (int64_t)C[c] - (int64_t)S[c];
}

// ---- range bitmaps -------------------------------------------------------
// Base level: one workgroup per aligned run of B0 rows; LDS bitmap, then store.
__global__ void __launch_bounds__(kThreads) k_bm_base(const uint32_t* __restrict__ bwt,
                                                     uint32_t log2b0, uint32_t words,
                                                     uint32_t* __restrict__ out) {
  extern __shared__ uint32_t bits[];
  for (uint32_t w = threadIdx.x; w < words; w += kThreads) bits[w] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x << log2b0;
  const uint32_t cnt = 1u << log2b0;
  const uint4* src = reinterpret_cast<const uint4*>(bwt + base);
  for (uint32_t j = threadIdx.x; j < cnt / 4; j += kThreads) {
    const uint4 q = src[j];
    atomicOr(&bits[q.x >> 5], 1u << (q.x & 31));
    atomicOr(&bits[q.y >> 5], 1u << (q.y & 31));
    atomicOr(&bits[q.z >> 5], 1u << (q.z & 31));
    atomicOr(&bits[q.w >> 5], 1u << (q.w & 31));
  }
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(out + (uint64_t)blockIdx.x * words);
  const uint4* s4 = reinterpret_cast<const uint4*>(bits);
  for (uint32_t w = threadIdx.x; w < words / 4; w += kThreads) dst[w] = s4[w];
}

// Bitmap of every symbol in BWT[0, n): LDS bitmap per workgroup over a grid
// stride, merged with global atomicOr (once per set word per workgroup).
__global__ void __launch_bounds__(kThreads) k_bm_full(const uint32_t* __restrict__ bwt, uint64_t n,
                                                     uint32_t words, uint32_t* __restrict__ out) {
  extern __shared__ uint32_t bits[];
  for (uint32_t w = threadIdx.x; w < words; w += kThreads) bits[w] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads) {
    const uint32_t c = bwt[i];
    atomicOr(&bits[c >> 5], 1u << (c & 31));
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < words; w += kThreads)
    if (bits[w]) atomicOr(&out[w], bits[w]);
}

__global__ void __launch_bounds__(kThreads) k_bm_up(const uint32_t* __restrict__ child,
                                                   uint32_t words, uint32_t* __restrict__ out) {
  const uint64_t p = blockIdx.x;
  const uint4* c = reinterpret_cast<const uint4*>(child + p * 4 * words);
  uint4* o = reinterpret_cast<uint4*>(out + p * words);
  const uint32_t w4 = words / 4;
  for (uint32_t w = threadIdx.x; w < w4; w += kThreads) {
    uint4 a = c[w], b = c[w4 + w], d = c[2 * w4 + w], e = c[3 * w4 + w];
    a.x |= b.x | d.x | e.x;
    a.y |= b.y | d.y | e.y;
    a.z |= b.z | d.z | e.z;
    a.w |= b.w | d.w | e.w;
    o[w] = a;
  }
}

// ---- 2-level wavelet matrix (LF path) ------------------------------------
// One workgroup per superblock (64 blocks of 1024 digits): per block, the
// header (running digit counts since the superblock start) is written before
// the block's own digits are counted; the superblock totals go to sbtot.
__global__ void __launch_bounds__(kThreads) k_w2_super(const uint32_t* __restrict__ cur, uint64_t n,
                                                      uint32_t shift, uint32_t bits, uint64_t nblk,
                                                      uint8_t* __restrict__ blocks, uint64_t blk_bytes,
                                                      uint32_t* __restrict__ sbtot) {
  extern __shared__ uint32_t sh[];   // run[R], cnt[R]
  const uint32_t R = 1u << bits;
  uint32_t* run = sh;
  uint32_t* cnt = sh + R;
  for (uint32_t d = threadIdx.x; d < 2 * R; d += kThreads) sh[d] = 0;
  __syncthreads();
  const uint64_t sbk = blockIdx.x;
  const uint32_t per_sb = 1u << (kW2SbLog2 - kW2BlkLog2);
  for (uint32_t j = 0; j < per_sb; ++j) {
    const uint64_t b = sbk * per_sb + j;
    if (b >= nblk) break;
    uint8_t* blk = blocks + b * blk_bytes;
    uint16_t* hdr = reinterpret_cast<uint16_t*>(blk);
    for (uint32_t d = threadIdx.x; d < R; d += kThreads) hdr[d] = (uint16_t)run[d];
    uint8_t* pay = blk + 2 * R;
#pragma unroll
    for (int t = 0; t < kW2Blk / kThreads; ++t) {
      const uint32_t k = t * kThreads + threadIdx.x;
      const uint64_t i = b * kW2Blk + k;
      uint32_t d = 0;
      if (i < n) {
        d = (cur[i] >> shift) & (R - 1);
        atomicAdd(&cnt[d], 1u);
      }
      if (bits > 8)
        reinterpret_cast<uint16_t*>(pay)[k] = (uint16_t)d;
      else
        pay[k] = (uint8_t)d;
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < R; d += kThreads) {
      run[d] += cnt[d];
      cnt[d] = 0;
    }
    __syncthreads();
  }
  for (uint32_t d = threadIdx.x; d < R; d += kThreads) sbtot[sbk * R + d] = run[d];
}

// Per digit: absolute counts before every superblock, and the total.
__global__ void k_w2_sbscan(const uint32_t* __restrict__ sbtot, uint64_t nsb, uint32_t R,
                            uint64_t* __restrict__ sb, uint64_t* __restrict__ total) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= R) return;
  uint64_t acc = 0;
#pragma unroll 8
  for (uint64_t s = 0; s < nsb; ++s) {
    const uint32_t v = sbtot[s * R + d];
    sb[s * R + d] = acc;
    acc += v;
  }
  total[d] = acc;
}

// ---- E array: LF(i) | BWT[i] << 36 ----------------------------------------
struct InSymRange {
  uint32_t c0, c1;
  __host__ __device__ bool operator()(uint32_t x) const { return x >= c0 && x < c1; }
};

__global__ void __launch_bounds__(kThreads) k_gather_keys(const uint32_t* __restrict__ bwt,
                                                         const uint64_t* __restrict__ pos, uint64_t m,
                                                         uint32_t c0, uint32_t* __restrict__ key) {
  for (uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x; k < m; k += (uint64_t)gridDim.x * kThreads)
    key[k] = bwt[pos[k]] - c0;
}

// k-th position in (symbol, position) order has LF = base + k
__global__ void __launch_bounds__(kThreads) k_write_e(const uint64_t* __restrict__ pos,
                                                     const uint32_t* __restrict__ key, uint64_t m, uint64_t base,
                                                     uint32_t c0, uint64_t* __restrict__ E) {
  for (uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x; k < m; k += (uint64_t)gridDim.x * kThreads)
    E[pos[k]] = (base + k) | ((uint64_t)(key[k] + c0) << kESymShift);
}

// E2[i] = BWT[LF(i)]
__global__ void __launch_bounds__(kThreads) k_write_e2(const uint64_t* __restrict__ E, const uint32_t* __restrict__ bwt,
                                                      uint64_t n, uint32_t* __restrict__ E2) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads)
    E2[i] = bwt[E[i] & kELfMask];
}

template <typename T>
int dmalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  FM_HIP(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return 0;
}

}  // namespace

int exclusive_scan_u64(const uint64_t* d_in, uint64_t* d_out, uint64_t n, hipStream_t s,
                       uint64_t* d_total) {
  if (n == 0) {
    if (d_total) FM_HIP(hipMemsetAsync(d_total, 0, sizeof(uint64_t), s));
    return 0;
  }
  const uint64_t per = kThreads * 4;
  const uint64_t chunks = (n + per - 1) / per;
  uint64_t* offs = nullptr;
  if (chunks > 1) {
    uint64_t* sums = nullptr;
    if (dmalloc(&sums, chunks) || dmalloc(&offs, chunks)) return -1;
    k_chunk_sums<<<(unsigned)chunks, kThreads, 0, s>>>(d_in, n, sums);
    if (exclusive_scan_u64(sums, offs, chunks, s, nullptr)) return -1;
    FM_HIP(hipStreamSynchronize(s));
    FM_HIP(hipFree(sums));
  }
  k_chunk_scan<<<(unsigned)chunks, kThreads, 0, s>>>(d_in, n, offs, d_out, d_total);
  FM_HIP(hipGetLastError());
  if (offs) {
    FM_HIP(hipStreamSynchronize(s));
    FM_HIP(hipFree(offs));
  }
  return 0;
}

__global__ void __launch_bounds__(kThreads) k_e_symbols(const uint64_t* __restrict__ E, uint64_t n,
                                                        uint32_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads)
    out[i] = (uint32_t)(E[i] >> kESymShift);
}

// The BWT as plain uint32 symbols: the kept copy, or one materialised from E
// (owned by h, freed with it) -- for fm_device_bwt / fm_save, not the query path.
int device_bwt_view(Index* h, const uint32_t** out) {
  if (h->bwt) {
    *out = h->bwt;
    return 0;
  }
  if (!h->bwt_view) {
    if (!h->E) {
      set_error("index has neither a BWT nor E");
      return -1;
    }
    if (dmalloc(&h->bwt_view, h->n)) return -1;
    k_e_symbols<<<2048, kThreads, 0, h->stream>>>(h->E, h->n, h->bwt_view);
    FM_HIP(hipGetLastError());
    FM_HIP(hipStreamSynchronize(h->stream));
  }
  *out = h->bwt_view;
  return 0;
}

// h->bwt must already hold the BWT (device, owned by h).
int device_build_from_bwt(Index* h, const uint32_t* d_bwt, uint64_t n, hipStream_t s) {
  if (n == 0) {
    set_error("empty BWT");
    return -1;
  }
  // the range-cache table packs hi below a 34-bit id shift and the transition
  // slots pack child start / width in 34 bits: positions must fit 34 bits
  static_assert(kCacheIdShift == 34 && kMask34 == (1ull << 34) - 1, "position packing");
  static_assert(kTSymShift + 18 == 38, "transition key: 20-bit parent id, 18-bit symbol (wider ones left out)");
  if (n >= (1ull << 34)) {
    set_error("n = %llu rows: the index packs row positions in 34 bits (n < 2^34)", (unsigned long long)n);
    return -1;
  }
  const unsigned grid_stream = 2048;
  // -- alphabet
  uint32_t* d_max = nullptr;
  unsigned long long* d_z = nullptr;
  if (dmalloc(&d_max, 1) || dmalloc(&d_z, 1)) return -1;
  FM_HIP(hipMemsetAsync(d_max, 0, 4, s));
  FM_HIP(hipMemsetAsync(d_z, 0, 8, s));
  k_max_sym<<<grid_stream, kThreads, 0, s>>>(d_bwt, n, d_max);
  k_count_zero<<<grid_stream, kThreads, 0, s>>>(d_bwt, n, d_z);
  uint32_t max_sym = 0;
  unsigned long long nzero = 0;
  FM_HIP(hipMemcpyAsync(&max_sym, d_max, 4, hipMemcpyDeviceToHost, s));
  FM_HIP(hipMemcpyAsync(&nzero, d_z, 8, hipMemcpyDeviceToHost, s));
  FM_HIP(hipStreamSynchronize(s));
  FM_HIP(hipFree(d_max));
  FM_HIP(hipFree(d_z));
  if (nzero != 1) {
    set_error("BWT must contain exactly one sentinel 0 (found %llu)", nzero);
    return -1;
  }
  uint32_t L = 1;
  while (L < 32 && (max_sym >> L) != 0) ++L;
  if (L > (uint32_t)kMaxLevels) {
    set_error("symbol %u too large (max %d bits)", max_sym, kMaxLevels);
    return -1;
  }
  h->n = n;
  h->L = L;
  h->max_sym = max_sym;
  // -- the 2-level wavelet matrix, with C / sigma from its final order
  {
    const double t = build_clock();
    if (device_build_w2(h, d_bwt, n, s)) return -1;
    build_phase("2-level wavelet matrix", t, s);
  }
  uint64_t* C = h->C;

  // -- range bitmaps
  // Base block of the aligned bitmap hierarchy.  A decode step never reads the
  // hierarchy at scale (every range of >= cache_min rows it can reach is in
  // the range cache, and a narrower range holds no aligned 4096-row block);
  // it serves arbitrary user ranges and the cache's own construction.  At C3
  // 2^14-row blocks instead of 2^12 free 16.5 GiB (200.4 -> 183.9) with the
  // same step (13.4 us cold) and build time (profiles/r03_memory/bm_log2/);
  // small indexes keep 2^12 so that they still get a hierarchy and a cache.
  // From 2^31 rows 2^16 (round 4, with the plain BWT freed: C3 122.0 -> 117.9 GiB,
  // 13.72 vs 13.86 us cold, build 12.0 -> 14.6 s; profiles/r04_memory/).
  const uint32_t log2b0 = h->opts.bm_log2 >= 0 ? (uint32_t)h->opts.bm_log2
                                               : (n >= (1ull << 31) ? 16 : n >= (1ull << 26) ? 14 : 12);
  const uint32_t words = (uint32_t)(((uint64_t)max_sym + 1 + 127) / 128 * 4);
  const uint64_t nb0 = n >> log2b0;
  uint32_t bm_levels = 0;
  uint64_t bm_off[kMaxBmLevels] = {0}, bm_count[kMaxBmLevels] = {0};
  uint64_t total_words = 0;
  // bitmaps only pay off for vocabulary-sized alphabets (LDS holds one bitmap)
  const bool bm_ok = (uint64_t)words * 4 <= 64 * 1024;
  for (uint64_t c = bm_ok ? nb0 : 0; c > 0 && bm_levels < (uint32_t)kMaxBmLevels; c >>= 2) {
    bm_off[bm_levels] = total_words;
    bm_count[bm_levels] = c;
    total_words += c * words;
    ++bm_levels;
  }
  uint32_t* bm = nullptr;
  uint32_t* bm_full = nullptr;
  if (dmalloc(&bm, total_words)) return -1;
  if (bm_ok) {
    if (dmalloc(&bm_full, words)) return -1;
    FM_HIP(hipMemsetAsync(bm_full, 0, (size_t)words * 4, s));
    k_bm_full<<<1024, kThreads, words * 4, s>>>(d_bwt, n, words, bm_full);
    FM_HIP(hipGetLastError());
  }
  if (bm_levels > 0) {
    k_bm_base<<<(unsigned)nb0, kThreads, words * 4, s>>>(d_bwt, log2b0, words, bm + bm_off[0]);
    FM_HIP(hipGetLastError());
    for (uint32_t j = 1; j < bm_levels; ++j) {
      k_bm_up<<<(unsigned)bm_count[j], kThreads, 0, s>>>(bm + bm_off[j - 1], words, bm + bm_off[j]);
      FM_HIP(hipGetLastError());
    }
  }
  FM_HIP(hipStreamSynchronize(s));

  h->bm = bm;
  h->bm_full = bm_full;
  h->bm_bytes = total_words * 4;
  DevView& v = h->view;   // (device_build_w2 set C, D2 and the levels)
  v.n = n;
  v.C = C;
  v.bwt = d_bwt;
  v.bm = bm;
  v.bm_full = bm_full;
  for (uint32_t j = 0; j < bm_levels; ++j) {
    v.bm_off[j] = bm_off[j];
    v.bm_count[j] = bm_count[j];
  }
  v.L = L;
  v.max_sym = max_sym;
  v.bm_words = words;
  v.bm_levels = bm_levels;
  v.bm_log2 = log2b0;
  // a decode range of >= cache_min rows is cached (every such range reachable
  // from the root is), so its probe hits: waiting for the probe alone before
  // any rank load measured 17.5 -> 16.1 us/step cold, 10.4 -> 9.8 warm at C3
  v.probe_first = h->opts.probe_first != 0;
  // -- follow-set bitmaps (one per symbol's C-block), built with the mask
  //    kernel itself once the view above is complete
  // (off by default: the range-bitmap cache below holds every C-block of
  // width >= its threshold, and narrower ones are streamed)
  if (bm_ok && h->opts.follow_bitmaps != 0) {
    const uint64_t nsym = (uint64_t)max_sym + 1;
    uint32_t* fb = nullptr;
    if (dmalloc(&fb, nsym * words)) return -1;
    if (launch_follow_bitmaps(v, C, nsym, fb, s)) return -1;
    FM_HIP(hipStreamSynchronize(s));
    h->bm_follow = fb;
    h->follow_bytes = nsym * words * 4;
    v.bm_follow = fb;
  }
  double t = build_clock();
  if (device_build_lfe(h, d_bwt, n, s)) return -1;
  build_phase("E array", t, s);
  t = build_clock();
  if (device_build_cache(h, s)) return -1;
  build_phase("range cache + transitions", t, s);
  // The plain BWT duplicates E's symbol field (4 bytes per row: 16.8 GiB at C3).  Once E is
  // built every kernel reads symbols through bwt_sym() / stream_symbols_e(), so the copy is
  // freed; fm_device_bwt materialises one on request (the keep_bwt option keeps it).
  if (h->E && d_bwt == h->bwt && h->opts.keep_bwt == 0) {
    FM_HIP(hipStreamSynchronize(s));
    FM_HIP(hipFree(h->bwt));
    h->bwt = nullptr;
    v.bwt = nullptr;
  }
  h->built = true;
  return 0;
}

// 2-level wavelet matrix over the BWT (see W2Level).  Level l holds the
// sequence stably partitioned by the digits of levels < l (a stable radix sort
// by each digit's bit range); after the last level every symbol c occupies one
// run [S2[c], E2[c]), which gives C (the runs' lengths, scanned) and
// LF(i, c) = descent + C[c] - S2[c].  Resets h->view and sets C, D2, sigma.
int device_build_w2(Index* h, const uint32_t* d_bwt, uint64_t n, hipStream_t s) {
  h->view = DevView{};
  const uint32_t L = h->L;
  const uint32_t NL2 = (L + 8) / 9;
  if (NL2 > (uint32_t)kW2MaxLevels) {
    set_error("2-level wavelet matrix: %u symbol bits need %u levels", L, NL2);
    return -1;
  }
  uint32_t bits[kW2MaxLevels] = {0, 0, 0}, shift[kW2MaxLevels] = {0, 0, 0};
  {
    uint32_t left = L, sh = L;
    for (uint32_t l = 0; l < NL2; ++l) {
      const uint32_t w = (left + (NL2 - l) - 1) / (NL2 - l);   // ceil split, widest first
      bits[l] = w;
      sh -= w;
      shift[l] = sh;
      left -= w;
    }
  }
  const uint64_t nblk = (n >> kW2BlkLog2) + 1;
  const uint64_t nsb = (nblk >> (kW2SbLog2 - kW2BlkLog2)) + 1;
  uint32_t *cur = nullptr, *nxt = nullptr, *sbtot = nullptr;
  uint32_t maxR = 1u << bits[0];
  if (dmalloc(&cur, n) || dmalloc(&nxt, n) || dmalloc(&sbtot, nsb * maxR) || dmalloc(&h->w2_Z, NL2 * (uint64_t)maxR))
    return -1;
  FM_HIP(hipMemcpyAsync(cur, d_bwt, n * 4, hipMemcpyDeviceToDevice, s));
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  FM_HIP(rocprim::radix_sort_keys(nullptr, tmp_bytes, cur, nxt, (size_t)n, 0, L, s));
  if (dmalloc(reinterpret_cast<uint8_t**>(&tmp), tmp_bytes)) return -1;
  uint64_t* total = nullptr;
  if (dmalloc(&total, maxR)) return -1;
  uint64_t bytes = 0;
  for (uint32_t l = 0; l < NL2; ++l) {
    const uint32_t R = 1u << bits[l];
    const uint64_t blk_bytes = 2ull * R + (uint64_t)kW2Blk * (bits[l] > 8 ? 2 : 1);
    if (dmalloc(&h->w2_blocks[l], nblk * blk_bytes) || dmalloc(&h->w2_sb[l], nsb * (uint64_t)R)) return -1;
    bytes += nblk * blk_bytes + nsb * (uint64_t)R * 8;
    k_w2_super<<<(unsigned)nsb, kThreads, 2 * R * 4, s>>>(cur, n, shift[l], bits[l], nblk, h->w2_blocks[l],
                                                         blk_bytes, sbtot);
    FM_HIP(hipGetLastError());
    k_w2_sbscan<<<(R + 255) / 256, 256, 0, s>>>(sbtot, nsb, R, h->w2_sb[l], total);
    FM_HIP(hipGetLastError());
    // Z[d] = digits < d at this level
    std::vector<uint64_t> tot(R), z(R);
    FM_HIP(hipMemcpyAsync(tot.data(), total, R * 8, hipMemcpyDeviceToHost, s));
    FM_HIP(hipStreamSynchronize(s));
    uint64_t acc = 0;
    for (uint32_t d = 0; d < R; ++d) {
      z[d] = acc;
      acc += tot[d];
    }
    uint64_t* Zl = h->w2_Z + (uint64_t)l * maxR;
    FM_HIP(hipMemcpyAsync(Zl, z.data(), R * 8, hipMemcpyHostToDevice, s));
    // next level's sequence: stable partition by this digit
    size_t tb = tmp_bytes;
    FM_HIP(rocprim::radix_sort_keys(tmp, tb, cur, nxt, (size_t)n, shift[l], shift[l] + bits[l], s));
    std::swap(cur, nxt);
    DevView& v = h->view;
    v.w2[l].blocks = h->w2_blocks[l];
    v.w2[l].sb = h->w2_sb[l];
    v.w2[l].Z = Zl;
    v.w2[l].blk_bytes = blk_bytes;
    v.w2[l].bits = bits[l];
    v.w2[l].shift = shift[l];
  }
  FM_HIP(hipStreamSynchronize(s));
  FM_HIP(hipFree(tmp));
  FM_HIP(hipFree(total));
  FM_HIP(hipFree(sbtot));
  FM_HIP(hipFree(nxt));
  // S2 / C / D2 from the final order
  const uint64_t K = 1ull << L;
  uint64_t *S = nullptr, *E = nullptr, *cnt = nullptr;
  unsigned long long* d_sigma = nullptr;
  if (dmalloc(&S, K) || dmalloc(&E, K) || dmalloc(&cnt, K + 1) || dmalloc(&h->C, K + 1) || dmalloc(&h->D2, K) ||
      dmalloc(&d_sigma, 1))
    return -1;
  FM_HIP(hipMemsetAsync(S, 0, K * 8, s));
  FM_HIP(hipMemsetAsync(E, 0, K * 8, s));
  FM_HIP(hipMemsetAsync(cnt, 0, (K + 1) * 8, s));
  FM_HIP(hipMemsetAsync(d_sigma, 0, 8, s));
  k_bounds<<<(unsigned)std::min<uint64_t>((n + kThreads - 1) / kThreads, 1u << 20), kThreads, 0, s>>>(cur, n, S,
                                                                                                     E);
  k_counts<<<(unsigned)((K + kThreads - 1) / kThreads), kThreads, 0, s>>>(S, E, K, cnt, d_sigma);
  if (exclusive_scan_u64(cnt, h->C, K + 1, s, nullptr)) return -1;
  k_dtable<<<(unsigned)((K + kThreads - 1) / kThreads), kThreads, 0, s>>>(h->C, S, K, h->D2);
  FM_HIP(hipGetLastError());
  unsigned long long sigma = 0;
  FM_HIP(hipMemcpyAsync(&sigma, d_sigma, 8, hipMemcpyDeviceToHost, s));
  FM_HIP(hipStreamSynchronize(s));
  h->sigma = sigma;
  FM_HIP(hipFree(S));
  FM_HIP(hipFree(E));
  FM_HIP(hipFree(cnt));
  FM_HIP(hipFree(d_sigma));
  FM_HIP(hipFree(cur));
  h->view.D2 = h->D2;
  h->view.NL2 = NL2;
  h->w2_bytes = bytes;
  return 0;
}

// E[i] = LF(i) | BWT[i] << kESymShift.  LF(i) = C[c] + rank_c(i) is the index
// of position i in the (symbol, position) order, so symbols are processed in
// chunks of <= 2^29 occurrences (cut at C boundaries): select the chunk's
// positions (ascending), stable radix sort them by symbol, write base + k.
int device_build_lfe(Index* h, const uint32_t* d_bwt, uint64_t n, hipStream_t s) {
  if (h->opts.lf_e == 0) return 0;
  if (n >= (1ull << kESymShift) || h->max_sym >= (1ull << (64 - kESymShift))) return 0;
  const uint64_t K = (uint64_t)h->max_sym + 1;
  std::vector<uint64_t> C(K + 1);
  FM_HIP(hipMemcpyAsync(C.data(), h->C, (K + 1) * 8, hipMemcpyDeviceToHost, s));
  FM_HIP(hipStreamSynchronize(s));
  const uint64_t kChunk = 1ull << 29;
  uint64_t maxm = 0;
  std::vector<uint32_t> cuts{0};
  while (cuts.back() < K) {
    uint32_t c = cuts.back();
    const uint64_t start = C[c];
    uint32_t e = c + 1;
    while (e < K && C[e + 1] - start <= kChunk) ++e;
    cuts.push_back(e);
    maxm = std::max(maxm, C[e] - start);
  }
  if (dmalloc(&h->E, n)) return -1;
  uint64_t *pos = nullptr, *pos2 = nullptr, *d_cnt = nullptr;
  uint32_t *key = nullptr, *key2 = nullptr;
  if (dmalloc(&pos, maxm) || dmalloc(&pos2, maxm) || dmalloc(&key, maxm) || dmalloc(&key2, maxm) ||
      dmalloc(&d_cnt, 1))
    return -1;
  rocprim::counting_iterator<uint64_t> iota(0);
  size_t t1 = 0, t2 = 0;
  auto flags0 = rocprim::make_transform_iterator(d_bwt, InSymRange{0, 1});
  FM_HIP(rocprim::select(nullptr, t1, iota, flags0, pos, d_cnt, (size_t)n, s));
  FM_HIP(rocprim::radix_sort_pairs(nullptr, t2, key, key2, pos, pos2, (size_t)maxm, 0, 32, s));
  uint8_t* tmp = nullptr;
  const size_t tb = std::max(t1, t2);
  if (dmalloc(&tmp, tb)) return -1;
  const unsigned g = (unsigned)std::min<uint64_t>((maxm + kThreads - 1) / kThreads, 1u << 18);
  for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
    const uint32_t c0 = cuts[ci], c1 = cuts[ci + 1];
    const uint64_t m = C[c1] - C[c0];
    if (m == 0) continue;
    size_t need = tb;
    auto flags = rocprim::make_transform_iterator(d_bwt, InSymRange{c0, c1});
    FM_HIP(rocprim::select(tmp, need, iota, flags, pos, d_cnt, (size_t)n, s));
    k_gather_keys<<<g, kThreads, 0, s>>>(d_bwt, pos, m, c0, key);
    FM_HIP(hipGetLastError());
    uint32_t bits = 1;
    while (bits < 32 && ((uint64_t)(c1 - c0 - 1) >> bits) != 0) ++bits;
    need = tb;
    FM_HIP(rocprim::radix_sort_pairs(tmp, need, key, key2, pos, pos2, (size_t)m, 0, bits, s));
    k_write_e<<<g, kThreads, 0, s>>>(pos2, key2, m, C[c0], c0, h->E);
    FM_HIP(hipGetLastError());
  }
  FM_HIP(hipStreamSynchronize(s));
  FM_HIP(hipFree(tmp));
  FM_HIP(hipFree(pos));
  FM_HIP(hipFree(pos2));
  FM_HIP(hipFree(key));
  FM_HIP(hipFree(key2));
  FM_HIP(hipFree(d_cnt));
  h->view.E = h->E;
  // E2 (the lf_e2 option, off by default): the decode kernel's narrow rows read
  // their new range's content with the LF scan instead of streaming it after
  // the plan.  Measured (profiles/r02_cold_sweep/r02e2b_*): C3 13.5 vs 13.4 us
  // cold, C2 8.4 vs 8.5, C5 46.7 vs 48.1 -- the second array's cold misses
  // lengthen the scan about as much as the stream round trip it removes, so
  // its 4n bytes (17 GiB at C3) are not spent by default.
  h->view.E2 = nullptr;
  if (h->opts.lf_e2 != 0) {
    if (dmalloc(&h->E2, n)) return -1;
    k_write_e2<<<(unsigned)std::min<uint64_t>((n + kThreads - 1) / kThreads, 1u << 18), kThreads, 0, s>>>(
        h->E, d_bwt, n, h->E2);
    FM_HIP(hipGetLastError());
    FM_HIP(hipStreamSynchronize(s));
    h->view.E2 = h->E2;
  }
  return 0;
}

}  // namespace fmidx
