// fmidx_internal.h -- HBM layout of the FM-index and the device primitives
// shared by the build and query kernels (gfx950 / CDNA4, wave64).
//
// Layout (all resident in HBM, built once per index):
//
//   wm      wavelet matrix over the BWT, L levels (L = bit width of the largest
//           symbol; 17 for a 128k vocabulary + SHIFT).  Level l is an array of
//           64-byte rank blocks: word 0 = number of 1 bits before the block
//           (absolute, uint64), words 1..7 = 448 payload bits.  One rank costs
//           exactly one 64-B line.  The MSB of the symbol is level 0.
//   zeros   number of 0 bits of every level (kernel-argument array).
//   D       D[c] = C[c] - S[c] as int64, where C[c] is the FM-index C array and
//           S[c] the start of symbol c in the wavelet matrix's final order, so
//           LF(i, c) = desc_c(i) + D[c] (desc = the L-level descent).
//   C       C[0 .. 2^L] (C[c+1]-C[c] = occurrences of c).
//   bwt     the BWT as plain uint32 symbols (streamed for narrow ranges).
//   bm      range-presence bitmaps: level j holds one bitmap of W bits for each
//           aligned run of B0*4^j BWT rows (bit s set iff symbol s occurs).
//           A wide range is answered by OR-ing O(levels) bitmaps plus
//           streaming its two partial ends.
//   sa/text optional: suffix array (uint64) and T' (uint32) for locate/extract.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace fmidx {

constexpr int kMaxLevels = 26;         // 2^26 symbol table; token ids + 10 need 18 at most
constexpr int kBlockBits = 448;        // payload bits per 64-B rank block
constexpr int kBlockWords = 8;         // uint64 words per rank block
constexpr int kMaxBmLevels = 24;

// Everything a kernel needs, passed by value as a kernel argument.
struct DevView {
  uint64_t n;                 // BWT length (corpus tokens + 1 sentinel)
  uint64_t nblk;              // rank blocks per level = n / 448 + 1
  const uint64_t* wm;         // L * nblk * 8 words
  const int64_t* D;           // [2^L]
  const uint64_t* C;          // [2^L + 1]
  const uint32_t* bwt;        // [n]
  const uint32_t* bm;         // bitmap hierarchy
  uint64_t bm_off[kMaxBmLevels];   // word offset of each bitmap level
  uint64_t bm_count[kMaxBmLevels]; // bitmaps per level
  uint64_t zeros[kMaxLevels];
  uint32_t L;                 // wavelet levels
  uint32_t max_sym;           // largest symbol value present
  uint32_t bm_words;          // uint32 words per bitmap (multiple of 4)
  uint32_t bm_levels;         // number of bitmap levels (0 = none)
  uint32_t bm_log2;           // log2(B0)
  uint32_t pad_;
};

// ---------------------------------------------------------------------------
// rank1 inside one 64-byte block: ones before bit ``off`` (off < 448).
__device__ __forceinline__ uint64_t block_rank(const uint64_t* __restrict__ line, uint32_t off) {
  const uint4* p = reinterpret_cast<const uint4*>(line);
  const uint4 a = p[0];
  const uint4 b = p[1];
  const uint4 c = p[2];
  const uint4 d = p[3];
  uint64_t w[8];
  w[0] = (uint64_t)a.x | ((uint64_t)a.y << 32);
  w[1] = (uint64_t)a.z | ((uint64_t)a.w << 32);
  w[2] = (uint64_t)b.x | ((uint64_t)b.y << 32);
  w[3] = (uint64_t)b.z | ((uint64_t)b.w << 32);
  w[4] = (uint64_t)c.x | ((uint64_t)c.y << 32);
  w[5] = (uint64_t)c.z | ((uint64_t)c.w << 32);
  w[6] = (uint64_t)d.x | ((uint64_t)d.y << 32);
  w[7] = (uint64_t)d.z | ((uint64_t)d.w << 32);
  const uint32_t q = off >> 6;
  const uint32_t r = off & 63u;
  uint64_t cnt = w[0];
#pragma unroll
  for (uint32_t j = 0; j < 7; ++j) {
    const uint64_t word = w[1 + j];
    const uint64_t m = (j < q) ? ~0ull : ((j == q) ? ((r == 0) ? 0ull : (~0ull >> (64 - r))) : 0ull);
    cnt += (uint64_t)__popcll(word & m);
  }
  return cnt;
}

__device__ __forceinline__ const uint64_t* level_base(const DevView& v, uint32_t lev) {
  return v.wm + (uint64_t)lev * v.nblk * kBlockWords;
}

// ones in level ``lev`` before position i (0 <= i <= n)
__device__ __forceinline__ uint64_t rank1(const DevView& v, uint32_t lev, uint64_t i) {
  const uint64_t b = i / kBlockBits;
  const uint32_t off = (uint32_t)(i - b * kBlockBits);
  return block_rank(level_base(v, lev) + b * kBlockWords, off);
}

// L-level descent of the half-open range [l, r) along symbol c.  On return
// [l, r) is the run of c's occurrences inside the wavelet matrix's final
// order; r - l = occurrences of c in BWT[l0, r0).  Stops early when empty.
__device__ __forceinline__ void wm_descend(const DevView& v, uint32_t c, uint64_t& l, uint64_t& r) {
  for (uint32_t lev = 0; lev < v.L; ++lev) {
    const uint64_t bl = l / kBlockBits;
    const uint64_t br = r / kBlockBits;
    const uint64_t* base = level_base(v, lev);
    const uint64_t r1l = block_rank(base + bl * kBlockWords, (uint32_t)(l - bl * kBlockBits));
    const uint64_t r1r = block_rank(base + br * kBlockWords, (uint32_t)(r - br * kBlockBits));
    if ((c >> (v.L - 1 - lev)) & 1u) {
      l = v.zeros[lev] + r1l;
      r = v.zeros[lev] + r1r;
    } else {
      l -= r1l;
      r -= r1r;
    }
    if (l >= r) return;
  }
}

// One reference backward_search_step on a half-open state (fm_index.cpp:67-97
// as driven by index.py:110): (0,0) = empty in and out.
__device__ __forceinline__ void lf_step(const DevView& v, int64_t sym, uint64_t& lo, uint64_t& hi) {
  if (hi > v.n) hi = v.n;                    // high clamp (fm_index.cpp:74-76)
  if (lo >= hi || sym < 0 || (uint64_t)sym > v.max_sym) {  // low > high / unknown symbol
    lo = 0;
    hi = 0;
    return;
  }
  const uint32_t c = (uint32_t)sym;
  uint64_t l = lo, r = hi;
  wm_descend(v, c, l, r);
  if (l >= r) {
    lo = 0;
    hi = 0;
    return;
  }
  const int64_t d = v.D[c];
  lo = (uint64_t)((int64_t)l + d);
  hi = (uint64_t)((int64_t)r + d);
}

// ---------------------------------------------------------------------------
// host-side owner of the device structures
struct Index {
  int device = 0;
  hipStream_t stream = nullptr;  // internal stream for host-API calls
  DevView view{};
  uint64_t n = 0;
  uint64_t sigma = 0;            // distinct symbols in the BWT
  uint64_t max_sym = 0;
  uint32_t L = 0;
  // device allocations
  uint64_t* wm = nullptr;
  int64_t* D = nullptr;
  uint64_t* C = nullptr;
  uint32_t* bwt = nullptr;
  uint32_t* bm = nullptr;
  uint64_t* sa = nullptr;
  uint32_t* text = nullptr;
  uint64_t wm_bytes = 0, bm_bytes = 0;
  // grow-only workspace for batched traversals
  void* ws = nullptr;
  size_t ws_bytes = 0;
  bool built = false;
  void release();
};

// build.hip
int device_build_from_bwt(Index* h, const uint32_t* d_bwt_owned, uint64_t n, hipStream_t s);
int exclusive_scan_u64(const uint64_t* d_in, uint64_t* d_out, uint64_t n, hipStream_t s,
                       uint64_t* d_total);

// query.hip launchers
int launch_lf_step(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                   const uint64_t* lo, const uint64_t* hi, uint64_t* lo_out, uint64_t* hi_out,
                   uint64_t m, hipStream_t s);
int launch_search(const DevView& v, const int64_t* tok, const int64_t* off, uint64_t m,
                  int64_t shift, const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out,
                  uint64_t* hi_out, hipStream_t s);
int launch_raw_multi(const DevView& v, const uint64_t* q, uint64_t len, uint64_t* out2,
                     hipStream_t s);
int launch_step_raw(const DevView& v, uint64_t sym, uint64_t low, uint64_t high, uint64_t* out2,
                    hipStream_t s);
int launch_mask(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                uint8_t* mask, uint64_t ld, uint64_t vocab, int64_t shift, int packed,
                hipStream_t s);
int launch_decode(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                  const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out, uint64_t* hi_out,
                  uint64_t m, uint8_t* mask, uint64_t ld, uint64_t vocab, int packed, hipStream_t s);
int launch_distinct(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                    const uint64_t* cap_off, uint64_t* syms, uint64_t* counts, uint64_t* k,
                    void* ws, uint64_t total_cap, hipStream_t s);
size_t distinct_ws_bytes(uint64_t total_cap);

void set_error(const char* fmt, ...);

}  // namespace fmidx

#define FM_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::fmidx::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
      return -1;                                                                        \
    }                                                                                   \
  } while (0)
