// fmidx_internal.h -- HBM layout of the FM-index and the device primitives
// shared by the build and query kernels (gfx950 / CDNA4, wave64).
//
// Layout (all resident in HBM, built once per index):
//
//   w2      2-level wavelet matrix over the BWT (W2Level below): digits of
//           <= 9 bits, 17 = 9 + 8 for a 128k vocabulary + SHIFT, so an LF step
//           is 2 dependent rank round trips (a binary wavelet tree: 17).  Level
//           l is an array of 1024-digit rank blocks (per-digit uint16 header +
//           the digits as uint8 / uint16), with per-superblock (2^16 digits)
//           absolute counts and Z[l][d] = digits < d in that level.
//   D2      D2[c] = C[c] - S2[c] as int64 (S2[c] = start of symbol c in the
//           matrix's final order), so LF(i, c) = desc_c(i) + D2[c].
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

constexpr int kMaxSymBits = 26;        // 2^26 symbol table; token ids + 10 need 18 at most
constexpr int kMaxLevels = kMaxSymBits;
constexpr int kMaxBmLevels = 24;
// 2-level wavelet matrix (the LF path): digits of <= 9 bits, so L <= 18 bits
// in 2 levels (17 = 9 + 8 for a 128k vocabulary + SHIFT), <= 27 in 3.
constexpr int kW2MaxLevels = 3;
constexpr int kW2BlkLog2 = 10;                 // 1024 digits per rank block
constexpr int kW2Blk = 1 << kW2BlkLog2;
constexpr int kW2SbLog2 = 16;                  // 64 blocks per superblock (u16 block headers)
// E[i] = LF(i) | BWT[i] << 36: a narrow range's LF step reads E[lo, hi) once.
constexpr uint32_t kESymShift = 36;
constexpr uint64_t kELfMask = (1ull << kESymShift) - 1;
constexpr uint32_t kENarrow = 512;             // widest range whose LF step scans E (8 entries per lane)
constexpr uint32_t kEWide = 4096;              // widest range the decode kernel's workgroup scans E for
constexpr uint32_t kContentPath = 1u << 31;    // lf_step_decode<true>: the content came with the E scan

// One level of the 2-level wavelet matrix.  Block b (digits [1024 b, 1024 b +
// 1024)) = [R x uint16 count of each digit before the block, relative to its
// superblock][1024 digits as uint8 (bits <= 8) or uint16].  rank_d(i) = sb +
// header[d] + matches of d in the block's first i mod 1024 digits: three
// independent loads, one round trip.
struct W2Level {
  const uint8_t* blocks;      // nblk2 * blk_bytes
  const uint64_t* sb;         // [nsb2][R] absolute counts before each superblock
  const uint64_t* Z;          // [R] digits < d in this level
  uint64_t blk_bytes;         // 2R + 1024 * digit bytes
  uint32_t bits, shift;       // digit = (c >> shift) & (R - 1)
};

// Everything a kernel needs, passed by value as a kernel argument.
struct DevView {
  uint64_t n;                 // BWT length (corpus tokens + 1 sentinel)
  const uint64_t* C;          // [2^L + 1]
  const uint32_t* bwt;        // [n], or null once E holds the symbols (bwt_sym)
  const uint32_t* bm;         // bitmap hierarchy
  const uint32_t* bm_full;    // bitmap of BWT[0, n) (all symbols), bm_words words
  const uint32_t* bm_follow;  // per symbol c: bitmap of BWT[C[c], C[c+1]) (follow set), or null
  uint64_t bm_off[kMaxBmLevels];   // word offset of each bitmap level
  uint64_t bm_count[kMaxBmLevels]; // bitmaps per level
  // range-bitmap cache: the bitmap of every SA range reachable from the root
  // by LF steps with width >= cache_min (suffix-tree nodes), found by (lo, hi)
  const uint32_t* cache_bm;   // [nodes][bm_words]
  const uint64_t* cache_tab;  // [cap][2] = {lo, hi | id << 34}; lo = ~0: empty
  uint64_t cache_mask;        // cap - 1 (cap a power of 2); 0 = no cache
  uint64_t cache_min;         // width threshold Wc
  // transition table of the cached ranges: (cached parent P, symbol c) ->
  // LF_c(P) for every symbol c occurring in P (or, under a memory budget, only
  // the cached children), with the child's bitmap id or, for a one-row child,
  // its only symbol; 2 words per slot, keyed by the parent's cache id (layout at trans_key below)
  const uint64_t* trans_tab;
  uint64_t trans_cap;         // slots; 0 = none
  const uint32_t* cblock;     // per symbol c: cache id + 1 of its C-block [C[c], C[c+1]) (0 = not cached), or null
  const uint64_t* E;          // [n] LF(i) | BWT[i] << kESymShift (narrow-range LF + streaming), or null
  const uint32_t* E2;         // [n] BWT[LF(i)]: the content of a narrow range's LF image, read with E, or null
  W2Level w2[kW2MaxLevels];   // 2-level wavelet matrix (LF path)
  const int64_t* D2;          // D2[c] = C[c] - S2[c] (S2 = start of c in its final order)
  uint32_t NL2;               // its levels (0 = not built)
  uint32_t L;                 // symbol bits
  uint32_t max_sym;           // largest symbol value present
  uint32_t bm_words;          // uint32 words per bitmap (multiple of 4)
  uint32_t bm_levels;         // number of bitmap levels (0 = none)
  uint32_t bm_log2;           // log2(B0)
  uint32_t probe_first;       // bit 0: a cached range's LF step waits for its transition probe before
                              //    issuing the descent (a hit needs no rank loads); else issued together
                              // bit 1 (kProbeComplete): the table holds every child of every cached
                              //    parent, so a miss beside a free slot proves the symbol absent
#ifdef FMIDX_STAMPS
  uint64_t* stamps;           // diagnostic build only: per-workgroup phase timestamps
#endif
};

// BWT symbol i.  The plain BWT is freed once E exists (E's symbol field holds
// the same symbols; device_build_from_bwt, FMIDX_KEEP_BWT=1 keeps it), so
// every kernel reads single symbols through here.
__device__ __forceinline__ uint32_t bwt_sym(const DevView& v, uint64_t i) {
  return v.bwt ? v.bwt[i] : (uint32_t)(v.E[i] >> kESymShift);
}

// Diagnostic phase stamps (s_memrealtime, 100 MHz), compiled only with
// -DFMIDX_STAMPS.  They are kept in LDS and written out once at the end of the
// workgroup, so the stamped kernel issues no extra global store inside its
// dependent chain (a store ahead of a load in the shared vmcnt queue would
// make the load's wait include the store's acknowledgement).
#ifdef FMIDX_STAMPS
#define FM_STAMP_DECL                                                    \
  __shared__ uint64_t s_stamp_[8];                                       \
  if (threadIdx.x == 0)                                                  \
    for (int s_ = 0; s_ < 8; ++s_)                                       \
      if (s_ != 5) s_stamp_[s_] = 0
#define FM_STAMP(v, slot)                                                \
  do {                                                                   \
    if (threadIdx.x == 0) s_stamp_[(slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define FM_STAMP_T(v, slot, tid)                                         \
  do {                                                                   \
    if (threadIdx.x == (tid)) s_stamp_[(slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define FM_STAMP_FLUSH(v, row)                                           \
  do {                                                                   \
    if (threadIdx.x == 0 && (v).stamps) {                                \
      for (int s_ = 0; s_ < 8; ++s_) (v).stamps[(uint64_t)blockIdx.x * 16 + s_] = s_stamp_[s_]; \
      (v).stamps[(uint64_t)blockIdx.x * 16 + 8] = (row);                 \
    }                                                                    \
  } while (0)
#else
#define FM_STAMP_DECL
#define FM_STAMP_T(v, slot, tid) \
  do {                           \
  } while (0)
#define FM_STAMP(v, slot) \
  do {                    \
  } while (0)
#define FM_STAMP_FLUSH(v, row) \
  do {                         \
  } while (0)
#endif

// Kernel arguments live in memory and reach the wave through the scalar cache:
// a field first touched deep inside a dependent chain costs a scalar-load
// round trip there (measured ~1 us under load per phase).  Materialising every
// hot field at kernel entry issues all those loads together, up front.
#define FM_PRELOAD_VIEW(v)                                                                                 \
  do {                                                                                                     \
    asm volatile("" ::"s"((v).n), "s"((v).C));                                                             \
    asm volatile("" ::"s"((v).bwt), "s"((v).bm), "s"((v).bm_full), "s"((v).bm_follow),                     \
                 "s"((v).bm_count[0]), "s"((v).L), "s"((v).max_sym), "s"((v).bm_words),                    \
                 "s"((v).bm_levels), "s"((v).bm_log2));                                                    \
    asm volatile("" ::"s"((v).D2), "s"((v).NL2), "s"((v).cache_bm), "s"((v).cache_tab),                   \
                 "s"((v).cache_mask), "s"((v).cache_min), "s"((v).E), "s"((v).E2), "s"((v).trans_tab),                  \
                 "s"((v).trans_cap), "s"((v).cblock), "s"((v).probe_first));                                               \
    asm volatile("" ::"s"((v).w2[0].blocks), "s"((v).w2[0].sb), "s"((v).w2[0].Z), "s"((v).w2[0].blk_bytes), \
                 "s"((v).w2[0].bits), "s"((v).w2[0].shift));                                               \
    asm volatile("" ::"s"((v).w2[1].blocks), "s"((v).w2[1].sb), "s"((v).w2[1].Z), "s"((v).w2[1].blk_bytes), \
                 "s"((v).w2[1].bits), "s"((v).w2[1].shift));                                               \
  } while (0)

// ---------------------------------------------------------------------------
// Buffer descriptor over [base, base + bytes) from wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* b = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(b, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// One 8-byte element of a per-row array, as a range-checked buffer load: the
// compiler cannot sink such a load into the branch that uses it, so a row's
// state loads (token, lo, hi) go out together, one round trip.
__device__ __forceinline__ uint64_t row_load_u64(const void* base, uint64_t count, uint64_t i) {
  typedef unsigned v2u_ __attribute__((ext_vector_type(2)));
  const v2u_ q = __builtin_amdgcn_raw_buffer_load_b64(make_rsrc(base, (uint32_t)(count * 8)), (uint32_t)(i * 8), 0, 0);
  return (uint64_t)q.x | ((uint64_t)q.y << 32);
}

// 2-level wavelet matrix rank / LF, computed by 32 lanes (q = lane & 31): lane
// q covers digits [32 q, 32 q + 32) of the block (64 B of uint16 or 32 B of
// uint8 digits), the partial counts meet in an xor-shuffle tree.
__device__ __forceinline__ uint32_t eq16_count(uint32_t w, uint32_t dd, uint32_t valid2) {
  const uint32_t x = w ^ dd;   // dd = d | d << 16
  return ((valid2 & 1u) && (x & 0xFFFFu) == 0) + ((valid2 & 2u) && (x >> 16) == 0);
}

__device__ __forceinline__ uint32_t eq8_count(uint32_t w, uint32_t dd, uint32_t nvalid) {
  const uint32_t x = w ^ dd;   // dd = d * 0x01010101
  uint32_t c = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) c += (j < nvalid) && ((x >> (8 * j)) & 0xFFu) == 0;
  return c;
}

__device__ __forceinline__ uint64_t rank_w2_at(const uint8_t* blocks, const uint64_t* sbp, uint64_t blk_bytes,
                                            uint32_t bits, uint64_t i, uint32_t d, uint32_t q) {
  const uint64_t b = i >> kW2BlkLog2;
  const uint32_t k = (uint32_t)(i & (kW2Blk - 1));
  const uint8_t* base = blocks + b * blk_bytes;
  const uint32_t R = 1u << bits;
  const uint64_t sbv = sbp[(i >> kW2SbLog2) * R + d];
  const uint32_t hdr = reinterpret_cast<const uint16_t*>(base)[d];
  const uint32_t first = 32 * q;   // first digit of this lane
  uint32_t cnt = 0;
  if (bits > 8) {
    const uint4* p = reinterpret_cast<const uint4*>(base + 2 * R) + 4 * q;
    // A lane's 4 loads are issued together under one lane guard and consumed
    // unconditionally (a digit group past k counts nothing): a load guarded
    // per group was sunk into its own branch with a vmcnt(0) behind it, i.e.
    // up to 4 dependent round trips per level.
    uint4 x[4] = {};
    if (first < k) {
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = p[u];
    }
    const uint32_t dd = d | (d << 16);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t j0 = first + 8 * u;   // digits j0 .. j0+7
      const uint32_t nv = j0 < k ? min(8u, k - j0) : 0u;
      cnt += eq16_count(x[u].x, dd, nv >= 2 ? 3u : (nv >= 1 ? 1u : 0u));
      cnt += eq16_count(x[u].y, dd, nv >= 4 ? 3u : (nv >= 3 ? 1u : 0u));
      cnt += eq16_count(x[u].z, dd, nv >= 6 ? 3u : (nv >= 5 ? 1u : 0u));
      cnt += eq16_count(x[u].w, dd, nv >= 8 ? 3u : (nv >= 7 ? 1u : 0u));
    }
  } else {
    const uint4* p = reinterpret_cast<const uint4*>(base + 2 * R) + 2 * q;
    uint4 x[2] = {};
    if (first < k) {
#pragma unroll
      for (int u = 0; u < 2; ++u) x[u] = p[u];
    }
    const uint32_t dd = d * 0x01010101u;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t j0 = first + 16 * u;
      const uint32_t nv = j0 < k ? min(16u, k - j0) : 0u;
      cnt += eq8_count(x[u].x, dd, nv >= 4 ? 4u : nv);
      cnt += eq8_count(x[u].y, dd, nv >= 8 ? 4u : (nv > 4 ? nv - 4 : 0u));
      cnt += eq8_count(x[u].z, dd, nv >= 12 ? 4u : (nv > 8 ? nv - 8 : 0u));
      cnt += eq8_count(x[u].w, dd, nv >= 16 ? 4u : (nv > 12 ? nv - 12 : 0u));
    }
  }
  cnt += __shfl_xor(cnt, 1, 64);
  cnt += __shfl_xor(cnt, 2, 64);
  cnt += __shfl_xor(cnt, 4, 64);
  cnt += __shfl_xor(cnt, 8, 64);
  cnt += __shfl_xor(cnt, 16, 64);
  return sbv + hdr + cnt;
}

__device__ __forceinline__ uint64_t rank_w2(const W2Level& L, uint64_t i, uint32_t d, uint32_t q) {
  return rank_w2_at(L.blocks, L.sb, L.blk_bytes, L.bits, i, d, q);
}

// the four 8-bit digits of a word equal to d, counting those whose bit is set in m (4 bits)
__device__ __forceinline__ uint32_t eq8_count_mask(uint32_t x, uint32_t dd, uint32_t m) {
  const uint32_t y = x ^ dd;
  uint32_t c = 0;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) c += ((m >> j) & 1u) && ((y >> (8 * j)) & 0xFFu) == 0;
  return c;
}

// bits [max(lo - j0, 0), min(hi - j0, w)) of a w-digit chunk starting at block position j0
__device__ __forceinline__ uint32_t chunk_mask(uint32_t j0, uint32_t w, uint32_t lo, uint32_t hi) {
  const uint32_t a = lo > j0 ? min(lo - j0, w) : 0u;
  const uint32_t e = hi > j0 ? min(hi - j0, w) : 0u;
  return a < e ? (((1u << e) - 1u) & ~((1u << a) - 1u)) : 0u;
}

// The same rank by 8 lanes (q = lane & 7), reading at most half a block: a
// position in the block's first half counts the digits before it (rank(i) =
// rank(block start) + matches in [block start, i)), one in its second half the
// digits from it to the block's end (rank(i) = rank(next block's start) -
// matches in [i, block end); for the last block, the level's total of d from
// Z), so every rank reads <= 512 digits and lane q covers [base + 64 q, + 64)
// of them -- the LF sweep ranks eight positions at once (four rows' ends).
// (n = the level's length = the BWT length: block b + 1 exists while b < n / 1024.)
__device__ __forceinline__ uint64_t rank_w2_q8(const W2Level& L, uint64_t i, uint32_t d, uint32_t q, uint64_t n) {
  const uint64_t b = i >> kW2BlkLog2;
  const uint32_t k = (uint32_t)(i & (kW2Blk - 1));
  const uint32_t R = 1u << L.bits;
  const bool back = k > (uint32_t)kW2Blk / 2;
  const bool last = b >= (n >> kW2BlkLog2);   // no next block: the level's total of d instead
  const uint64_t hb = (back && !last) ? b + 1 : b;   // the block whose start rank is read
  const uint8_t* base = L.blocks + b * L.blk_bytes;
  const uint64_t sbv = L.sb[((hb << kW2BlkLog2) >> kW2SbLog2) * R + d];
  const uint32_t hdr = reinterpret_cast<const uint16_t*>(L.blocks + hb * L.blk_bytes)[d];
  // total of d in the level (Z[d + 1] - Z[d], n - Z[R - 1] for the last digit): only read for a
  // second-half position of the last block; clamped loads of Z[d], Z[d + 1] otherwise unused
  const uint64_t z0 = L.Z[d], z1 = L.Z[d + 1 < R ? d + 1 : d];
  const uint64_t tot = (d + 1 < R ? z1 : n) - z0;
  const uint32_t blk_end = last ? (uint32_t)(n & (kW2Blk - 1)) : (uint32_t)kW2Blk;
  const uint32_t lo = back ? k : 0u, hi = back ? blk_end : k;   // the block positions counted
  const uint32_t first = (back ? (uint32_t)kW2Blk / 2 : 0u) + 64 * q;
  const bool need = first < hi && first + 64 > lo;
  uint32_t cnt = 0;
  if (L.bits > 8) {
    const uint4* p = reinterpret_cast<const uint4*>(base + 2 * R) + first / 8;
    uint4 x[8] = {};
    if (need) {   // one guard for all eight loads (see rank_w2_at)
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = p[u];
    }
    const uint32_t dd = d | (d << 16);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t m = chunk_mask(first + 8 * u, 8, lo, hi);   // digits of the chunk counted
      cnt += eq16_count(x[u].x, dd, m & 3u);
      cnt += eq16_count(x[u].y, dd, (m >> 2) & 3u);
      cnt += eq16_count(x[u].z, dd, (m >> 4) & 3u);
      cnt += eq16_count(x[u].w, dd, (m >> 6) & 3u);
    }
  } else {
    const uint4* p = reinterpret_cast<const uint4*>(base + 2 * R) + first / 16;
    uint4 x[4] = {};
    if (need) {
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = p[u];
    }
    const uint32_t dd = d * 0x01010101u;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t m = chunk_mask(first + 16 * u, 16, lo, hi);
      cnt += eq8_count_mask(x[u].x, dd, m & 15u);
      cnt += eq8_count_mask(x[u].y, dd, (m >> 4) & 15u);
      cnt += eq8_count_mask(x[u].z, dd, (m >> 8) & 15u);
      cnt += eq8_count_mask(x[u].w, dd, (m >> 12) & 15u);
    }
  }
  cnt += __shfl_xor(cnt, 1, 64);
  cnt += __shfl_xor(cnt, 2, 64);
  cnt += __shfl_xor(cnt, 4, 64);
  if (!back) return sbv + hdr + cnt;
  return (last ? tot : sbv + hdr) - cnt;
}

// rank_d(i) of one level by ONE thread (the block's first i mod 1024 digits
// streamed 16 B at a time): the host API's scalar step and the few keys the
// transition table left out, never a batched path.
__device__ __forceinline__ uint64_t rank_w2_thread(const W2Level& L, uint64_t i, uint32_t d) {
  const uint64_t b = i >> kW2BlkLog2;
  const uint32_t k = (uint32_t)(i & (kW2Blk - 1));
  const uint8_t* base = L.blocks + b * L.blk_bytes;
  const uint32_t R = 1u << L.bits;
  uint64_t cnt = L.sb[(i >> kW2SbLog2) * R + d] + reinterpret_cast<const uint16_t*>(base)[d];
  const uint4* p = reinterpret_cast<const uint4*>(base + 2 * R);
  const uint32_t per = L.bits > 8 ? 8u : 16u;   // digits per 16 B
  for (uint32_t j0 = 0; j0 < k; j0 += per) {
    const uint4 x = p[j0 / per];
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) {
      const bool wide = L.bits > 8;
      const uint32_t dig = wide ? (w[(j >> 1) & 3] >> (16 * (j & 1))) & 0xFFFFu : (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      cnt += ((!wide || j < 8) && j0 + j < k && dig == d) ? 1u : 0u;
    }
  }
  return cnt;
}

// LF of both ends of [l, r) by symbol c (every level of the 2-level matrix) by
// one thread: [C[c] + rank_c(l), C[c] + rank_c(r)).
__device__ __forceinline__ void descend_w2_thread(const DevView& v, uint32_t c, uint64_t& l, uint64_t& r) {
  for (uint32_t lev = 0; lev < v.NL2; ++lev) {
    const W2Level& L = v.w2[lev];
    const uint32_t d = (c >> L.shift) & ((1u << L.bits) - 1u);
    const uint64_t z = L.Z[d];
    l = z + rank_w2_thread(L, l, d);
    r = z + rank_w2_thread(L, r, d);
  }
  l = (uint64_t)((int64_t)l + v.D2[c]);
  r = (uint64_t)((int64_t)r + v.D2[c]);
}

// LF step of a narrow range by a whole wave: E[lo, hi) is scanned (8 entries
// per lane, ONE round trip -- and usually L2 / Infinity-Cache hits, the rows
// the previous decode step streamed): the occurrences of c map to consecutive
// LF values, so the new range is [LF(first c), LF(last c) + 1).
// (precondition: v.E, 0 < hi - lo <= kENarrow, hi <= n, 0 <= sym <= max_sym)
// CONTENT: also read E2 with E, and return in content[j] / bit j of cmask the
// symbols BWT[LF(i)] of this lane's matching entries -- the new range's whole
// content (LF maps the matches onto it one to one), with no further load.
template <bool CONTENT>
__device__ __forceinline__ void lf_step_fast(const DevView& v, int64_t sym, uint64_t& lo, uint64_t& hi,
                                             uint32_t* content, uint32_t& cmask) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t c = (uint64_t)sym;
  uint64_t e[kENarrow / 64];
#pragma unroll
  for (uint32_t j = 0; j < kENarrow / 64; ++j) {
    // clamped, unconditional load, padded afterwards: a guarded load is sunk
    // into a branch with a vmcnt(0) behind it (one round trip per j)
    const uint64_t idx = lo + lane + 64 * j;
    const uint64_t x = v.E[idx < hi ? idx : hi - 1];
    if (CONTENT) content[j] = v.E2[idx < hi ? idx : hi - 1];
    e[j] = x | (idx < hi ? 0ull : ~0ull);
  }
  if (CONTENT) {
    // the E2 words are consumed here, with E's (zeroed unless matched): left
    // unused until the emit, their loads were sunk past the plan barrier --
    // one more round trip, which is what E2 exists to remove
    cmask = 0;
#pragma unroll
    for (uint32_t j = 0; j < kENarrow / 64; ++j) {
      const bool m = e[j] != ~0ull && (e[j] >> kESymShift) == c;
      cmask |= m ? (1u << j) : 0u;
      content[j] = m ? content[j] : 0u;
    }
  }
  uint64_t fmin = ~0ull, fmax = 0, lfmin = 0, lfmax = 0;   // first / last match (relative index + 1)
#pragma unroll
  for (uint32_t j = 0; j < kENarrow / 64; ++j) {
    if (e[j] != ~0ull && (e[j] >> kESymShift) == c) {
      const uint64_t r = lane + 64 * j + 1;
      if (r < fmin) {
        fmin = r;
        lfmin = e[j] & kELfMask;
      }
      if (r > fmax) {
        fmax = r;
        lfmax = e[j] & kELfMask;
      }
    }
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t om = __shfl_xor(fmin, d, 64), ol = __shfl_xor(lfmin, d, 64);
    const uint64_t xm = __shfl_xor(fmax, d, 64), xl = __shfl_xor(lfmax, d, 64);
    if (om < fmin) {
      fmin = om;
      lfmin = ol;
    }
    if (xm > fmax) {
      fmax = xm;
      lfmax = xl;
    }
  }
  if (fmax == 0) {
    lo = 0;
    hi = 0;
    return;
  }
  lo = lfmin;
  hi = lfmax + 1;
}

// ---------------------------------------------------------------------------
// range-bitmap cache lookup
__host__ __device__ __forceinline__ uint64_t cache_hash(uint64_t lo, uint64_t hi) {
  uint64_t x = lo * 0x9E3779B97F4A7C15ull ^ (hi + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  return x ^ (x >> 32);
}

constexpr uint64_t kCacheEmpty = ~0ull;
constexpr uint32_t kCacheIdShift = 34;

// Bitmap of [lo, hi) if cached, else null.  Called by all 64 lanes of a wave
// with uniform (lo, hi): lanes 0-15 read 16 consecutive probe slots (256 B) per
// round; linear probing stops at the first empty slot.
__device__ __forceinline__ const uint32_t* cache_find(const DevView& v, uint64_t lo, uint64_t hi) {
  if (!v.cache_mask || hi - lo < v.cache_min) return nullptr;
  const uint32_t lane = threadIdx.x & 63u;
  uint64_t slot = cache_hash(lo, hi) & v.cache_mask;
  for (int round = 0; round < 64; ++round) {
    uint64_t klo = kCacheEmpty, khi = 0;
    if (lane < 16) {
      const uint64_t* e = v.cache_tab + 2 * ((slot + lane) & v.cache_mask);
      klo = e[0];
      khi = e[1];
    }
    const bool hit = lane < 16 && klo == lo && (khi & ((1ull << kCacheIdShift) - 1)) == hi;
    const bool empty = lane < 16 && klo == kCacheEmpty;
    const uint64_t bh = __ballot(hit), be = __ballot(empty);
    if (bh && (!be || __ffsll((long long)bh) < __ffsll((long long)be))) {
      const uint32_t src = (uint32_t)__ffsll((long long)bh) - 1;
      const uint64_t id = __shfl(khi, (int)src, 64) >> kCacheIdShift;
      return v.cache_bm + id * v.bm_words;
    }
    if (be) return nullptr;
    slot += 16;
  }
  return nullptr;
}

__host__ __device__ __forceinline__ uint64_t trans_hash(uint64_t lo, uint64_t hi, uint64_t c) {
  return cache_hash(lo ^ (c * 0xD6E8FEB86659FD93ull), hi + c);
}

// Transition slot (16 B) in buckets of kTransBucket = 8 slots -- 128 B, one line -- with two-choice
// hashing: a key sits in one of the 8 slots of its bucket A or of its bucket B (k_trans_insert fills
// the emptier of the two; a key finding both full is left out and takes the descent), so a probe
// reads 16 slots in two 128-B lines.  The key is (the parent's CACHE ID, symbol): every parent is a
// cached range, and a probe reads the parent's range-cache run in the same round trip, so its id is
// there to compare with (the round-5 slot kept the parent's (lo, hi) itself: 24 B).
//   w0 = pid | c << 20 | kind << 38 | (clo & (2^24 - 1)) << 40        (empty slot: ~0)
//   w1 = clo >> 24 | cw << 10 | aux << 44
// kind 0: the child range [clo, clo + cw) alone; 1: aux = its only symbol (a one-row child);
// 2: aux = its cache id (a cached child: its bitmap).  pid < 2^20 - 1 (kTPidNone is the empty
// slot's), c < 2^18, aux < 2^20: keys outside these are left out (the descent).
constexpr uint32_t kTSymShift = 20;
constexpr uint64_t kTPidNone = (1ull << 20) - 1;
constexpr uint64_t kTSymLimit = 1ull << 18;
constexpr uint64_t kTKeyMask = (1ull << 38) - 1;
constexpr uint32_t kTKindOne = 1, kTKindCached = 2;
constexpr uint64_t kTAuxLimit = 1ull << 20;
constexpr uint32_t kTransBucket = 8;
constexpr uint32_t kTransProbe = 2 * kTransBucket;   // a key's candidate slots: bucket A's, then bucket B's
// DevView::probe_first bit 1.  The insert leaves a key out only when both of its buckets are
// full, and a bucket's fill never shrinks; so when the table was built with every child of every
// cached parent (transitions = 2, trans_min = 1, no parent skipped), a probe that finds the
// parent's id, no matching key and a free slot among its 16 has proved the symbol absent from the
// parent's range -- the step ends after the probe, without the parent's bitmap word.
constexpr uint32_t kProbeComplete = 2;
constexpr uint64_t kTransEmpty = ~0ull;
constexpr uint64_t kTransSlotBytes = 16;
constexpr uint64_t kMask34 = (1ull << 34) - 1;

__host__ __device__ __forceinline__ uint64_t trans_key(uint64_t pid, uint64_t c) { return pid | (c << kTSymShift); }
__host__ __device__ __forceinline__ bool trans_match(uint64_t w0, uint64_t key) { return (w0 & kTKeyMask) == key; }
__host__ __device__ __forceinline__ uint64_t trans_clo(uint64_t w0, uint64_t w1) {
  return (w0 >> 40) | ((w1 & 0x3FFull) << 24);
}
__host__ __device__ __forceinline__ uint64_t trans_cw(uint64_t w1) { return (w1 >> 10) & kMask34; }
__host__ __device__ __forceinline__ uint32_t trans_kind(uint64_t w0) { return (uint32_t)((w0 >> 38) & 3u); }
__host__ __device__ __forceinline__ uint64_t trans_aux(uint64_t w1) { return w1 >> 44; }

__host__ __device__ __forceinline__ uint64_t mul_hi64(uint64_t a, uint64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

struct TransHome {
  uint64_t a, b;   // first slots of the key's two buckets (cap = the table's slots, a multiple of 8)
};
__host__ __device__ __forceinline__ TransHome trans_home(uint64_t lo, uint64_t hi, uint64_t c, uint64_t cap) {
  const uint64_t h = trans_hash(lo, hi, c);
  uint64_t g = (h ^ (h >> 31)) * 0x94D049BB133111EBull;   // a second, independent bucket index
  g ^= g >> 29;
  const uint64_t nb = cap / kTransBucket;
  return TransHome{mul_hi64(h, nb) * kTransBucket, mul_hi64(g, nb) * kTransBucket};
}
// candidate k (0 .. kTransProbe - 1) of a key
__host__ __device__ __forceinline__ uint64_t trans_slot(const TransHome& t, uint32_t k) {
  return k < kTransBucket ? t.a + k : t.b + (k - kTransBucket);
}

// The LF step of the batched kernels, by all 64 lanes of a wave (uniform
// inputs), with exactly one inlined copy of each path (a kernel's code is
// fetched cold into the instruction cache at every launch, so duplicated
// inlined paths cost fetch latency on the dependent chain):
//   * full range: [C[c], C[c+1]) ([sdsl] backward_search shortcut), with the
//     C-block's cached bitmap (cblock) read in the same round trip;
//   * <= kENarrow rows: one scan of E[lo, hi) (lf_step_fast);
//   * otherwise the wavelet-matrix descent (NL2 round trips); a cached range
//     also probes the transition table, issued with the first descent level
//     -- a hit ends the step after one round trip and names the child's
//     bitmap in *cbm (else null) or, for a one-row child, its only symbol in
//     *one (else -1).
template <bool CONTENT = false>
__device__ __forceinline__ void lf_step_decode(const DevView& v, int64_t sym, uint64_t& lo, uint64_t& hi,
                                               const uint32_t*& cbm, int64_t& one, uint32_t* content = nullptr,
                                               uint32_t* cmask = nullptr) {
  cbm = nullptr;
  one = -1;
  if (CONTENT) *cmask = 0;
  if (hi > v.n) hi = v.n;
  if (lo >= hi || sym < 0 || (uint64_t)sym > v.max_sym) {
    lo = 0;
    hi = 0;
    return;
  }
  const uint32_t c32 = (uint32_t)sym;
  if (lo == 0 && hi == v.n) {   // the C-block, and its cached bitmap id in the same round trip
    const uint64_t a = v.C[c32], b = v.C[c32 + 1];
    const uint32_t cid = v.cblock ? v.cblock[c32] : 0u;
    lo = a < b ? a : 0;
    hi = a < b ? b : 0;
    if (cid && a < b) cbm = v.cache_bm + (uint64_t)(cid - 1) * v.bm_words;
    return;
  }
  if (v.E && hi - lo <= kENarrow) {
    uint32_t cm = 0;
    if (CONTENT && v.E2) {
      lf_step_fast<true>(v, sym, lo, hi, content, cm);
      *cmask = cm | kContentPath;
    } else {
      lf_step_fast<false>(v, sym, lo, hi, nullptr, cm);
    }
    return;
  }
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t q = lane & 31u;
  const bool side = lane >= 32;
  const uint64_t c = (uint64_t)sym;
  // (1) transition probe of a cached range: its 16 candidate slots x 2 words, one word per lane
  // 0-31; lanes 32-63 read the parent's own home run in the range cache (16 slots x 2 words) in
  // the same round trip -- the parent's cache id, which the slots' keys hold
  const bool probe = v.trans_cap && hi - lo >= v.cache_min;
  uint64_t tw = kTransEmpty;
  if (probe && lane < 2 * kTransProbe) {
    const uint64_t slot = trans_slot(trans_home(lo, hi, c, v.trans_cap), lane / 2);
    tw = v.trans_tab[2 * slot + (lane & 1u)];
  } else if (probe && v.cache_mask) {
    const uint32_t k = lane - 2 * kTransProbe;
    tw = v.cache_tab[2 * ((cache_hash(lo, hi) + k / 2) & v.cache_mask) + (k & 1)];
  }
  // the parent's cache id (kTPidNone: not in the run read -- no key can match, the descent serves)
  auto parent_id = [&](uint64_t w1n) -> uint64_t {
    const uint64_t bc = __ballot(lane >= 2 * kTransProbe && (lane & 1u) == 0 && tw == lo && (w1n & kMask34) == hi);
    return bc ? __shfl(w1n, __ffsll((long long)bc) - 1, 64) >> kCacheIdShift : kTPidNone;
  };
  // a hit: the child's range, and its bitmap (cached) or only symbol
  auto take_hit = [&](uint64_t bh) {
    const int src = __ffsll((long long)bh) - 1;
    const uint64_t w0 = __shfl(tw, src, 64), w1 = __shfl(tw, src + 1, 64);
    const uint64_t clo = trans_clo(w0, w1);
    lo = clo;
    hi = clo + trans_cw(w1);
    const uint32_t kind = trans_kind(w0);
    if (kind == kTKindOne)
      one = (int64_t)trans_aux(w1);
    else if (kind == kTKindCached)
      cbm = v.cache_bm + trans_aux(w1) * v.bm_words;
  };
  // A probe miss is a symbol the parent lacks -- or one of the few keys the
  // table left out.  The parent's cached bitmap tells which: its word for c
  // is loaded with the descent's first level, and an absent c ends the step
  // there (one round trip after the probe instead of the whole descent).
  uint32_t pword = ~0u;
  if (probe && (v.probe_first & 1u)) {   // the probe alone: one round trip of 256 B + the run for a hit
    const uint64_t w1n = __shfl_down(tw, 1, 64);
    const uint64_t pid = parent_id(w1n);
    const uint64_t key = trans_key(pid, c);
    // (a parent id of 2^20 - 1 or more is never a key: trans_key would spill into the symbol bits)
    const bool keyed = pid < kTPidNone && c < kTSymLimit;
    const bool even = lane < 2 * kTransProbe && (lane & 1u) == 0;
    const uint64_t bh = __ballot(even && keyed && trans_match(tw, key));
    if (bh) {
      take_hit(bh);
      return;
    }
    if (keyed && (v.probe_first & kProbeComplete) && __ballot(even && tw == kTransEmpty)) {
      lo = 0;   // c is absent from the parent's range (kProbeComplete)
      hi = 0;
      return;
    }
    if (pid < kTPidNone) pword = v.cache_bm[pid * v.bm_words + (c32 >> 5)];
  }
  // (2) level-independent loads, then the descent
  const int64_t dd = v.D2[c32];
  uint64_t z[kW2MaxLevels];
#pragma unroll
  for (int l = 0; l < kW2MaxLevels; ++l)
    z[l] = (l < (int)v.NL2) ? v.w2[l].Z[(c32 >> v.w2[l].shift) & ((1u << v.w2[l].bits) - 1u)] : 0;
  uint64_t pos = side ? hi : lo;
#pragma unroll 1
  for (int l = 0; l < (int)v.NL2; ++l) {
    const uint32_t d = (c32 >> v.w2[l].shift) & ((1u << v.w2[l].bits) - 1u);
    const uint64_t r = rank_w2(v.w2[l], pos, d, q);
    if (l == 0 && !((pword >> (c32 & 31u)) & 1u)) {   // the parent's bitmap lacks c
      lo = 0;
      hi = 0;
      return;
    }
    if (l == 0 && probe && !(v.probe_first & 1u)) {   // the probe's loads were issued before this level's
      const uint64_t w1n = __shfl_down(tw, 1, 64);
      const uint64_t pid = parent_id(w1n);
      const uint64_t key = trans_key(pid, c);
      const uint64_t bh = __ballot(lane < 2 * kTransProbe && (lane & 1u) == 0 && pid < kTPidNone &&
                                   c < kTSymLimit && trans_match(tw, key));
      if (bh) {
        take_hit(bh);
        return;
      }
    }
    pos = z[l] + r;
  }
  const uint64_t other = __shfl_xor(pos, 32, 64);
  const uint64_t l2 = side ? other : pos, h2 = side ? pos : other;
  if (l2 >= h2) {
    lo = 0;
    hi = 0;
    return;
  }
  lo = (uint64_t)((int64_t)l2 + dd);
  hi = (uint64_t)((int64_t)h2 + dd);
}

// ---------------------------------------------------------------------------
// suffix-array / inverse-suffix-array samples (locate.hip): text-order
// sampling at sdsl csa_wt's default rates
constexpr uint64_t kSaRate = 32;
constexpr uint64_t kIsaRate = 64;
struct SampleView {
  const uint64_t* mark;       // n bits: SA[i] % kSaRate == 0
  const uint64_t* mark_cnt;   // marked rows before each 512-row block
  const uint32_t* sa_samp;    // SA[i] / kSaRate of the marked rows, row order
  const uint64_t* isa_samp;   // row of text position kIsaRate * k
};

// ---------------------------------------------------------------------------
// Index-structure options (fm_build_options, include/fmidx.h), resolved: the
// profile's values, then the caller's explicit fields, then the
// FMIDX_BUILD_OPTIONS overrides ("key=value,..."; options.cpp).
struct BuildOpts {
  int32_t profile = 0;          // 0 default, 1 compact
  int32_t transitions = 2;      // 0 none, 1 cached children only, 2 every child of a cached range
  int32_t lf_e = 1;             // the E array
  int32_t lf_e2 = 0;            // BWT[LF(i)] beside E
  int32_t probe_first = 1;      // a cached range's LF step waits for its transition probe
  int32_t keep_bwt = 0;         // keep the plain BWT although E holds its symbols
  int32_t follow_bitmaps = 0;   // per-symbol C-block bitmaps
  int32_t bm_log2 = -1;         // aligned bitmap block; -1: by n
  int32_t trans_min = 1;        // transitions = 2: the children of >= trans_min occurrences
  uint64_t cache_min = 4096;    // range-bitmap cache threshold (rows)
  uint64_t cache_mb = 48ull << 10;
  uint64_t trans_mb = 72ull << 10;
  uint64_t gpu_sort_min = 1ull << 20;
};
BuildOpts build_profile(int profile);
// the FMIDX_BUILD_OPTIONS overrides applied to o (0, or -1 + set_error on a malformed string)
int apply_build_overrides(BuildOpts& o);

// Launch tuning of the query kernels, process-wide (fm_tuning): library
// defaults, then fm_set_tuning, with FMIDX_TUNING overrides on top.
struct Tuning {
  uint32_t lf_group = 2;         // lanes per row of LF launches above lf_group_min rows (64 = never group)
  uint32_t search_group = 1;     // the same for get_range launches
  uint32_t dec_threads = 0;      // decode workgroup size; 0 = by batch
  uint32_t mask_slices = 0;      // decode slices per row; 0 = by the wave budget
  uint64_t lf_group_min = 8192;
  int32_t lf_work = -1;          // -1 by row count, 0 grouped kernel, 1 worklist + tail, 2 in-wave sweep,
                                 // 4 persistent sweep (heads, then a shared tail-queue drain)
  int32_t lf_gprobe = 1;
  int32_t lf_quad = 1;
  int32_t lf_split = 0;
  int32_t search_p8 = 1;
  uint64_t lf_sweep_min = 1ull << 18;
  uint64_t sa_chunk = 1ull << 29;
};
const Tuning& tuning();
// replaces the process tuning (FMIDX_TUNING overrides on top); 0 or -1 + set_error
int set_tuning(const Tuning& t);

// ---------------------------------------------------------------------------
// host-side owner of the device structures
struct Index {
  BuildOpts opts;                // resolved index-structure options (kept across release())
  int device = 0;
  hipStream_t stream = nullptr;  // internal stream for host-API calls
  DevView view{};
  uint64_t n = 0;
  uint64_t sigma = 0;            // distinct symbols in the BWT
  uint64_t max_sym = 0;
  uint32_t L = 0;
  // device allocations
  uint64_t* C = nullptr;
  uint32_t* bwt = nullptr;        // freed after the build when E holds the symbols
  uint32_t* bwt_view = nullptr;   // materialised on request (fm_device_bwt) when bwt is freed
  uint32_t* bm = nullptr;
  uint32_t* bm_full = nullptr;
  uint32_t* bm_follow = nullptr;
  uint8_t* w2_blocks[kW2MaxLevels] = {nullptr, nullptr, nullptr};
  uint64_t* w2_sb[kW2MaxLevels] = {nullptr, nullptr, nullptr};
  uint64_t* w2_Z = nullptr;
  uint64_t* E = nullptr;
  uint32_t* E2 = nullptr;
  uint32_t* cache_bm = nullptr;
  uint64_t* cache_tab = nullptr;
  uint64_t* trans_tab = nullptr;
  uint32_t* cblock = nullptr;
  uint64_t cache_nodes = 0, cache_bytes = 0, trans_entries = 0, trans_dropped = 0, trans_bytes = 0;
  int64_t* D2 = nullptr;
  uint64_t* sa = nullptr;         // legacy (v1 files / no samples): full suffix array
  uint32_t* text = nullptr;       // legacy: T' (extract without ISA samples)
  uint64_t* mark = nullptr;       // SA / ISA samples (locate.hip)
  uint64_t* mark_cnt = nullptr;
  uint32_t* sa_samp = nullptr;
  uint64_t* isa_samp = nullptr;
  uint64_t samp_bytes = 0;
  uint64_t bm_bytes = 0, follow_bytes = 0, w2_bytes = 0;
  SampleView samples() const { return SampleView{mark, mark_cnt, sa_samp, isa_samp}; }
  // grow-only workspace for batched traversals
  void* ws = nullptr;
  size_t ws_bytes = 0;
  bool built = false;
  void release();
};

// build.hip
int device_build_from_bwt(Index* h, const uint32_t* d_bwt_owned, uint64_t n, hipStream_t s);
int device_bwt_view(Index* h, const uint32_t** out);
int device_build_w2(Index* h, const uint32_t* d_bwt, uint64_t n, hipStream_t s);
int device_build_cache(Index* h, hipStream_t s);   // cache.hip
int device_build_lfe(Index* h, const uint32_t* d_bwt, uint64_t n, hipStream_t s);
int exclusive_scan_u64(const uint64_t* d_in, uint64_t* d_out, uint64_t n, hipStream_t s,
                       uint64_t* d_total);

// locate.hip: samples from a device suffix array (uint64[n]); from loaded samples
int device_build_samples(Index* h, const uint64_t* d_sa, uint64_t n, hipStream_t s);
int device_finish_samples(Index* h, uint64_t n, hipStream_t s);
// locate.hip: samples of an index built from a BWT, from ISA samples (isa[k] = row of position 64 k)
int device_samples_from_isa(Index* h, const uint64_t* d_isa, uint64_t nisa, hipStream_t s);
int launch_locate(const DevView& v, const SampleView& sv, const uint64_t* rows, uint64_t m, uint64_t* out,
                  hipStream_t s);
int launch_extract(const DevView& v, const SampleView& sv, const uint64_t* begin, const uint64_t* end,
                   const uint64_t* off, uint64_t m, uint64_t* out, hipStream_t s);

// query.hip launchers
// re-reads the LF / search launch variants from the environment (query.hip)
void reload_lf_tuning();
// locate.hip: rows of the positions that are multiples of kSaRate, from ISA samples
int launch_isa_walk(const DevView& v, const uint64_t* isa, uint64_t nisa, uint64_t* rows_out, hipStream_t s);
// ws: workspace of lf_ws_bytes(m) bytes for the worklist sweeps (null: the grouped kernels)
int launch_lf_step(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                   const uint64_t* lo, const uint64_t* hi, uint64_t* lo_out, uint64_t* hi_out,
                   uint64_t m, hipStream_t s, void* ws = nullptr);
size_t lf_ws_bytes(uint64_t m);   // 0: this launch takes no workspace
// the persistent LF sweep (tuning lf_work 4): whether it serves m rows, its own workspace (zeroed
// when allocated, never shared), the launch (epoch: nonzero, new per launch), the error word's offset
bool lf_persist(uint64_t m);
size_t lf_persist_ws_bytes(uint64_t m);
size_t lf_persist_err_offset();
int launch_lf_persist(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below, const uint64_t* lo,
                      const uint64_t* hi, uint64_t* lo_out, uint64_t* hi_out, uint64_t m, hipStream_t s, void* ws,
                      size_t ws_bytes, uint32_t epoch, int dev);
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
// the same step writing the shard exchange's payload with fixed row slots (PeerExchange)
int launch_decode_payload(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                          const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out, uint64_t* hi_out,
                          uint64_t m, uint32_t* pay, uint64_t cap, uint64_t vocab, uint32_t* pay_alt,
                          const uint32_t* pay_sel, hipStream_t s, const uint64_t* sig_dst = nullptr,
                          uint64_t sig_world = 0, uint32_t* sig_done = nullptr);
int launch_cache_probe(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m, uint8_t* out,
                       hipStream_t s);
int launch_follow_bitmaps(const DevView& v, const uint64_t* C, uint64_t nsym, uint32_t* out,
                          hipStream_t s);
int launch_distinct(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                    const uint64_t* cap_off, uint64_t* syms, uint64_t* counts, uint64_t* k,
                    void* ws, uint64_t total_cap, hipStream_t s, uint64_t min_count = 1,
                    uint64_t* child_lo = nullptr);
size_t distinct_ws_bytes(uint64_t total_cap);
// dense CSR (off[m + 1], interleaved (symbol, count) pairs) of launch_distinct's output
int launch_distinct_csr(const uint64_t* k, const uint64_t* cap_off, const uint64_t* syms, const uint64_t* counts,
                        uint64_t m, uint64_t* off, uint64_t* pairs, hipStream_t s);

// shard.hip: OR of the shards' packed allowed rows (+ expansion to uint8)
// The exchange payload's header (uint32 words): [0] total words [1] B [2] W [3] magic, desc[B] and
// off[B] from word 4 (padded to 4 words), then the processors' facts area -- facts[k * B + b], k = 0..2
// (count([last]) > 0, range non-empty, distinct non-empty: 0/1; zeros when the payload carries none)
// -- padded to 4 words; row data after it.
__host__ __device__ __forceinline__ uint64_t payload_facts_at(uint64_t B) { return 4 + ((2 * B + 3) & ~3ull); }
__host__ __device__ __forceinline__ uint64_t payload_header_words(uint64_t B) {
  return payload_facts_at(B) + ((3 * B + 3) & ~3ull);
}
uint64_t shard_payload_capacity(uint64_t B, uint64_t vocab);
int launch_shard_pack(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t B, const uint32_t* bits,
                      uint64_t ldw, uint64_t vocab, const int32_t* facts, uint32_t* pay, uint64_t cap, hipStream_t s);
int launch_shard_or_rows(const uint32_t* parts, uint64_t nparts, uint64_t stride, uint64_t B, uint64_t vocab,
                         int64_t shift, void* out, uint64_t ld, int unpack, int32_t* facts_out, hipStream_t s);
int launch_shard_or_rows_peers(const uint64_t* ptrs, uint64_t nparts, uint64_t cap, uint64_t B, uint64_t vocab,
                               int64_t shift, void* out, uint64_t ld, int unpack, const uint32_t* flags,
                               const uint32_t* ctr, uint32_t spins, uint32_t* err, int32_t* facts_out, hipStream_t s);
int launch_peer_signal(const uint64_t* dst, uint64_t world, uint32_t* ctr, hipStream_t s);
int launch_or_bits(const uint32_t* parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t wpr,
                   uint64_t vocab, void* out, uint64_t ld_out, int unpack, hipStream_t s);

// probe.hip (bench roofline): random 64-B gathers / dependent chase
int launch_probe_gather(const void* buf, uint64_t bytes, int chase, uint64_t loads, uint32_t threads_or_chains,
                        uint64_t* sink, hipStream_t s);

// epilogue.hip
int gpu_suffix_sort(const uint32_t* text, uint64_t n, uint32_t* bwt_out, uint64_t* sa_out, hipStream_t s);
int gpu_wt_int_levels(const uint32_t* bwt, uint64_t n, uint32_t L, uint64_t* words, hipStream_t s);
int launch_epilogue(int dtype, const void* scores, void* out, uint64_t B, uint64_t V, uint64_t lds,
                    uint64_t ldo, const uint32_t* bits, uint64_t ldb, const uint32_t* uni,
                    const void* row_params, int64_t eos, hipStream_t s);

void set_error(const char* fmt, ...);

// FMIDX_BUILD_TIMES=1: construction phases report their wall time on stderr.
double build_clock();                                   // seconds, monotonic
void build_phase(const char* name, double t0, hipStream_t s);   // syncs s and prints when enabled

}  // namespace fmidx

#define FM_HIP(expr)                                                                    \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::fmidx::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
      return -1;                                                                        \
    }                                                                                   \
  } while (0)
