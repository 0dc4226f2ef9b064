// sa.hip -- index construction on the GPU.
//
// The reference builds its index with sdsl construct_im / construct
// (cpp_modules_linux/fm_index.cpp:33-48), i.e. divsufsort on the host; for an
// enwiki-scale corpus (n ~ 4-6e9 tokens) that needs 64-bit positions and more
// host memory than a node has to spare.  Here the suffix array of T' is built
// in HBM by prefix doubling with discarding:
//
//   init   sort positions by their first symbol (radix sort, keys = T' itself,
//          values = a counting iterator): SA grouped by 1-symbol prefixes,
//          rank[p] = start of p's group (an SA index).
//   round  for every suffix still in a group of size > 1 ("active"), key2 =
//          the next 2 symbols (first round) or rank[p + h]; sort each group by
//          key2; split groups where key2 changes; new rank = new group start;
//          drop suffixes whose group became a singleton.  h: 1 -> 3 -> 6 -> ...
//
// Active suffixes are processed in chunks of whole groups (<= 2^29 suffixes,
// a larger group is a chunk of its own), so one 64-bit radix key holds
// (group ordinal within the chunk << 34 | key2) and the working set is
// bounded: T' (4n) + SA (8n) + rank (8n) + active list (8n) + head flags (n)
// + 4 chunk buffers.  Ranks are only rewritten after every chunk of a round
// has read them (phase 1: sort + split, phase 2: rank update + compaction).
// Requires n < 2^34 and symbols < 2^26.
//
// The same file exports wt_int-compatible level bit vectors (the levelwise
// wavelet tree sdsl's csa_wt_int<> stores; level l = the BWT stably sorted by
// its top l bits), used to feed the CPU baseline at full scale.
#include "fmidx_internal.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>
#include <rocprim/functional.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace fmidx {

namespace {

constexpr int kT = 256;
constexpr uint32_t kKey2Bits = 34;

inline unsigned grid_for(uint64_t n) {
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + kT - 1) / kT, 1u << 18));
}

template <typename T>
struct Buf {
  T* p = nullptr;
  size_t count = 0;
  Buf() = default;
  Buf(const Buf&) = delete;
  ~Buf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    count = 0;
  }
  int alloc(size_t c) {
    release();
    if (c == 0) c = 1;
    FM_HIP(hipMalloc(reinterpret_cast<void**>(&p), c * sizeof(T)));
    count = c;
    return 0;
  }
  int reserve(size_t c) { return c <= count ? 0 : alloc(c); }
};

#define GRID_STRIDE(i, n) \
  for (uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x; i < (n); i += (uint64_t)gridDim.x * kT)

__global__ void __launch_bounds__(kT) k_sa_check(const uint32_t* __restrict__ t, uint64_t n,
                                                  unsigned long long* zeros, uint32_t* maxsym) {
  uint32_t mx = 0;
  unsigned long long z = 0;
  GRID_STRIDE(i, n) {
    const uint32_t v = t[i];
    mx = max(mx, v);
    z += (v == 0);
  }
  if (z) atomicAdd(zeros, z);
  atomicMax(maxsym, mx);
}

// group boundaries of the symbol-sorted keys
__global__ void __launch_bounds__(kT) k_sa_bounds(const uint32_t* __restrict__ keys, uint64_t n,
                                                   uint64_t* __restrict__ start, uint64_t* __restrict__ end) {
  GRID_STRIDE(j, n) {
    const uint32_t c = keys[j];
    if (j == 0 || keys[j - 1] != c) start[c] = j;
    if (j + 1 == n || keys[j + 1] != c) end[c] = j + 1;
  }
}

__global__ void __launch_bounds__(kT) k_sa_init(const uint32_t* __restrict__ text, const uint32_t* __restrict__ keys,
                                                 uint64_t n, const uint64_t* __restrict__ start,
                                                 const uint64_t* __restrict__ end, uint64_t* __restrict__ rank,
                                                 uint8_t* __restrict__ active) {
  GRID_STRIDE(i, n) {
    rank[i] = start[text[i]];
    const uint32_t c = keys[i];
    active[i] = (end[c] - start[c]) > 1;
  }
}

// One thread: the end of the chunk starting at active index s, given the
// tentative end e (< A): e moved back to the start of the group containing
// it, or -- when that group starts at s -- forward to the group's end.
__global__ void k_sa_chunk_end(const uint64_t* __restrict__ act, const uint64_t* __restrict__ sa,
                               const uint64_t* __restrict__ rank, uint64_t s, uint64_t e, uint64_t A,
                               uint64_t* out) {
  const uint64_t G = rank[sa[act[e]]];
  uint64_t lo = s, hi = e;
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (act[mid] < G) lo = mid + 1; else hi = mid;
  }
  if (lo > s) {
    *out = lo;
    return;
  }
  lo = e + 1;
  hi = A;
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (rank[sa[act[mid]]] == G) lo = mid + 1; else hi = mid;
  }
  *out = lo;
}

// Phase 1a: keys and values of one chunk.
__global__ void __launch_bounds__(kT) k_sa_gather(const uint64_t* __restrict__ act, uint64_t m,
                                                   const uint64_t* __restrict__ sa,
                                                   const uint64_t* __restrict__ rank,
                                                   const uint32_t* __restrict__ text, uint64_t n, uint64_t h,
                                                   int first, uint32_t tpk, uint32_t bits,
                                                   uint64_t* __restrict__ key, uint64_t* __restrict__ val,
                                                   uint64_t* __restrict__ gstart) {
  GRID_STRIDE(k, m) {
    const uint64_t j = act[k];
    const uint64_t p = sa[j];
    gstart[k] = (rank[p] == j) ? 1 : 0;
    uint64_t v;
    if (first) {
      v = 0;
      for (uint32_t t = 1; t <= tpk; ++t) {
        const uint64_t q = p + t;
        v = (v << bits) | (q < n ? text[q] : 0u);
      }
    } else {
      v = rank[p + h];   // p + h < n for every active suffix (shorter ones hold the sentinel)
    }
    key[k] = v;
    val[k] = p;
  }
}

// Phase 1b: prepend the group ordinal (inclusive count of group starts - 1).
__global__ void __launch_bounds__(kT) k_sa_pack(uint64_t* __restrict__ key, const uint64_t* __restrict__ ord,
                                                 uint64_t m) {
  GRID_STRIDE(k, m) key[k] |= (ord[k] - 1) << kKey2Bits;
}

// Phase 1c: write the sorted suffixes back and mark the new group heads.
__global__ void __launch_bounds__(kT) k_sa_scatter(const uint64_t* __restrict__ act, uint64_t m,
                                                    const uint64_t* __restrict__ key,
                                                    const uint64_t* __restrict__ val, uint64_t* __restrict__ sa,
                                                    uint8_t* __restrict__ head) {
  GRID_STRIDE(k, m) {
    sa[act[k]] = val[k];
    head[k] = (k == 0 || key[k] != key[k - 1]) ? 1 : 0;
  }
}

// Phase 2a: head positions for the max-scan (act is ascending, so max = last head).
__global__ void __launch_bounds__(kT) k_sa_headval(const uint64_t* __restrict__ act,
                                                    const uint8_t* __restrict__ head, uint64_t m,
                                                    uint64_t* __restrict__ out) {
  GRID_STRIDE(k, m) out[k] = head[k] ? act[k] : 0;
}

// Phase 2b: new ranks; keep only suffixes still in a group of size > 1.
__global__ void __launch_bounds__(kT) k_sa_rank(const uint64_t* __restrict__ act, const uint8_t* __restrict__ head,
                                                 uint64_t m, const uint64_t* __restrict__ sa,
                                                 const uint64_t* __restrict__ newg, uint64_t* __restrict__ rank,
                                                 uint8_t* __restrict__ keep) {
  GRID_STRIDE(k, m) {
    rank[sa[act[k]]] = newg[k];
    const bool next_head = (k + 1 == m) || head[k + 1];
    keep[k] = (head[k] && next_head) ? 0 : 1;
  }
}

__global__ void __launch_bounds__(kT) k_sa_bwt(const uint32_t* __restrict__ text, const uint64_t* __restrict__ sa,
                                                uint64_t n, uint32_t* __restrict__ bwt) {
  GRID_STRIDE(j, n) {
    const uint64_t p = sa[j];
    bwt[j] = text[p == 0 ? n - 1 : p - 1];
  }
}

// 64 consecutive sorted keys -> one word of level bits (bit b of the key).
__global__ void __launch_bounds__(kT) k_level_bits(const uint32_t* __restrict__ keys, uint64_t n, uint32_t b,
                                                    uint64_t* __restrict__ words) {
  const uint64_t nw = (n + 63) / 64;
  GRID_STRIDE(w, nw) {
    uint64_t x = 0;
    const uint64_t base = w * 64;
    const uint64_t lim = min<uint64_t>(64, n - base);
    for (uint64_t i = 0; i < lim; ++i) x |= (uint64_t)((keys[base + i] >> b) & 1u) << i;
    words[w] = x;
  }
}

uint32_t bit_width_u64(uint64_t x) {
  uint32_t b = 0;
  while (x) {
    ++b;
    x >>= 1;
  }
  return b;
}


}  // namespace

#define RP(expr) FM_HIP(expr)

int gpu_suffix_sort(const uint32_t* text, uint64_t n, uint32_t* bwt_out, uint64_t* sa_out, hipStream_t s) {
  if (n == 0) {
    set_error("empty text");
    return -1;
  }
  if (n >= (1ull << kKey2Bits)) {
    set_error("gpu suffix sort: n = %llu exceeds 2^34", (unsigned long long)n);
    return -1;
  }
  // ---- validate: T'[n-1] == 0 is the only 0, symbols < 2^26
  Buf<unsigned long long> d_zero;
  Buf<uint32_t> d_max;
  if (d_zero.alloc(1) || d_max.alloc(1)) return -1;
  RP(hipMemsetAsync(d_zero.p, 0, 8, s));
  RP(hipMemsetAsync(d_max.p, 0, 4, s));
  k_sa_check<<<grid_for(n), kT, 0, s>>>(text, n, d_zero.p, d_max.p);
  RP(hipGetLastError());
  unsigned long long zeros = 0;
  uint32_t maxsym = 0, last = 1;
  RP(hipMemcpyAsync(&zeros, d_zero.p, 8, hipMemcpyDeviceToHost, s));
  RP(hipMemcpyAsync(&maxsym, d_max.p, 4, hipMemcpyDeviceToHost, s));
  RP(hipMemcpyAsync(&last, text + (n - 1), 4, hipMemcpyDeviceToHost, s));
  RP(hipStreamSynchronize(s));
  if (zeros != 1 || last != 0) {
    set_error("text must end with the unique sentinel 0 (found %llu zeros, last symbol %u)", zeros, last);
    return -1;
  }
  if (maxsym >= (1u << kMaxSymBits)) {
    set_error("symbol %u exceeds 2^%d", maxsym, kMaxSymBits);
    return -1;
  }
  const uint32_t bits = std::max<uint32_t>(1, bit_width_u64(maxsym));
  const uint32_t tpk = std::max<uint32_t>(1, kKey2Bits / bits);   // symbols packed into the first key2
  const uint64_t K = 1ull << bits;

  Buf<uint64_t> sa_own;
  uint64_t* sa = sa_out;
  if (!sa) {
    if (sa_own.alloc(n)) return -1;
    sa = sa_own.p;
  }
  Buf<uint64_t> rank, act;
  Buf<uint8_t> flag;   // initial active flags, then per-round head flags
  Buf<unsigned char> tmp;
  size_t tmp_bytes = 0;
  uint64_t A = 0;
  {
    // ---- init: sort positions by their first symbol
    Buf<uint32_t> keys;
    Buf<uint64_t> start, end;
    if (keys.alloc(n) || start.alloc(K) || end.alloc(K)) return -1;
    rocprim::counting_iterator<uint64_t> iota(0);
    size_t need = 0;
    RP(rocprim::radix_sort_pairs(nullptr, need, text, keys.p, iota, sa, (size_t)n, 0, bits, s));
    if (tmp.alloc(need)) return -1;
    tmp_bytes = need;
    RP(rocprim::radix_sort_pairs(tmp.p, need, text, keys.p, iota, sa, (size_t)n, 0, bits, s));
    RP(hipMemsetAsync(start.p, 0, K * 8, s));
    RP(hipMemsetAsync(end.p, 0, K * 8, s));
    k_sa_bounds<<<grid_for(n), kT, 0, s>>>(keys.p, n, start.p, end.p);
    RP(hipGetLastError());
    if (rank.alloc(n) || flag.alloc(n)) return -1;
    k_sa_init<<<grid_for(n), kT, 0, s>>>(text, keys.p, n, start.p, end.p, rank.p, flag.p);
    RP(hipGetLastError());
    keys.release();
    start.release();
    end.release();
    if (act.alloc(n)) return -1;
    Buf<uint64_t> d_cnt;
    if (d_cnt.alloc(1)) return -1;
    need = 0;
    RP(rocprim::select(nullptr, need, iota, flag.p, act.p, d_cnt.p, (size_t)n, s));
    if (need > tmp_bytes) {
      if (tmp.alloc(need)) return -1;
      tmp_bytes = need;
    }
    RP(rocprim::select(tmp.p, need, iota, flag.p, act.p, d_cnt.p, (size_t)n, s));
    RP(hipMemcpyAsync(&A, d_cnt.p, 8, hipMemcpyDeviceToHost, s));
    RP(hipStreamSynchronize(s));
  }

  const uint64_t CH = std::max<uint64_t>(1024, tuning().sa_chunk);
  Buf<uint64_t> kin, kout, vin, vout, d_cnt, d_end;
  if (d_cnt.alloc(1) || d_end.alloc(1)) return -1;
  uint8_t* head = flag.p;
  bool first = true;
  uint64_t h = 1;
  int rounds = 0;
  while (A > 0) {
    if (++rounds > 64) {
      set_error("gpu suffix sort did not converge");
      return -1;
    }
    // ---- chunk boundaries at group starts
    std::vector<uint64_t> cuts{0};
    uint64_t maxm = 0;
    while (cuts.back() < A) {
      const uint64_t s0 = cuts.back();
      uint64_t e = std::min(A, s0 + CH);
      if (e < A) {
        k_sa_chunk_end<<<1, 1, 0, s>>>(act.p, sa, rank.p, s0, e, A, d_end.p);
        RP(hipGetLastError());
        RP(hipMemcpyAsync(&e, d_end.p, 8, hipMemcpyDeviceToHost, s));
        RP(hipStreamSynchronize(s));
      }
      cuts.push_back(e);
      maxm = std::max(maxm, e - s0);
    }
    if (kin.reserve(maxm) || kout.reserve(maxm) || vin.reserve(maxm) || vout.reserve(maxm)) return -1;
    {
      size_t a = 0, b = 0, c = 0, d = 0;
      RP(rocprim::radix_sort_pairs(nullptr, a, kin.p, kout.p, vin.p, vout.p, (size_t)maxm, 0, 64, s));
      RP(rocprim::inclusive_scan(nullptr, b, kin.p, kout.p, (size_t)maxm, rocprim::plus<uint64_t>(), s));
      RP(rocprim::inclusive_scan(nullptr, c, kin.p, kout.p, (size_t)maxm, rocprim::maximum<uint64_t>(), s));
      RP(rocprim::select(nullptr, d, act.p, head, kin.p, d_cnt.p, (size_t)maxm, s));
      const size_t need = std::max(std::max(a, b), std::max(c, d));
      if (need > tmp_bytes) {
        if (tmp.alloc(need)) return -1;
        tmp_bytes = need;
      }
    }
    // ---- phase 1: sort every chunk's groups by key2, split, write SA
    for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
      const uint64_t s0 = cuts[ci], m = cuts[ci + 1] - s0;
      const unsigned g = grid_for(m);
      k_sa_gather<<<g, kT, 0, s>>>(act.p + s0, m, sa, rank.p, text, n, h, first ? 1 : 0, tpk, bits, kin.p,
                                   vin.p, kout.p);
      RP(hipGetLastError());
      size_t need = tmp_bytes;
      RP(rocprim::inclusive_scan(tmp.p, need, kout.p, vout.p, (size_t)m, rocprim::plus<uint64_t>(), s));
      k_sa_pack<<<g, kT, 0, s>>>(kin.p, vout.p, m);
      RP(hipGetLastError());
      const uint32_t end_bit = std::min<uint32_t>(64, kKey2Bits + std::max<uint32_t>(1, bit_width_u64(m)));
      need = tmp_bytes;
      RP(rocprim::radix_sort_pairs(tmp.p, need, kin.p, kout.p, vin.p, vout.p, (size_t)m, 0, end_bit, s));
      k_sa_scatter<<<g, kT, 0, s>>>(act.p + s0, m, kout.p, vout.p, sa, head + s0);
      RP(hipGetLastError());
    }
    // ---- phase 2: new ranks, compaction of the still-active suffixes
    uint64_t out = 0;
    for (size_t ci = 0; ci + 1 < cuts.size(); ++ci) {
      const uint64_t s0 = cuts[ci], m = cuts[ci + 1] - s0;
      const unsigned g = grid_for(m);
      k_sa_headval<<<g, kT, 0, s>>>(act.p + s0, head + s0, m, kin.p);
      RP(hipGetLastError());
      size_t need = tmp_bytes;
      RP(rocprim::inclusive_scan(tmp.p, need, kin.p, kout.p, (size_t)m, rocprim::maximum<uint64_t>(), s));
      uint8_t* keep = reinterpret_cast<uint8_t*>(vin.p);
      k_sa_rank<<<g, kT, 0, s>>>(act.p + s0, head + s0, m, sa, kout.p, rank.p, keep);
      RP(hipGetLastError());
      need = tmp_bytes;
      RP(rocprim::select(tmp.p, need, act.p + s0, keep, kin.p, d_cnt.p, (size_t)m, s));
      uint64_t cnt = 0;
      RP(hipMemcpyAsync(&cnt, d_cnt.p, 8, hipMemcpyDeviceToHost, s));
      RP(hipStreamSynchronize(s));
      if (cnt) RP(hipMemcpyAsync(act.p + out, kin.p, cnt * 8, hipMemcpyDeviceToDevice, s));
      out += cnt;
    }
    A = out;
    h = first ? 1 + tpk : 2 * h;
    first = false;
  }
  rank.release();
  act.release();
  flag.release();
  kin.release();
  kout.release();
  vin.release();
  vout.release();
  tmp.release();
  if (bwt_out) {
    k_sa_bwt<<<grid_for(n), kT, 0, s>>>(text, sa, n, bwt_out);
    RP(hipGetLastError());
  }
  RP(hipStreamSynchronize(s));
  return 0;
}

int gpu_wt_int_levels(const uint32_t* bwt, uint64_t n, uint32_t L, uint64_t* words, hipStream_t s) {
  if (L == 0 || L > 32) {
    set_error("bad level count %u", L);
    return -1;
  }
  const uint64_t nw = (n + 63) / 64;
  Buf<uint32_t> keys;
  Buf<unsigned char> tmp;
  if (keys.alloc(n)) return -1;
  size_t need = 0;
  RP(rocprim::radix_sort_keys(nullptr, need, bwt, keys.p, (size_t)n, 0, L, s));
  if (tmp.alloc(need)) return -1;
  for (uint32_t lev = 0; lev < L; ++lev) {
    const uint32_t* src = bwt;
    if (lev > 0) {
      size_t nb = tmp.count;
      // stable (LSD) sort by the top `lev` bits == the wt_int order of level `lev`
      RP(rocprim::radix_sort_keys(tmp.p, nb, bwt, keys.p, (size_t)n, L - lev, L, s));
      src = keys.p;
    }
    k_level_bits<<<grid_for(nw), kT, 0, s>>>(src, n, L - 1 - lev, words + (uint64_t)lev * nw);
    RP(hipGetLastError());
  }
  RP(hipStreamSynchronize(s));
  return 0;
}

}  // namespace fmidx
