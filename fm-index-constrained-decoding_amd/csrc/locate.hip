// locate.hip -- SA / ISA sampling and the LF-walk queries built on it
// (the sdsl csa_wt_int<> surface of fm_index.cpp:168-194: locate(row),
// extract_text(begin, end)), instead of a resident full suffix array.
//
// Layout (text-order sampling, rates 32 / 64 as sdsl's csa_wt defaults):
//   mark     n bits: row i is marked iff SA[i] % 32 == 0
//   mark_cnt per 512-row block, the marked rows before it (uint64)
//   sa_samp  SA[i] / 32 of every marked row, in row order (uint32: n < 2^34)
//   isa_samp isa_samp[k] = the row of text position 64 k
// At C3 (n = 4.5e9): 0.56 + 0.07 + 0.56 + 0.56 GB instead of 36 GB of SA.
//
// locate(i): walk LF from i until a marked row (<= 31 steps: each step moves
// one text position back, and every 32nd position is marked), then
// SA[i] = 32 * sa_samp[rank1(row)] + steps.
// extract_text(begin, end) (fm_index.cpp:174-194) walks LF from isa[end - 1],
// emitting BWT[row] = T'[pos - 1] per step; isa[end - 1] itself is reached by
// <= 63 LF steps from the next sampled position (or from row 0 = isa[n - 1],
// the sentinel suffix).  One LF step is one load of E (LF(i) | BWT[i]) when
// the index has it, else the 2-level wavelet-matrix descent of lf_step_decode.
#include "fmidx_internal.h"

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

namespace fmidx {

namespace {

constexpr int kThreads = 256;

template <typename T>
int dalloc(T** p, size_t count) {
  *p = nullptr;
  FM_HIP(hipMalloc(reinterpret_cast<void**>(p), (count ? count : 1) * sizeof(T)));
  return 0;
}

__global__ void __launch_bounds__(kThreads) k_iota_u32(uint32_t* __restrict__ out, uint64_t m) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < m) out[i] = (uint32_t)i;
}

// one wave per 64-row word: the mark bits, and the ISA samples (scatter)
__global__ void __launch_bounds__(kThreads) k_sa_mark(const uint64_t* __restrict__ sa, uint64_t n,
                                                      uint64_t* __restrict__ mark, uint64_t* __restrict__ isa) {
  const uint64_t nwords = (n + 63) / 64;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint64_t w = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) >> 6; w < nwords;
       w += ((uint64_t)gridDim.x * kThreads) >> 6) {
    const uint64_t i = w * 64 + lane;
    const uint64_t p = i < n ? sa[i] : 1;
    const uint64_t bits = __ballot(i < n && (p & (kSaRate - 1)) == 0);
    if (lane == 0) mark[w] = bits;
    if (i < n && (p & (kIsaRate - 1)) == 0) isa[p / kIsaRate] = i;
  }
}

// marked rows per 512-row block (8 words)
__global__ void __launch_bounds__(kThreads) k_mark_blocks(const uint64_t* __restrict__ mark, uint64_t nwords,
                                                          uint64_t nblocks, uint64_t* __restrict__ cnt) {
  const uint64_t b = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (b >= nblocks) return;
  uint64_t c = 0;
  for (uint64_t w = b * 8; w < min(nwords, b * 8 + 8); ++w) c += __popcll(mark[w]);
  cnt[b] = c;
}

__device__ __forceinline__ uint64_t rank_marked(const SampleView& sv, uint64_t i) {
  const uint64_t w = i >> 6;
  uint64_t r = sv.mark_cnt[i >> 9];
  for (uint64_t x = w & ~7ull; x < w; ++x) r += __popcll(sv.mark[x]);
  const uint32_t b = (uint32_t)(i & 63);
  if (b) r += __popcll(sv.mark[w] & ((1ull << b) - 1));
  return r;
}

__device__ __forceinline__ bool is_marked(const SampleView& sv, uint64_t i) {
  return (sv.mark[i >> 6] >> (i & 63)) & 1ull;
}

__global__ void __launch_bounds__(kThreads) k_sa_samples(const uint64_t* __restrict__ sa, uint64_t n,
                                                         SampleView sv, uint32_t* __restrict__ samp) {
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads) {
    const uint64_t p = sa[i];
    if ((p & (kSaRate - 1)) == 0) samp[rank_marked(sv, i)] = (uint32_t)(p / kSaRate);
  }
}

// LF(i) and BWT[i] by a whole wave (uniform i).
__device__ __forceinline__ void lf_row(const DevView& v, uint64_t i, uint64_t& lf, uint32_t& c) {
  if (v.E) {
    const uint64_t e = v.E[i];
    lf = e & kELfMask;
    c = (uint32_t)(e >> kESymShift);
    return;
  }
  c = bwt_sym(v, i);
  uint64_t l = i, h = i + 1;
  const uint32_t* cbm;
  int64_t one;
  lf_step_decode(v, (int64_t)c, l, h, cbm, one);
  lf = l;
}

// one wave per query row
__global__ void __launch_bounds__(kThreads) k_locate(DevView v, SampleView sv, const uint64_t* __restrict__ rows,
                                                     uint64_t m, uint64_t* __restrict__ out) {
  const uint64_t q = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  if (q >= m) return;
  uint64_t i = rows[q];
  if (i >= v.n) {   // fm_index.cpp:170
    if ((threadIdx.x & 63u) == 0) out[q] = ~0ull;
    return;
  }
  uint64_t steps = 0;
  while (!is_marked(sv, i) && steps < kSaRate) {
    uint64_t lf;
    uint32_t c;
    lf_row(v, i, lf, c);
    i = lf;
    ++steps;
  }
  if ((threadIdx.x & 63u) == 0) out[q] = (uint64_t)sv.sa_samp[rank_marked(sv, i)] * kSaRate + steps;
}

// one wave per request: out[off[q] + j] = T'[(end - 2 - j) mod n], j < off[q+1] - off[q]
__global__ void __launch_bounds__(kThreads) k_extract(DevView v, SampleView sv, const uint64_t* __restrict__ begin,
                                                      const uint64_t* __restrict__ end,
                                                      const uint64_t* __restrict__ off, uint64_t m,
                                                      uint64_t* __restrict__ out) {
  const uint64_t q = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  if (q >= m) return;
  const uint64_t len = off[q + 1] - off[q];
  uint64_t e = end[q];
  if (e > v.n) e = v.n;
  if (len == 0 || e == 0 || begin[q] >= e) return;
  const uint64_t p = e - 1;                               // isa[p] is where the walk starts
  uint64_t ps = (p + kIsaRate - 1) / kIsaRate * kIsaRate;  // the next sampled position
  uint64_t row;
  if (ps > v.n - 1) {
    ps = v.n - 1;
    row = 0;                                              // isa[n - 1]: the sentinel suffix is the smallest
  } else {
    row = sv.isa_samp[ps / kIsaRate];
  }
  for (uint64_t k = ps; k > p; --k) {                     // LF(isa[k]) = isa[k - 1]
    uint64_t lf;
    uint32_t c;
    lf_row(v, row, lf, c);
    row = lf;
  }
  uint64_t* o = out + off[q];
  for (uint64_t j = 0; j < len; ++j) {
    uint64_t lf;
    uint32_t c;
    lf_row(v, row, lf, c);
    if ((threadIdx.x & 63u) == 0) o[j] = c;
    row = lf;
  }
}

// The text-order SA samples from ISA samples alone (an index read from a file
// that holds the BWT and isa[k] = row of text position 64 k -- sdsl's
// isa_sampling<> of a csa_wt_int<>, fmidx/sdsl_fmi.py): block k walks LF from
// the row of position p_start = 64 (k + 1) (the last block: n - 1, whose row
// is 0 -- the sentinel suffix) down to position 64 k, each step one position
// back (LF(isa[p]) = isa[p - 1]), recording the row of every position that is
// a multiple of 32 in rows_out[p / 32].  The walk must arrive at isa[k]: the
// caller checks rows_out[2 k] == isa[k] for every block (a mismatch = an
// inconsistent BWT / sample pair; no atomics here).
// One lane per block when the index has the E array (LF | BWT in one load),
// one wave per block through lf_row otherwise.
template <bool LANE>
__global__ void __launch_bounds__(kThreads) k_isa_walk(DevView v, const uint64_t* __restrict__ isa, uint64_t nisa,
                                                       uint64_t* __restrict__ rows_out) {
  const uint64_t gid = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint64_t k = LANE ? gid : gid >> 6;
  if (k >= nisa) return;
  const bool last = k + 1 >= nisa;
  const uint64_t p_start = last ? v.n - 1 : kIsaRate * (k + 1);
  uint64_t row = last ? 0 : isa[k + 1];
  const uint64_t p_end = kIsaRate * k;
  const bool writer = LANE || (threadIdx.x & 63u) == 0;
  for (uint64_t p = p_start; p > p_end; --p) {
    if (writer && (p & (kSaRate - 1)) == 0 && p < kIsaRate * (k + 1)) rows_out[p / kSaRate] = row;
    if (row >= v.n) break;                                   // a corrupt sample: caught by the caller's check
    uint64_t lf;
    if (LANE) {
      lf = v.E[row] & kELfMask;
    } else {
      uint32_t c;
      lf_row(v, row, lf, c);
    }
    row = lf;
  }
  if (writer) rows_out[p_end / kSaRate] = row;
}

// mark words from the sorted marked rows, without atomics: the first row of
// every 64-row word ORs the (<= 64) sorted rows of that word and writes it
__global__ void __launch_bounds__(kThreads) k_mark_from_sorted(const uint64_t* __restrict__ rows, uint64_t m,
                                                               uint64_t* __restrict__ mark) {
  const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= m) return;
  const uint64_t w = rows[i] >> 6;
  if (i > 0 && (rows[i - 1] >> 6) == w) return;
  uint64_t bits = 0;
  for (uint64_t j = i; j < m && (rows[j] >> 6) == w; ++j) bits |= 1ull << (rows[j] & 63);
  mark[w] = bits;
}

struct IsaOutOfRange {
  const uint64_t* isa;
  uint64_t n;
  __host__ __device__ uint64_t operator()(uint64_t k) const { return isa[k] >= n ? 1ull : 0ull; }
};

// a block whose walk did not arrive at its own sample (rows[2 k] = the row reached for position 64 k)
struct WalkMismatch {
  const uint64_t* isa;
  const uint64_t* rows;
  __host__ __device__ uint64_t operator()(uint64_t k) const { return rows[2 * k] != isa[k] ? 1ull : 0ull; }
};

template <typename F>
int count_where(F f, uint64_t m, uint64_t* d_out, uint64_t& out, hipStream_t s) {
  rocprim::counting_iterator<uint64_t> iota(0);
  auto it = rocprim::make_transform_iterator(iota, f);
  size_t tb = 0;
  FM_HIP(rocprim::reduce(nullptr, tb, it, d_out, (uint64_t)0, (size_t)m, rocprim::plus<uint64_t>(), s));
  void* tmp = nullptr;
  FM_HIP(hipMalloc(&tmp, tb ? tb : 1));
  const hipError_t e = rocprim::reduce(tmp, tb, it, d_out, (uint64_t)0, (size_t)m, rocprim::plus<uint64_t>(), s);
  (void)hipStreamSynchronize(s);
  (void)hipFree(tmp);
  FM_HIP(e);
  FM_HIP(hipMemcpy(&out, d_out, 8, hipMemcpyDeviceToHost));
  return 0;
}

}  // namespace

// The text-order SA samples of an index built from a BWT, from ISA samples
// (isa[k] = row of text position 64 k, (n-1)/64 + 1 of them: sdsl
// isa_sampling<> of a csa_wt_int<>): every sample is checked to be a row, the
// LF walks (k_isa_walk) give the row of every position that is a multiple of
// 32, every walk must end at its own block's sample, then the rows are sorted
// (their order is sa_samp: SA / 32 by row) and the mark words written.
int device_samples_from_isa(Index* h, const uint64_t* d_isa, uint64_t nisa, hipStream_t s) {
  const uint64_t n = h->n;
  if (nisa != (n - 1) / kIsaRate + 1) {
    set_error("ISA samples: %llu given, (n - 1) / 64 + 1 = %llu expected", (unsigned long long)nisa,
              (unsigned long long)((n - 1) / kIsaRate + 1));
    return -1;
  }
  const uint64_t nwords = (n + 63) / 64, nblocks = (n + 511) / 512;
  const uint64_t nsamp = (n + kSaRate - 1) / kSaRate;
  uint64_t *isa = nullptr, *rows = nullptr, *rows2 = nullptr, *d_cnt = nullptr, *mark = nullptr, *cnt = nullptr,
           *tmp = nullptr;
  uint32_t *ord = nullptr, *samp = nullptr;
  auto cleanup = [&]() {
    for (void* p : {(void*)isa, (void*)rows, (void*)rows2, (void*)d_cnt, (void*)mark, (void*)cnt, (void*)tmp,
                    (void*)ord, (void*)samp})
      if (p) (void)hipFree(p);
  };
  if (dalloc(&isa, nisa) || dalloc(&rows, nsamp) || dalloc(&rows2, nsamp) || dalloc(&d_cnt, 1) ||
      dalloc(&ord, nsamp) || dalloc(&samp, nsamp)) {
    cleanup();
    return -1;
  }
  // every HIP failure below frees what this function allocated (ISA_CK), the
  // sort's temporary included
#define ISA_CK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      ::fmidx::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
      cleanup();                                                                          \
      return -1;                                                                          \
    }                                                                                     \
  } while (0)
  ISA_CK(hipMemcpyAsync(isa, d_isa, nisa * 8, hipMemcpyDeviceToDevice, s));
  uint64_t bad = 0;
  if (count_where(IsaOutOfRange{isa, n}, nisa, d_cnt, bad, s) || bad) {
    if (bad) set_error("ISA samples: %llu rows out of range (n = %llu)", (unsigned long long)bad, (unsigned long long)n);
    cleanup();
    return -1;
  }
  if (launch_isa_walk(h->view, isa, nisa, rows, s) || count_where(WalkMismatch{isa, rows}, nisa, d_cnt, bad, s) ||
      bad) {
    if (bad)
      set_error("ISA samples disagree with the BWT: %llu of %llu LF walks missed their sample", (unsigned long long)bad,
                (unsigned long long)nisa);
    cleanup();
    return -1;
  }
  // sort the marked rows; the permutation that sorts them is sa_samp (position / 32 in row order)
  uint32_t* seq = ord;
  {
    size_t tb = 0;
    int bits = 1;
    while (bits < 64 && (n - 1) >> bits) ++bits;
    ISA_CK(rocprim::radix_sort_pairs(nullptr, tb, rows, rows2, seq, samp, (size_t)nsamp, 0, bits, s));
    void* t = nullptr;
    ISA_CK(hipMalloc(&t, tb ? tb : 1));
    hipError_t e = hipSuccess;
    k_iota_u32<<<(unsigned)((nsamp + kThreads - 1) / kThreads), kThreads, 0, s>>>(seq, nsamp);
    e = hipGetLastError();
    if (e == hipSuccess) e = rocprim::radix_sort_pairs(t, tb, rows, rows2, seq, samp, (size_t)nsamp, 0, bits, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(t);
    if (e != hipSuccess) {
      cleanup();
      set_error("sorting the sampled rows: %s", hipGetErrorString(e));
      return -1;
    }
  }
  if (dalloc(&mark, nwords) || dalloc(&cnt, nblocks) || dalloc(&tmp, nblocks)) {
    cleanup();
    return -1;
  }
  ISA_CK(hipMemsetAsync(mark, 0, nwords * 8, s));
  k_mark_from_sorted<<<(unsigned)((nsamp + kThreads - 1) / kThreads), kThreads, 0, s>>>(rows2, nsamp, mark);
  k_mark_blocks<<<(unsigned)((nblocks + kThreads - 1) / kThreads), kThreads, 0, s>>>(mark, nwords, nblocks, tmp);
  ISA_CK(hipGetLastError());
  if (exclusive_scan_u64(tmp, cnt, nblocks, s, nullptr)) {
    cleanup();
    return -1;
  }
  ISA_CK(hipStreamSynchronize(s));
#undef ISA_CK
  for (void* p : {(void*)h->mark, (void*)h->mark_cnt, (void*)h->sa_samp, (void*)h->isa_samp})
    if (p) (void)hipFree(p);
  h->mark = mark;
  h->mark_cnt = cnt;
  h->sa_samp = samp;
  h->isa_samp = isa;
  h->samp_bytes = nwords * 8 + nblocks * 8 + nsamp * 4 + nisa * 8;
  mark = cnt = isa = nullptr;
  samp = nullptr;
  cleanup();
  return 0;
}

int launch_isa_walk(const DevView& v, const uint64_t* isa, uint64_t nisa, uint64_t* rows_out, hipStream_t s) {
  if (nisa == 0) return 0;
  if (v.E) {
    k_isa_walk<true><<<(unsigned)((nisa + kThreads - 1) / kThreads), kThreads, 0, s>>>(v, isa, nisa, rows_out);
  } else {
    k_isa_walk<false><<<(unsigned)((nisa * 64 + kThreads - 1) / kThreads), kThreads, 0, s>>>(v, isa, nisa, rows_out);
  }
  FM_HIP(hipGetLastError());
  return 0;
}

int device_build_samples(Index* h, const uint64_t* d_sa, uint64_t n, hipStream_t s) {
  const uint64_t nwords = (n + 63) / 64, nblocks = (n + 511) / 512;
  const uint64_t nsamp = (n + kSaRate - 1) / kSaRate, nisa = (n - 1) / kIsaRate + 1;
  uint64_t *mark = nullptr, *cnt = nullptr, *tmp = nullptr, *isa = nullptr;
  uint32_t* samp = nullptr;
  if (dalloc(&mark, nwords) || dalloc(&cnt, nblocks) || dalloc(&tmp, nblocks) || dalloc(&isa, nisa) ||
      dalloc(&samp, nsamp))
    return -1;
  const unsigned g = (unsigned)std::min<uint64_t>((n + kThreads - 1) / kThreads, 1u << 16);
  k_sa_mark<<<g, kThreads, 0, s>>>(d_sa, n, mark, isa);
  k_mark_blocks<<<(unsigned)((nblocks + kThreads - 1) / kThreads), kThreads, 0, s>>>(mark, nwords, nblocks, tmp);
  FM_HIP(hipGetLastError());
  if (exclusive_scan_u64(tmp, cnt, nblocks, s, nullptr)) return -1;
  SampleView sv{mark, cnt, nullptr, isa};
  k_sa_samples<<<g, kThreads, 0, s>>>(d_sa, n, sv, samp);
  FM_HIP(hipGetLastError());
  FM_HIP(hipStreamSynchronize(s));
  FM_HIP(hipFree(tmp));
  h->mark = mark;
  h->mark_cnt = cnt;
  h->sa_samp = samp;
  h->isa_samp = isa;
  h->samp_bytes = nwords * 8 + nblocks * 8 + nsamp * 4 + nisa * 8;
  return 0;
}

// From saved samples (fm_load): the mark bits, sa_samp and isa_samp are
// already on the device; rebuild the block counts.
int device_finish_samples(Index* h, uint64_t n, hipStream_t s) {
  const uint64_t nwords = (n + 63) / 64, nblocks = (n + 511) / 512;
  uint64_t *cnt = nullptr, *tmp = nullptr;
  if (dalloc(&cnt, nblocks) || dalloc(&tmp, nblocks)) return -1;
  k_mark_blocks<<<(unsigned)((nblocks + kThreads - 1) / kThreads), kThreads, 0, s>>>(h->mark, nwords, nblocks, tmp);
  FM_HIP(hipGetLastError());
  if (exclusive_scan_u64(tmp, cnt, nblocks, s, nullptr)) return -1;
  FM_HIP(hipStreamSynchronize(s));
  FM_HIP(hipFree(tmp));
  h->mark_cnt = cnt;
  h->samp_bytes = nwords * 8 + nblocks * 8 + ((n + kSaRate - 1) / kSaRate) * 4 + ((n - 1) / kIsaRate + 1) * 8;
  return 0;
}

int launch_locate(const DevView& v, const SampleView& sv, const uint64_t* rows, uint64_t m, uint64_t* out,
                  hipStream_t s) {
  if (m == 0) return 0;
  if (!sv.mark) {
    set_error("index has no suffix-array samples: locate unavailable");
    return -1;
  }
  k_locate<<<(unsigned)((m * 64 + kThreads - 1) / kThreads), kThreads, 0, s>>>(v, sv, rows, m, out);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_extract(const DevView& v, const SampleView& sv, const uint64_t* begin, const uint64_t* end,
                   const uint64_t* off, uint64_t m, uint64_t* out, hipStream_t s) {
  if (m == 0) return 0;
  if (!sv.isa_samp) {
    set_error("index has no inverse-suffix-array samples: extract_text unavailable");
    return -1;
  }
  k_extract<<<(unsigned)((m * 64 + kThreads - 1) / kThreads), kThreads, 0, s>>>(v, sv, begin, end, off, m, out);
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
