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

namespace fmidx {

namespace {

constexpr int kThreads = 256;

template <typename T>
int dalloc(T** p, size_t count) {
  *p = nullptr;
  FM_HIP(hipMalloc(reinterpret_cast<void**>(p), (count ? count : 1) * sizeof(T)));
  return 0;
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
  c = v.bwt[i];
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

}  // namespace

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
