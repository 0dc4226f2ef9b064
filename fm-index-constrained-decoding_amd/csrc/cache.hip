// cache.hip -- range-bitmap cache: one precomputed allowed-token bitmap for
// every wide SA range a decode step can land on.
//
// The range of a pattern P (index.py:103-112) is the SA interval of the
// T' suffixes that start with rev(P).  Every such interval is the leaf set of
// a node of T''s suffix tree, so the distinct ranges of width >= Wc are at
// most 2n/Wc, and all of them are reachable from the root [0, n) by LF steps
// (the decode steps themselves).  They are enumerated breadth-first:
// children of a range = LF_c(range) for every symbol c occurring >= Wc times
// in it (k_distinct with min_count = Wc, O(width / Wc) per range), dedup by
// (lo, hi) -- the same range is reached again from a longer pattern when a
// pattern is always preceded by the same token.  Each cached range gets its
// bitmap (the mask kernel over the aligned bitmap hierarchy, packed), and an
// open-addressing table maps (lo, hi) -> bitmap.
//
// In the decode step a wide row then reads ONE bitmap (V/8 bytes) instead of
// its partial ends (up to 2 x 4095 BWT symbols) plus up to ~6 aligned bitmaps
// per hierarchy level.  Ranges narrower than Wc stream BWT[lo, hi) directly;
// ranges outside the cache (arbitrary user ranges, or past the memory budget)
// fall back to the hierarchy.  Results are identical either way.
#include "fmidx_internal.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

namespace fmidx {

namespace {

struct PairHash {
  size_t operator()(const std::pair<uint64_t, uint64_t>& p) const { return (size_t)cache_hash(p.first, p.second); }
};

#ifndef FMIDX_CACHE_STATS
#define FMIDX_CACHE_STATS 0
#endif
constexpr bool kCacheStats = FMIDX_CACHE_STATS != 0;   // diagnostic build: cache construction statistics on stderr

template <typename T>
struct DBuf {
  T* p = nullptr;
  DBuf() = default;
  DBuf(const DBuf&) = delete;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  int alloc(size_t count) {
    if (p) (void)hipFree(p);
    p = nullptr;
    FM_HIP(hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(1, count) * sizeof(T)));
    return 0;
  }
};

}  // namespace

// Cache id + 1 of [lo, hi), or 0: one thread's linear probe of the cache table.
__device__ uint64_t cache_id_thread(const DevView& v, uint64_t lo, uint64_t hi) {
  if (!v.cache_mask || hi - lo < v.cache_min) return 0;
  uint64_t slot = cache_hash(lo, hi) & v.cache_mask;
  for (uint64_t i = 0; i <= v.cache_mask; ++i) {
    const uint64_t e0 = v.cache_tab[2 * slot], e1 = v.cache_tab[2 * slot + 1];
    if (e0 == kCacheEmpty) return 0;
    if (e0 == lo && (e1 & kMask34) == hi) return (e1 >> kCacheIdShift) + 1;
    slot = (slot + 1) & v.cache_mask;
  }
  return 0;
}

// Insert the children of a batch of cached parents (k_distinct output: row r's
// k[r] symbols, counts and child starts at off[r]) into the transition table.
// One workgroup per parent; a key goes to the emptier of its two buckets (fill
// counts in `fill`, read without synchronisation: a stale read only makes the
// choice less even), its slot claimed by an atomic increment of that bucket's
// count; a key finding both buckets full is left out (the decode step then
// takes the wavelet-matrix descent for it).
__global__ void __launch_bounds__(256) k_trans_insert(DevView v, const uint64_t* __restrict__ plo,
                                                      const uint64_t* __restrict__ phi,
                                                      const uint64_t* __restrict__ off,
                                                      const uint64_t* __restrict__ k,
                                                      const uint64_t* __restrict__ syms,
                                                      const uint64_t* __restrict__ cnt,
                                                      const uint64_t* __restrict__ child, uint64_t m,
                                                      uint64_t* __restrict__ tab, uint64_t cap,
                                                      uint32_t* __restrict__ fill,
                                                      unsigned long long* __restrict__ stats) {
  __shared__ uint64_t s_pid;
  const uint64_t r = blockIdx.x;
  if (r >= m) return;
  const uint64_t kr = k[r];
  if (kr == ~0ull) {   // a parent whose children were not listed: the table is not complete
    if (threadIdx.x == 0) atomicAdd(&stats[2], 1ull);
    return;
  }
  const uint64_t lo = plo[r], hi = phi[r], base = off[r];
  if (threadIdx.x == 0) s_pid = cache_id_thread(v, lo, hi);   // the parent's cache id + 1 (0: not cached)
  __syncthreads();
  const uint64_t pid1 = s_pid;
  unsigned long long ins = 0, drop = 0;
  for (uint64_t j = threadIdx.x; j < kr; j += 256) {
    const uint64_t c = syms[base + j], cw = cnt[base + j], clo = child[base + j];
    // kind / aux: a cached child's cache id, a one-row child's only symbol, else the range alone
    uint64_t kind = 0, aux = 0;
    if (cw >= v.cache_min) {
      const uint64_t id1 = cache_id_thread(v, clo, clo + cw);
      if (id1 && id1 - 1 < kTAuxLimit) {
        kind = kTKindCached;
        aux = id1 - 1;
      }
    } else if (cw == 1) {
      const uint64_t sym = bwt_sym(v, clo);
      if (sym < kTAuxLimit) {
        kind = kTKindOne;
        aux = sym;
      }
    }
    // a key the slot cannot hold (a parent outside the cache or past 2^20 - 2 ids, a symbol of 18+
    // bits) is left out: the descent serves it
    const bool fits = pid1 && pid1 - 1 < kTPidNone && c < kTSymLimit;
    const uint64_t w0 = trans_key(fits ? pid1 - 1 : 0, c) | (kind << 38) | ((clo & ((1ull << 24) - 1)) << 40);
    const uint64_t w1 = (clo >> 24) | (cw << 10) | (aux << 44);
    const TransHome th = trans_home(lo, hi, c, cap);
    const uint64_t ba = th.a / kTransBucket, bb = th.b / kTransBucket;
    const bool a_first = __hip_atomic_load(fill + ba, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <=
                         __hip_atomic_load(fill + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool done = false;
    for (uint32_t t = 0; t < 2 && !done && fits; ++t) {
      const uint64_t bk = (t == 0) == a_first ? ba : bb;
      const uint32_t k = atomicAdd(fill + bk, 1u);
      if (k < kTransBucket) {
        uint64_t* p = tab + 2 * (bk * kTransBucket + k);
        p[0] = w0;
        p[1] = w1;
        done = true;
      }
    }
    if (done) ++ins; else ++drop;
  }
  if (ins) atomicAdd(&stats[0], ins);
  if (drop) atomicAdd(&stats[1], drop);
}

// Transition table of the cached ranges (all their children, or -- when that
// would exceed the trans_mb budget -- only the cached ones), built on the GPU from
// two k_distinct passes over the cached parents: one to count the entries,
// one to insert them.
constexpr double kTransLoad = 0.85;

int build_transitions(Index* h, const std::vector<std::pair<uint64_t, uint64_t>>& nodes, hipStream_t s) {
  DevView& v = h->view;
  v.trans_cap = 0;
  v.trans_tab = nullptr;
  v.probe_first &= ~kProbeComplete;
  if (h->trans_tab) (void)hipFree(h->trans_tab);
  h->trans_tab = nullptr;
  h->trans_entries = h->trans_dropped = h->trans_bytes = 0;
  const uint64_t mode = (uint64_t)h->opts.transitions;   // 2 = every child, 1 = cached children only, 0 = none
  if (mode == 0 || nodes.size() < 2 || !v.cache_mask) return 0;
  const uint64_t budget = h->opts.trans_mb << 20;
  const uint64_t sigma = (uint64_t)h->max_sym + 1;
  const uint64_t kChunkCap = 1ull << 26;   // child slots per k_distinct launch
  const uint64_t kChunkRows = 1ull << 20;
  // chunk buffers, allocated once and reused by every chunk of both passes
  DBuf<uint64_t> d_lo, d_hi, d_off, d_syms, d_cnt, d_child, d_k;
  DBuf<uint8_t> d_ws;
  if (d_lo.alloc(kChunkRows) || d_hi.alloc(kChunkRows) || d_off.alloc(kChunkRows + 1) || d_syms.alloc(kChunkCap) ||
      d_cnt.alloc(kChunkCap) || d_child.alloc(kChunkCap) || d_k.alloc(kChunkRows) ||
      d_ws.alloc(distinct_ws_bytes(kChunkCap)))
    return -1;
  std::vector<uint64_t> lo, hi, off, k;
  lo.reserve(kChunkRows);
  hi.reserve(kChunkRows);
  off.reserve(kChunkRows + 1);
  // parents: every cached range but the root (whose LF step is the C lookup)
  auto pass = [&](uint64_t min_count, uint64_t* tab, uint64_t cap, uint32_t* d_fill, uint64_t& total,
                  unsigned long long* d_stats) -> int {
    total = 0;
    for (size_t i0 = 1; i0 < nodes.size();) {
      lo.clear();
      hi.clear();
      off.assign(1, 0);
      size_t i1 = i0;
      while (i1 < nodes.size() && i1 - i0 < kChunkRows) {
        const uint64_t w = nodes[i1].second - nodes[i1].first;
        const uint64_t c = std::min<uint64_t>(min_count > 1 ? w / min_count + 1 : w, sigma);
        if (i1 > i0 && off.back() + c > kChunkCap) break;
        lo.push_back(nodes[i1].first);
        hi.push_back(nodes[i1].second);
        off.push_back(off.back() + c);
        ++i1;
      }
      const uint64_t m = i1 - i0, tot = off.back();
      FM_HIP(hipMemcpyAsync(d_lo.p, lo.data(), m * 8, hipMemcpyHostToDevice, s));
      FM_HIP(hipMemcpyAsync(d_hi.p, hi.data(), m * 8, hipMemcpyHostToDevice, s));
      FM_HIP(hipMemcpyAsync(d_off.p, off.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
      if (launch_distinct(v, d_lo.p, d_hi.p, m, d_off.p, d_syms.p, d_cnt.p, d_k.p, d_ws.p, tot, s, min_count,
                          d_child.p))
        return -1;
      if (tab) {
        k_trans_insert<<<(unsigned)m, 256, 0, s>>>(v, d_lo.p, d_hi.p, d_off.p, d_k.p, d_syms.p, d_cnt.p,
                                                   d_child.p, m, tab, cap, d_fill, d_stats);
        FM_HIP(hipGetLastError());
        FM_HIP(hipStreamSynchronize(s));   // the host staging vectors are refilled next chunk
      } else {
        k.resize(m);
        FM_HIP(hipMemcpyAsync(k.data(), d_k.p, m * 8, hipMemcpyDeviceToHost, s));
        FM_HIP(hipStreamSynchronize(s));
        for (uint64_t r = 0; r < m; ++r) total += (k[r] == ~0ull) ? 0 : k[r];
      }
      i0 = i1;
    }
    return 0;
  };
  uint64_t min_count = mode >= 2 ? (uint64_t)std::max(1, h->opts.trans_min) : v.cache_min;
  uint64_t entries = 0;
  double t = build_clock();
  if (pass(min_count, nullptr, 0, nullptr, entries, nullptr)) return -1;
  build_phase("transitions: count pass", t, s);
  // buckets of 8 slots at load <= kTransLoad (two-choice: fmidx_internal.h)
  auto slots_for = [](uint64_t e) {
    const uint64_t nb = std::max<uint64_t>(128, (uint64_t)((double)e / (kTransLoad * kTransBucket)) + 1);
    return nb * kTransBucket;
  };
  uint64_t cap = slots_for(entries);
  if (cap * kTransSlotBytes > budget && min_count < v.cache_min) {   // over budget: the cached children only
    min_count = v.cache_min;
    if (pass(min_count, nullptr, 0, nullptr, entries, nullptr)) return -1;
    cap = slots_for(entries);
  }
  if (entries == 0 || cap * kTransSlotBytes > budget) return 0;
  uint64_t* tab = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&tab), cap * kTransSlotBytes) != hipSuccess) {
    (void)hipGetLastError();
    return 0;   // no room: the descent serves every step
  }
  FM_HIP(hipMemsetAsync(tab, 0xFF, cap * kTransSlotBytes, s));
  DBuf<unsigned long long> d_stats;
  DBuf<uint32_t> d_fill;   // per-bucket fill counts, for the insert only
  if (d_stats.alloc(3) || d_fill.alloc(cap / kTransBucket)) {
    (void)hipFree(tab);
    return -1;
  }
  FM_HIP(hipMemsetAsync(d_stats.p, 0, 24, s));
  FM_HIP(hipMemsetAsync(d_fill.p, 0, cap / kTransBucket * 4, s));
  uint64_t dummy = 0;
  t = build_clock();
  if (pass(min_count, tab, cap, d_fill.p, dummy, d_stats.p)) {
    (void)hipFree(tab);
    return -1;
  }
  build_phase("transitions: insert pass", t, s);
  unsigned long long st[3] = {0, 0, 0};
  FM_HIP(hipMemcpy(st, d_stats.p, 24, hipMemcpyDeviceToHost));
  FM_HIP(hipStreamSynchronize(s));
  h->trans_tab = tab;
  h->trans_entries = st[0];
  h->trans_dropped = st[1];
  h->trans_bytes = cap * kTransSlotBytes;
  h->cache_bytes += cap * kTransSlotBytes;
  v.trans_tab = tab;
  v.trans_cap = cap;
  // every child of every cached parent offered to the table (kProbeComplete, fmidx_internal.h);
  // FMIDX_PROBE_COMPLETE=0 turns the absent-symbol shortcut off (measurement)
  const char* pc_env = getenv("FMIDX_PROBE_COMPLETE");
  if (min_count == 1 && st[2] == 0 && !(pc_env && pc_env[0] == '0')) v.probe_first |= kProbeComplete;
  return 0;
}

int device_build_cache(Index* h, hipStream_t s) {
  DevView& v = h->view;
  v.cache_mask = 0;
  v.cache_bm = nullptr;
  v.cblock = nullptr;
  v.cache_tab = nullptr;
  const uint64_t n = h->n;
  const uint64_t Wc = std::max<uint64_t>(2, h->opts.cache_min);
  const uint64_t budget = h->opts.cache_mb << 20;
  const uint64_t words = v.bm_words;
  if (words == 0 || v.bm_levels == 0 || n < Wc || budget == 0) return 0;
  const uint64_t max_nodes = std::max<uint64_t>(1, budget / (words * 4));

  // ---- breadth-first enumeration of the ranges with width >= Wc
  const double t_bfs = build_clock();
  std::vector<std::pair<uint64_t, uint64_t>> nodes;
  std::unordered_map<std::pair<uint64_t, uint64_t>, uint64_t, PairHash> seen;   // range -> id
  std::vector<std::pair<uint64_t, uint64_t>> frontier{{0, n}}, next;
  std::vector<std::pair<uint64_t, uint64_t>> root_child;   // (symbol, cache id) of the cached C-blocks
  nodes.push_back({0, n});
  seen.emplace(std::make_pair(uint64_t(0), n), 0);
  const uint64_t kChunkCap = 1ull << 24;   // child slots per k_distinct launch
  bool full = false;
  while (!frontier.empty() && !full) {
    next.clear();
    size_t i0 = 0;
    while (i0 < frontier.size() && !full) {
      // rows [i0, i1) with sum of capacities <= kChunkCap (at least one row)
      std::vector<uint64_t> lo, hi, off{0};
      size_t i1 = i0;
      while (i1 < frontier.size()) {
        const uint64_t cap = (frontier[i1].second - frontier[i1].first) / Wc + 1;
        if (i1 > i0 && off.back() + cap > kChunkCap) break;
        lo.push_back(frontier[i1].first);
        hi.push_back(frontier[i1].second);
        off.push_back(off.back() + cap);
        ++i1;
      }
      const uint64_t m = i1 - i0, total = off.back();
      DBuf<uint64_t> d_lo, d_hi, d_off, d_syms, d_cnt, d_child, d_k;
      DBuf<uint8_t> d_ws;
      if (d_lo.alloc(m) || d_hi.alloc(m) || d_off.alloc(m + 1) || d_syms.alloc(total) || d_cnt.alloc(total) ||
          d_child.alloc(total) || d_k.alloc(m) || d_ws.alloc(distinct_ws_bytes(total)))
        return -1;
      FM_HIP(hipMemcpyAsync(d_lo.p, lo.data(), m * 8, hipMemcpyHostToDevice, s));
      FM_HIP(hipMemcpyAsync(d_hi.p, hi.data(), m * 8, hipMemcpyHostToDevice, s));
      FM_HIP(hipMemcpyAsync(d_off.p, off.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
      if (launch_distinct(v, d_lo.p, d_hi.p, m, d_off.p, d_syms.p, d_cnt.p, d_k.p, d_ws.p, total, s, Wc,
                          d_child.p))
        return -1;
      std::vector<uint64_t> k(m), cnt(total), child(total), sym(total);
      FM_HIP(hipMemcpyAsync(k.data(), d_k.p, m * 8, hipMemcpyDeviceToHost, s));
      FM_HIP(hipMemcpyAsync(sym.data(), d_syms.p, total * 8, hipMemcpyDeviceToHost, s));
      FM_HIP(hipMemcpyAsync(cnt.data(), d_cnt.p, total * 8, hipMemcpyDeviceToHost, s));
      FM_HIP(hipMemcpyAsync(child.data(), d_child.p, total * 8, hipMemcpyDeviceToHost, s));
      FM_HIP(hipStreamSynchronize(s));
      for (uint64_t r = 0; r < m && !full; ++r) {
        if (k[r] == ~0ull) {
          set_error("range cache: child overflow at [%llu, %llu)", (unsigned long long)lo[r],
                    (unsigned long long)hi[r]);
          return -1;
        }
        for (uint64_t j = 0; j < k[r]; ++j) {
          const uint64_t a = child[off[r] + j], b = a + cnt[off[r] + j];
          auto it = seen.find({a, b});
          uint64_t id;
          if (it == seen.end()) {
            if (nodes.size() >= max_nodes) {
              full = true;
              break;
            }
            id = nodes.size();
            seen.emplace(std::make_pair(a, b), id);
            nodes.push_back({a, b});
            next.push_back({a, b});
          } else {
            id = it->second;
          }
          if (lo[r] == 0 && hi[r] == n) root_child.push_back({sym[off[r] + j], id});
        }
      }
      i0 = i1;
    }
    frontier.swap(next);
  }
  seen.clear();

  if (kCacheStats) {
    // diagnostic: distinct symbols summed over the cached ranges, and their width histogram
    uint64_t sum = 0, maxk = 0, hist[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t wsum = 0, ksum_w[6] = {0, 0, 0, 0, 0, 0};   // distinct summed over parents of width < 8K,32K,128K,512K,2M,inf
    for (size_t i = 1; i < nodes.size(); ++i) wsum += nodes[i].second - nodes[i].first;
    const auto t_stats = std::chrono::steady_clock::now();
    const uint64_t sigma = (uint64_t)h->max_sym + 1;
    for (size_t i0 = 1; i0 < nodes.size();) {
      std::vector<uint64_t> lo, hi, off{0};
      size_t i1 = i0;
      while (i1 < nodes.size()) {
        const uint64_t cap = std::min<uint64_t>(nodes[i1].second - nodes[i1].first, sigma);
        if (i1 > i0 && off.back() + cap > (1ull << 25)) break;
        lo.push_back(nodes[i1].first);
        hi.push_back(nodes[i1].second);
        off.push_back(off.back() + cap);
        ++i1;
      }
      const uint64_t m = i1 - i0, total = off.back();
      DBuf<uint64_t> d_lo, d_hi, d_off, d_syms, d_cnt, d_k;
      DBuf<uint8_t> d_ws;
      if (d_lo.alloc(m) || d_hi.alloc(m) || d_off.alloc(m + 1) || d_syms.alloc(total) || d_cnt.alloc(total) ||
          d_k.alloc(m) || d_ws.alloc(distinct_ws_bytes(total)))
        return -1;
      FM_HIP(hipMemcpyAsync(d_lo.p, lo.data(), m * 8, hipMemcpyHostToDevice, s));
      FM_HIP(hipMemcpyAsync(d_hi.p, hi.data(), m * 8, hipMemcpyHostToDevice, s));
      FM_HIP(hipMemcpyAsync(d_off.p, off.data(), (m + 1) * 8, hipMemcpyHostToDevice, s));
      if (launch_distinct(v, d_lo.p, d_hi.p, m, d_off.p, d_syms.p, d_cnt.p, d_k.p, d_ws.p, total, s)) return -1;
      std::vector<uint64_t> k(m);
      FM_HIP(hipMemcpyAsync(k.data(), d_k.p, m * 8, hipMemcpyDeviceToHost, s));
      FM_HIP(hipStreamSynchronize(s));
      for (uint64_t r = 0; r < m; ++r) {
        sum += k[r];
        maxk = std::max(maxk, k[r]);
        {
          const uint64_t w = hi[r] - lo[r];
          int c = 0;
          while (c < 5 && w >= (8192ull << (2 * c))) ++c;
          ksum_w[c] += k[r];
        }
        int b = 0;
        while (b < 7 && k[r] >= (16ull << (2 * b))) ++b;
        hist[b]++;
      }
      i0 = i1;
    }
    fprintf(stderr, "[fmidx] cache: %zu ranges >= %llu, distinct symbols summed %llu (max %llu); "
            "distinct-count histogram <16,<64,<256,<1K,<4K,<16K,<64K,>=: %llu %llu %llu %llu %llu %llu %llu %llu; "
            "\n", nodes.size(), (unsigned long long)Wc, (unsigned long long)sum,
            (unsigned long long)maxk, (unsigned long long)hist[0], (unsigned long long)hist[1],
            (unsigned long long)hist[2], (unsigned long long)hist[3], (unsigned long long)hist[4],
            (unsigned long long)hist[5], (unsigned long long)hist[6], (unsigned long long)hist[7]);
    fprintf(stderr, "[fmidx] cache: widths summed %llu; distinct summed by parent width <8K,<32K,<128K,<512K,<2M,>=: "
            "%llu %llu %llu %llu %llu %llu; stats pass %.1f s\n", (unsigned long long)wsum,
            (unsigned long long)ksum_w[0], (unsigned long long)ksum_w[1], (unsigned long long)ksum_w[2],
            (unsigned long long)ksum_w[3], (unsigned long long)ksum_w[4], (unsigned long long)ksum_w[5],
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t_stats).count());
  }

  build_phase("range cache: BFS", t_bfs, s);
  // ---- bitmaps (packed masks in symbol space, exactly the hierarchy layout)
  const double t_bm = build_clock();
  const uint64_t N = nodes.size();
  if (h->cache_bm) (void)hipFree(h->cache_bm);
  h->cache_bm = nullptr;
  FM_HIP(hipMalloc(reinterpret_cast<void**>(&h->cache_bm), N * words * 4));
  {
    const uint64_t chunk = 32768;
    DBuf<uint64_t> d_lo, d_hi;
    if (d_lo.alloc(chunk) || d_hi.alloc(chunk)) return -1;
    std::vector<uint64_t> lo(chunk), hi(chunk);
    for (uint64_t c0 = 0; c0 < N; c0 += chunk) {
      const uint64_t m = std::min(chunk, N - c0);
      for (uint64_t i = 0; i < m; ++i) {
        lo[i] = nodes[c0 + i].first;
        hi[i] = nodes[c0 + i].second;
      }
      FM_HIP(hipMemcpyAsync(d_lo.p, lo.data(), m * 8, hipMemcpyHostToDevice, s));
      FM_HIP(hipMemcpyAsync(d_hi.p, hi.data(), m * 8, hipMemcpyHostToDevice, s));
      if (launch_mask(v, d_lo.p, d_hi.p, m, reinterpret_cast<uint8_t*>(h->cache_bm + c0 * words), words * 4,
                      words * 32, 0, 1, s))
        return -1;
      FM_HIP(hipStreamSynchronize(s));   // lo/hi host staging is reused
    }
  }

  build_phase("range cache: bitmaps", t_bm, s);
  // ---- (lo, hi) -> bitmap id, linear probing, load factor <= 1/2
  uint64_t cap = 1024;
  while (cap < 2 * N) cap <<= 1;
  std::vector<uint64_t> tab(2 * cap);
  for (uint64_t i = 0; i < cap; ++i) {
    tab[2 * i] = kCacheEmpty;
    tab[2 * i + 1] = 0;
  }
  for (uint64_t id = 0; id < N; ++id) {
    uint64_t slot = cache_hash(nodes[id].first, nodes[id].second) & (cap - 1);
    while (tab[2 * slot] != kCacheEmpty) slot = (slot + 1) & (cap - 1);
    tab[2 * slot] = nodes[id].first;
    tab[2 * slot + 1] = nodes[id].second | (id << kCacheIdShift);
  }
  if (h->cache_tab) (void)hipFree(h->cache_tab);
  h->cache_tab = nullptr;
  FM_HIP(hipMalloc(reinterpret_cast<void**>(&h->cache_tab), cap * 16));
  FM_HIP(hipMemcpyAsync(h->cache_tab, tab.data(), cap * 16, hipMemcpyHostToDevice, s));
  FM_HIP(hipStreamSynchronize(s));
  h->cache_nodes = N;
  h->cache_bytes = N * words * 4 + cap * 16;
  v.cache_bm = h->cache_bm;
  v.cache_tab = h->cache_tab;
  v.cache_min = Wc;
  v.cache_mask = cap - 1;

  // ---- per symbol: cache id + 1 of its C-block (the LF step from the full range)
  v.cblock = nullptr;
  if (h->cblock) (void)hipFree(h->cblock);
  h->cblock = nullptr;
  if (!root_child.empty()) {
    std::vector<uint32_t> cb((size_t)h->max_sym + 2, 0u);
    for (const auto& e : root_child)
      if (e.first < cb.size()) cb[e.first] = (uint32_t)(e.second + 1);
    FM_HIP(hipMalloc(reinterpret_cast<void**>(&h->cblock), cb.size() * 4));
    FM_HIP(hipMemcpyAsync(h->cblock, cb.data(), cb.size() * 4, hipMemcpyHostToDevice, s));
    FM_HIP(hipStreamSynchronize(s));
    v.cblock = h->cblock;
    h->cache_bytes += cb.size() * 4;
  }

  return build_transitions(h, nodes, s);
}

}  // namespace fmidx
