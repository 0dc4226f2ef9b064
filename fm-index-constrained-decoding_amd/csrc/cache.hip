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

uint64_t env_u64(const char* name, uint64_t dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::strtoull(v, nullptr, 10) : dflt;
}

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

int device_build_cache(Index* h, hipStream_t s) {
  DevView& v = h->view;
  v.cache_mask = 0;
  v.cache_bm = nullptr;
  v.cache_tab = nullptr;
  const uint64_t n = h->n;
  const uint64_t Wc = std::max<uint64_t>(2, env_u64("FMIDX_CACHE_MIN", 4096));
  const uint64_t budget = env_u64("FMIDX_CACHE_MB", 48ull << 10) << 20;
  const uint64_t words = v.bm_words;
  if (words == 0 || v.bm_levels == 0 || n < Wc || budget == 0) return 0;
  const uint64_t max_nodes = std::max<uint64_t>(1, budget / (words * 4));

  // ---- breadth-first enumeration of the ranges with width >= Wc
  std::vector<std::pair<uint64_t, uint64_t>> nodes;
  std::unordered_map<std::pair<uint64_t, uint64_t>, uint64_t, PairHash> seen;   // range -> id
  std::vector<std::pair<uint64_t, uint64_t>> frontier{{0, n}}, next;
  nodes.push_back({0, n});
  seen.emplace(std::make_pair(uint64_t(0), n), 0);
  struct Edge {
    uint64_t plo, phi, c, clo, cw, id;
  };
  std::vector<Edge> edges;   // parent (not the root) -> cached child
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
          if (!(lo[r] == 0 && hi[r] == n)) edges.push_back({lo[r], hi[r], sym[off[r] + j], a, b - a, id});
        }
      }
      i0 = i1;
    }
    frontier.swap(next);
  }
  seen.clear();

  if (env_u64("FMIDX_CACHE_STATS", 0)) {
    // diagnostic: distinct symbols summed over the cached ranges, and their width histogram
    uint64_t sum = 0, maxk = 0, hist[8] = {0, 0, 0, 0, 0, 0, 0, 0};
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
        int b = 0;
        while (b < 7 && k[r] >= (16ull << (2 * b))) ++b;
        hist[b]++;
      }
      i0 = i1;
    }
    fprintf(stderr, "[fmidx] cache: %zu ranges >= %llu, distinct symbols summed %llu (max %llu); "
            "distinct-count histogram <16,<64,<256,<1K,<4K,<16K,<64K,>=: %llu %llu %llu %llu %llu %llu %llu %llu; "
            "edges between cached ranges %zu\n", nodes.size(), (unsigned long long)Wc, (unsigned long long)sum,
            (unsigned long long)maxk, (unsigned long long)hist[0], (unsigned long long)hist[1],
            (unsigned long long)hist[2], (unsigned long long)hist[3], (unsigned long long)hist[4],
            (unsigned long long)hist[5], (unsigned long long)hist[6], (unsigned long long)hist[7], edges.size());
  }

  // ---- bitmaps (packed masks in symbol space, exactly the hierarchy layout)
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

  // ---- edge table (cached parent, c) -> cached child: linear probing with
  //      every key within 16 slots of its home (one 512-B probe round)
  v.trans_mask = 0;
  v.trans_tab = nullptr;
  if (edges.empty() || env_u64("FMIDX_EDGE_TABLE", 1) == 0) return 0;
  uint64_t tcap = 1024;
  while (tcap < 4 * edges.size()) tcap <<= 1;
  std::vector<uint64_t> et;
  for (;;) {
    et.assign(4 * tcap, 0);
    for (uint64_t i = 0; i < tcap; ++i) et[4 * i] = kCacheEmpty;
    bool ok = true;
    for (const Edge& e : edges) {
      const uint64_t home = trans_hash(e.plo, e.phi, e.c) & (tcap - 1);
      uint64_t d = 0;
      while (d < 16 && et[4 * ((home + d) & (tcap - 1))] != kCacheEmpty) ++d;
      if (d == 16) {
        ok = false;
        break;
      }
      uint64_t* slot = &et[4 * ((home + d) & (tcap - 1))];
      slot[0] = e.plo;
      slot[1] = e.phi | (e.c << kCacheIdShift);
      slot[2] = e.clo;
      slot[3] = e.cw | ((e.id + 1) << kCacheIdShift);
    }
    if (ok) break;
    tcap <<= 1;
  }
  FM_HIP(hipMalloc(reinterpret_cast<void**>(&h->trans_tab), tcap * 32));
  FM_HIP(hipMemcpyAsync(h->trans_tab, et.data(), tcap * 32, hipMemcpyHostToDevice, s));
  FM_HIP(hipStreamSynchronize(s));
  h->trans_entries = edges.size();
  h->cache_bytes += tcap * 32;
  v.trans_tab = h->trans_tab;
  v.trans_mask = tcap - 1;
  return 0;
}

}  // namespace fmidx
