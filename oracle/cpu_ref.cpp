// cpu_ref.cpp -- CPU ORACLE / BASELINE, TEST INFRASTRUCTURE ONLY.
//
// A C++ -O3 restatement of the reference's hot path as the reference
// executes it on the CPU.  sdsl-lite (the library the reference links,
// README.md:23-31) is not vendored and cannot be built offline, so this
// restates its data structures and call pattern rather than linking it:
//
//   * wt_int-style levelwise wavelet TREE over the BWT: level l holds the
//     BWT stably sorted by the top l bits of the symbol; one concatenated
//     bit vector of L*n bits ([sdsl] wt_int, m_tree).
//   * rank_support_v-style directory: per 512-bit superblock one absolute
//     uint64 count + one uint64 of 7x9-bit relative counts ([sdsl]
//     rank_support_v<1>), i.e. two cache lines per rank.
//   * wt_int::rank(i, c): three rank queries per level (node offset, i, node
//     end); backward_search = two of those ([sdsl] backward_search,
//     called from fm_index.cpp:84).
//   * distinct_count (fm_index.cpp:119-144): three sigma-sized zeroed vectors
//     per call, then interval_symbols (width-1/2 special cases via
//     inverse_select, otherwise a left-first DFS with four ranks per node).
//   * distinct_count_multi (fm_index.cpp:146-166): rows fanned out over
//     threads (a fixed pool here instead of one std::async per row -- a
//     cheaper fan-out than the reference's, so the baseline is conservative).
//   * the mask row the processor scatters (document_constrained_generation_
//     causal_qwen.py:189-204) as a uint8 [vocab] row: zero + set.
//
// Only tests/ and bench.py's cpu_baseline leg load this library.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct RankV {
  const uint64_t* bits = nullptr;
  uint64_t nbits = 0;
  std::vector<uint64_t> dir;  // 2 words per 512-bit superblock
  void build(const uint64_t* b, uint64_t n) {
    bits = b;
    nbits = n;
    const uint64_t nwords = (n + 63) / 64;
    const uint64_t nsb = n / 512 + 1;
    dir.assign(2 * nsb, 0);
    uint64_t total = 0;
    for (uint64_t sb = 0; sb < nsb; ++sb) {
      dir[2 * sb] = total;
      uint64_t rel = 0, acc = 0;
      for (int w = 0; w < 8; ++w) {
        const uint64_t wi = sb * 8 + w;
        if (w > 0) rel |= acc << (9 * (w - 1));
        if (wi < nwords) acc += (uint64_t)__builtin_popcountll(b[wi]);
      }
      dir[2 * sb + 1] = rel;
      total += acc;
    }
  }
  inline uint64_t rank(uint64_t i) const {  // ones in [0, i)
    const uint64_t sb = i >> 9;
    const uint64_t w = (i >> 6) & 7;
    uint64_t r = dir[2 * sb];
    if (w) r += (dir[2 * sb + 1] >> (9 * (w - 1))) & 0x1FF;
    const uint64_t rem = i & 63;
    if (rem) r += (uint64_t)__builtin_popcountll(bits[i >> 6] & ((1ull << rem) - 1));
    return r;
  }
  inline bool access(uint64_t i) const { return (bits[i >> 6] >> (i & 63)) & 1ull; }
};

struct CpuRef {
  uint64_t n = 0;
  uint32_t L = 0;
  uint64_t sigma = 0;
  std::vector<uint64_t> tree;       // L*n bits
  RankV rk;
  std::vector<uint64_t> C;          // 2^L + 1 over symbol values
  std::vector<uint64_t> zero_cnt;   // zeros per level (for inverse_select)

  uint64_t tree_rank(uint64_t pos) const { return rk.rank(pos); }

  // [sdsl] wt_int::rank
  uint64_t rank(uint64_t i, uint64_t c) const {
    if ((1ull << L) <= c) return 0;
    uint64_t offset = 0, node_size = n;
    uint64_t mask = 1ull << (L - 1);
    for (uint32_t k = 0; k < L && i; ++k) {
      const uint64_t ones_o = tree_rank(offset);
      const uint64_t ones_i = tree_rank(offset + i) - ones_o;
      const uint64_t ones_end = tree_rank(offset + node_size) - ones_o;
      if (c & mask) {
        offset += (node_size - ones_end);
        node_size = ones_end;
        i = ones_i;
      } else {
        node_size = node_size - ones_end;
        i = i - ones_i;
      }
      offset += n;
      mask >>= 1;
    }
    return i;
  }

  // [sdsl] wt_int::inverse_select: (rank of symbol at i, symbol)
  std::pair<uint64_t, uint64_t> inverse_select(uint64_t i) const {
    uint64_t value = 0, offset = 0, node_size = n;
    for (uint32_t k = 0; k < L; ++k) {
      const uint64_t ones_o = tree_rank(offset);
      const uint64_t ones_i = tree_rank(offset + i) - ones_o;
      const uint64_t ones_end = tree_rank(offset + node_size) - ones_o;
      value <<= 1;
      if (rk.access(offset + i)) {
        offset += (node_size - ones_end);
        node_size = ones_end;
        i = ones_i;
        value |= 1;
      } else {
        node_size = node_size - ones_end;
        i = i - ones_i;
      }
      offset += n;
    }
    return {i, value};
  }

  void dfs(uint64_t i, uint64_t j, uint64_t& k, std::vector<uint64_t>& cs, std::vector<uint64_t>& ri,
           std::vector<uint64_t>& rj, uint32_t level, uint64_t path, uint64_t node_size,
           uint64_t offset) const {
    if (level >= L) {
      ri[k] = i;
      rj[k] = j;
      cs[k++] = path;
      return;
    }
    const uint64_t ones_o = tree_rank(offset);
    const uint64_t ones_i = tree_rank(offset + i) - ones_o;
    const uint64_t ones_j = tree_rank(offset + j) - ones_o;
    const uint64_t ones_end = tree_rank(offset + node_size) - ones_o;
    if ((j - i) - (ones_j - ones_i) > 0)
      dfs(i - ones_i, j - ones_j, k, cs, ri, rj, level + 1, path << 1, node_size - ones_end, offset + n);
    if ((ones_j - ones_i) > 0)
      dfs(ones_i, ones_j, k, cs, ri, rj, level + 1, (path << 1) | 1, ones_end,
          offset + (node_size - ones_end) + n);
  }

  // [sdsl] wt_int::interval_symbols
  void interval_symbols(uint64_t i, uint64_t j, uint64_t& k, std::vector<uint64_t>& cs,
                        std::vector<uint64_t>& ri, std::vector<uint64_t>& rj) const {
    if (i == j) {
      k = 0;
    } else if (j - i == 1) {
      k = 1;
      auto rc = inverse_select(i);
      ri[0] = rc.first;
      cs[0] = rc.second;
      rj[0] = ri[0] + 1;
    } else if (j - i == 2) {
      auto a = inverse_select(i);
      auto b = inverse_select(i + 1);
      ri[0] = a.first;
      cs[0] = a.second;
      ri[1] = b.first;
      cs[1] = b.second;
      if (cs[0] == cs[1]) {
        k = 1;
        rj[0] = ri[0] + 2;
      } else {
        k = 2;
        if (cs[0] > cs[1]) {
          std::swap(cs[0], cs[1]);
          std::swap(ri[0], ri[1]);
        }
        rj[0] = ri[0] + 1;
        rj[1] = ri[1] + 1;
      }
    } else {
      k = 0;
      dfs(i, j, k, cs, ri, rj, 0, 0, n, 0);
    }
  }

  bool known(uint64_t c) const { return c < (1ull << L) && (c == 0 || C[c + 1] > C[c]); }

  // fm_index.cpp:67-97 (+ sdsl backward_search): inclusive high in, half-open out
  void backward_search_step(uint64_t c, uint64_t low, uint64_t high, uint64_t& ol, uint64_t& oh) const {
    if (high >= n) high = n - 1;
    if (low > high) {
      ol = oh = 0;
      return;
    }
    uint64_t lr, rr;
    if (!known(c)) {
      lr = 1;
      rr = 0;
    } else {
      lr = C[c] + rank(low, c);
      rr = C[c] + rank(high + 1, c) - 1;
    }
    if (lr > rr) {
      ol = oh = 0;
      return;
    }
    ol = lr;
    oh = rr + 1;
  }

  // fm_index.cpp:119-144
  uint64_t distinct_count(uint64_t low, uint64_t high, std::vector<uint64_t>& out) const {
    std::vector<uint64_t> chars(sigma), rci(sigma), rcj(sigma);  // fresh, zeroed, per call
    out.clear();
    if (low == high) return 0;
    if (high > n) high = n;
    if (low >= high) return 0;
    uint64_t k = 0;
    interval_symbols(low, high, k, chars, rci, rcj);
    for (uint64_t q = 0; q < k; ++q) {
      out.push_back(chars[q]);
      out.push_back(rcj[q] - rci[q]);
    }
    return k;
  }
};

template <typename F>
void parallel_rows(uint64_t m, int threads, F&& f) {
  std::atomic<uint64_t> next{0};
  auto work = [&]() {
    std::vector<uint64_t> buf;
    for (;;) {
      const uint64_t i = next.fetch_add(1);
      if (i >= m) break;
      f(i, buf);
    }
  };
  if (threads <= 1) {
    work();
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) pool.emplace_back(work);
  for (auto& t : pool) t.join();
}

}  // namespace

extern "C" {

// levels: L arrays of ceil(n/64) words (level l = BWT stably sorted by its top l
// bits, bit l of each symbol, MSB first), concatenated per level; C: 2^L + 1.
void* cr_build(const uint64_t* level_words, uint64_t n, uint32_t L, const uint64_t* C, uint64_t sigma) {
  auto* h = new CpuRef();
  h->n = n;
  h->L = L;
  h->sigma = sigma;
  const uint64_t total_bits = (uint64_t)L * n;
  h->tree.assign((total_bits + 63) / 64 + 1, 0);
  const uint64_t wpl = (n + 63) / 64;
  for (uint32_t l = 0; l < L; ++l) {
    const uint64_t* src = level_words + (uint64_t)l * wpl;
    const uint64_t base = (uint64_t)l * n;
    if ((base & 63) == 0) {
      std::memcpy(&h->tree[base >> 6], src, wpl * 8);
      // clear bits past n in the last word (they belong to the next level)
      const uint64_t tail = n & 63;
      if (tail) h->tree[(base >> 6) + wpl - 1] &= (1ull << tail) - 1;
    } else {
      // unaligned level start: each source word lands in two destination words
      const uint32_t off = (uint32_t)(base & 63);
      uint64_t* dst = &h->tree[base >> 6];
      for (uint64_t w = 0; w < wpl; ++w) {
        uint64_t x = src[w];
        if (w + 1 == wpl && (n & 63)) x &= (1ull << (n & 63)) - 1;
        dst[w] |= x << off;
        dst[w + 1] |= x >> (64 - off);
      }
    }
  }
  h->rk.build(h->tree.data(), total_bits);
  h->C.assign(C, C + (1ull << L) + 1);
  return h;
}

void cr_free(void* p) { delete static_cast<CpuRef*>(p); }

void cr_backward_search_step(void* p, uint64_t c, uint64_t low, uint64_t high, uint64_t* out) {
  static_cast<CpuRef*>(p)->backward_search_step(c, low, high, out[0], out[1]);
}

uint64_t cr_distinct_count(void* p, uint64_t low, uint64_t high, uint64_t* out, uint64_t cap) {
  std::vector<uint64_t> v;
  const uint64_t k = static_cast<CpuRef*>(p)->distinct_count(low, high, v);
  std::memcpy(out, v.data(), std::min<uint64_t>(cap, v.size()) * 8);
  return k;
}

// One incremental decode step for m rows: LF step (token < reset_below ->
// full range), then distinct_count of the new range, then the uint8 mask row.
// distinct_seconds (single thread only, may be null): += the time spent in distinct_count, measured
// inside the same step -- the bench's breakdown of a single-thread step, a part of the same run.
void cr_decode_step_timed(void* p, const int64_t* tok, int64_t shift, int64_t reset_below, uint64_t* lo,
                          uint64_t* hi, uint64_t m, uint8_t* mask, uint64_t vocab, int threads,
                          double* distinct_seconds);

void cr_decode_step(void* p, const int64_t* tok, int64_t shift, int64_t reset_below, uint64_t* lo,
                    uint64_t* hi, uint64_t m, uint8_t* mask, uint64_t vocab, int threads) {
  cr_decode_step_timed(p, tok, shift, reset_below, lo, hi, m, mask, vocab, threads, nullptr);
}

void cr_decode_step_timed(void* p, const int64_t* tok, int64_t shift, int64_t reset_below, uint64_t* lo,
                          uint64_t* hi, uint64_t m, uint8_t* mask, uint64_t vocab, int threads,
                          double* distinct_seconds) {
  const CpuRef& h = *static_cast<CpuRef*>(p);
  const bool timed = distinct_seconds && threads <= 1;
  parallel_rows(m, threads, [&](uint64_t i, std::vector<uint64_t>& buf) {
    uint64_t l = lo[i], r = hi[i];
    if (tok[i] < reset_below) {
      l = 0;
      r = h.n;
    } else if (l >= r) {
      l = r = 0;
    } else {
      const int64_t s = tok[i] + shift;
      if (s < 0) {
        l = r = 0;
      } else {
        uint64_t ol, oh;
        h.backward_search_step((uint64_t)s, l, r - 1, ol, oh);
        l = ol;
        r = oh;
      }
    }
    lo[i] = l;
    hi[i] = r;
    const auto t0 = timed ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
    const uint64_t k = h.distinct_count(l, r, buf);
    if (timed) *distinct_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint8_t* row = mask + i * vocab;
    std::memset(row, 0, vocab);
    for (uint64_t q = 0; q < k; ++q) {
      const int64_t t = (int64_t)buf[2 * q] - shift;
      if (t >= 0 && (uint64_t)t < vocab) row[t] = 1;
    }
  });
}

// distinct_count (fm_index.cpp:119-144, sigma-sized zeroed scratch included) of
// m ranges, results discarded: the bench's single-thread step breakdown.
void cr_distinct_only(void* p, const uint64_t* lo, const uint64_t* hi, uint64_t m, int threads) {
  const CpuRef& h = *static_cast<CpuRef*>(p);
  parallel_rows(m, threads, [&](uint64_t i, std::vector<uint64_t>& buf) { h.distinct_count(lo[i], hi[i], buf); });
}

// index.py:103-114: get_range of tokens[a, b) from scratch, one
// backward_search_step per token, early exit at (0, 0).
inline void get_range(const CpuRef& h, const int64_t* tokens, int64_t a, int64_t b, int64_t shift, uint64_t& l,
                      uint64_t& r) {
  l = 0;
  r = h.n;
  for (int64_t j = a; j < b; ++j) {
    const int64_t s = tokens[j] + shift;
    uint64_t ol = 0, oh = 0;
    if (s >= 0) h.backward_search_step((uint64_t)s, l, r - 1, ol, oh);
    l = ol;
    r = oh;
    if (l == 0 && r == 0) break;
  }
}

// Reference-faithful step: get_range of the whole pattern from scratch +
// distinct_count.  faithful != 0 repeats the searches the Qwen processor makes
// per row (document_constrained_generation_causal_qwen.py:97,135,138):
// get_count([last]), get_range(sent), get_count(sent).
void cr_full_step(void* p, const int64_t* tokens, const int64_t* offsets, int64_t shift, uint64_t m,
                  uint64_t* lo, uint64_t* hi, uint8_t* mask, uint64_t vocab, int threads, int faithful) {
  const CpuRef& h = *static_cast<CpuRef*>(p);
  parallel_rows(m, threads, [&](uint64_t i, std::vector<uint64_t>& buf) {
    uint64_t l = 0, r = h.n;
    if (faithful && offsets[i + 1] > offsets[i]) {
      uint64_t l1, r1;
      get_range(h, tokens, offsets[i + 1] - 1, offsets[i + 1], shift, l1, r1);   // count([last])
      get_range(h, tokens, offsets[i], offsets[i + 1], shift, l1, r1);           // get_count(sent)
      buf.push_back(r1 - l1);   // keep the results live
      buf.clear();
    }
    get_range(h, tokens, offsets[i], offsets[i + 1], shift, l, r);
    lo[i] = l;
    hi[i] = r;
    const uint64_t k = h.distinct_count(l, r, buf);
    uint8_t* row = mask + i * vocab;
    std::memset(row, 0, vocab);
    for (uint64_t q = 0; q < k; ++q) {
      const int64_t t = (int64_t)buf[2 * q] - shift;
      if (t >= 0 && (uint64_t)t < vocab) row[t] = 1;
    }
  });
}

}  // extern "C"
