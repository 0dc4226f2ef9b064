// host_checks.cpp -- the host-only native code under AddressSanitizer +
// UndefinedBehaviorSanitizer (built and run by tests/test_native_sanitizers.py
// on the CPU; never on the GPU box, whose pool refuses sanitizer runs of GPU
// code).  Covers:
//   * csrc/sais.h: SA-IS (the host suffix sorter of FMIndex.initialize for
//     corpora below 2^20 tokens) against sorting the suffixes by definition,
//     over random, periodic and single-symbol texts and wide alphabets;
//   * csrc/fileformat.h: fm_save / fm_load's parse -- a valid file round trips,
//     and truncated, extended and corrupt files (header, sizes, samples,
//     sentinel, symbols) are refused with a message, never a crash;
//   * oracle/cpu_ref.cpp (linked in): backward_search_step, distinct_count and
//     decode_step on a small index against counting over the suffix array.
// Exit status 0 = every check passed; sanitizer reports abort the run.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../fm-index-constrained-decoding_amd/csrc/fileformat.h"
#include "../../fm-index-constrained-decoding_amd/csrc/sais.h"

extern "C" {
void* cr_build(const uint64_t* level_words, uint64_t n, uint32_t L, const uint64_t* C, uint64_t sigma);
void cr_free(void* p);
void cr_backward_search_step(void* p, uint64_t c, uint64_t low, uint64_t high, uint64_t* out);
uint64_t cr_distinct_count(void* p, uint64_t low, uint64_t high, uint64_t* out, uint64_t cap);
void cr_decode_step(void* p, const int64_t* tok, int64_t shift, int64_t reset_below, uint64_t* lo, uint64_t* hi,
                    uint64_t m, uint8_t* mask, uint64_t vocab, int threads);
}

static int g_fail = 0;
#define CHECK(cond, ...)                                      \
  do {                                                        \
    if (!(cond)) {                                            \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                      \
      std::fprintf(stderr, "\n");                             \
      ++g_fail;                                               \
    }                                                         \
  } while (0)

static std::vector<uint64_t> naive_sa(const std::vector<uint32_t>& t) {
  std::vector<uint64_t> sa(t.size());
  for (uint64_t i = 0; i < t.size(); ++i) sa[i] = i;
  std::sort(sa.begin(), sa.end(), [&](uint64_t a, uint64_t b) {
    return std::lexicographical_compare(t.begin() + a, t.end(), t.begin() + b, t.end());
  });
  return sa;
}

// T' = body + sentinel 0, body symbols in [1, K)
static std::vector<uint32_t> make_text(std::mt19937_64& rng, uint64_t n, uint32_t K, int kind) {
  std::vector<uint32_t> t(n);
  for (uint64_t i = 0; i + 1 < n; ++i) {
    if (kind == 0) t[i] = 1 + (uint32_t)(rng() % (K - 1));
    else if (kind == 1) t[i] = 1 + (uint32_t)(i % 3);                   // periodic
    else if (kind == 2) t[i] = 7;                                       // one symbol
    else t[i] = 1 + (uint32_t)((i * i / 5 + (rng() % 4 == 0 ? rng() % 3 : 0)) % (K - 1));
  }
  t[n - 1] = 0;
  return t;
}

static void check_sais() {
  std::mt19937_64 rng(20250905);
  const uint64_t sizes[] = {1, 2, 3, 17, 64, 1000, 4099};
  const uint32_t alphas[] = {3, 40, 300, 130000};
  int cases = 0;
  for (uint64_t n : sizes)
    for (uint32_t K : alphas)
      for (int kind = 0; kind < 4; ++kind) {
        auto t = make_text(rng, n, std::max<uint32_t>(K, 9), kind == 0 && K == 3 ? 0 : kind);
        if (K == 3)   // a binary body {1, 2}
          for (uint64_t i = 0; i + 1 < n; ++i) t[i] = 1 + (t[i] & 1);
        uint32_t maxs = *std::max_element(t.begin(), t.end());
        std::vector<int32_t> sa32;
        fmidx::suffix_array<int32_t>(t.data(), (int64_t)n, maxs + 1, sa32);
        std::vector<int64_t> sa64;
        fmidx::suffix_array<int64_t>(t.data(), (int64_t)n, maxs + 1, sa64);
        const auto want = naive_sa(t);
        bool ok32 = sa32.size() == n, ok64 = sa64.size() == n;
        for (uint64_t i = 0; i < n && ok32 && ok64; ++i) {
          ok32 = (uint64_t)sa32[i] == want[i];
          ok64 = (uint64_t)sa64[i] == want[i];
        }
        CHECK(ok32 && ok64, "SA-IS differs from sorting (n=%llu K=%u kind=%d)", (unsigned long long)n, K, kind);
        ++cases;
      }
  // the empty text is refused
  bool threw = false;
  try {
    std::vector<int32_t> sa;
    fmidx::suffix_array<int32_t>(nullptr, 0, 1, sa);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw, "empty text accepted");
  std::printf("sais: %d cases\n", cases);
}

// The file of a text's index, built by definition (SA by SA-IS).
static fmidx::IndexFile file_of(const std::vector<uint32_t>& t) {
  const uint64_t n = t.size();
  std::vector<int64_t> sa;
  fmidx::suffix_array<int64_t>(t.data(), (int64_t)n, *std::max_element(t.begin(), t.end()) + 1, sa);
  fmidx::IndexFile f;
  f.n = n;
  f.bwt.resize(n);
  f.mark.assign(fmidx::file_mark_words(n), 0);
  f.isa.assign(fmidx::file_isa_count(n), 0);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t p = (uint64_t)sa[i];
    f.bwt[i] = t[p == 0 ? n - 1 : p - 1];
    if (p % 32 == 0) {
      f.mark[i >> 6] |= 1ull << (i & 63);
      f.samp.push_back((uint32_t)(p / 32));
    }
    if (p % 64 == 0) f.isa[p / 64] = i;
  }
  return f;
}

static std::vector<unsigned char> slurp(const std::string& path) {
  std::vector<unsigned char> b;
  if (std::FILE* f = std::fopen(path.c_str(), "rb")) {
    int c;
    while ((c = std::fgetc(f)) != EOF) b.push_back((unsigned char)c);
    std::fclose(f);
  }
  return b;
}

static void spit(const std::string& path, const std::vector<unsigned char>& b) {
  std::FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return;
  if (!b.empty()) std::fwrite(b.data(), 1, b.size(), f);
  std::fclose(f);
}

template <typename T>
static void poke(std::vector<unsigned char>& b, size_t off, T v) {
  if (off + sizeof(T) <= b.size()) std::memcpy(b.data() + off, &v, sizeof(T));
}

static void check_fileformat(const std::string& dir) {
  std::mt19937_64 rng(7);
  std::string err;
  int refused = 0;
  for (uint64_t n : {1ull, 2ull, 65ull, 200ull, 3001ull}) {
    const auto t = make_text(rng, n, 500, 0);
    const auto f = file_of(t);
    const std::string path = dir + "/ok_" + std::to_string(n) + ".fmidx";
    CHECK(fmidx::write_index_file(path.c_str(), f, err), "write failed: %s", err.c_str());
    fmidx::IndexFile g;
    CHECK(fmidx::read_index_file(path.c_str(), g, err), "read of a valid file failed: %s", err.c_str());
    CHECK(g.n == n && g.bwt == f.bwt && g.mark == f.mark && g.samp == f.samp && g.isa == f.isa,
          "round trip differs (n=%llu)", (unsigned long long)n);
    const auto good = slurp(path);
    CHECK(good.size() == fmidx::file_expected_bytes(2, 4, n), "size model");
    const uint64_t ob = 24, om = ob + 4 * n, os = om + 8 * fmidx::file_mark_words(n),
                   oi = os + 4 * fmidx::file_samp_count(n);
    auto refuse = [&](const char* what, std::vector<unsigned char> b) {
      const std::string p = dir + "/bad.fmidx";
      spit(p, b);
      fmidx::IndexFile h;
      std::string e;
      const bool ok = fmidx::read_index_file(p.c_str(), h, e);
      CHECK(!ok && !e.empty(), "corrupt file accepted (%s, n=%llu)", what, (unsigned long long)n);
      refused += !ok;
    };
    auto b = good;
    b.pop_back();
    refuse("truncated by one byte", b);
    refuse("truncated header", std::vector<unsigned char>(good.begin(), good.begin() + 12));
    refuse("empty file", {});
    b = good;
    b.push_back(0);
    refuse("one byte too many", b);
    b = good;
    b[0] = 'X';
    refuse("bad magic", b);
    b = good;
    poke<uint32_t>(b, 8, 3);
    refuse("unknown version", b);
    b = good;
    poke<uint32_t>(b, 12, 4 | 8);
    refuse("unknown flag", b);
    b = good;
    poke<uint64_t>(b, 16, 1ull << 40);
    refuse("n beyond 2^34", b);
    b = good;
    poke<uint64_t>(b, 16, ~0ull);
    refuse("n = 2^64 - 1", b);
    b = good;
    poke<uint64_t>(b, 16, 0);
    refuse("n = 0", b);
    b = good;
    poke<uint64_t>(b, 16, n + 1);
    refuse("n off by one", b);
    b = good;
    poke<uint32_t>(b, ob, f.bwt[0] == 0 ? 1u : 0u);         // a second (or no) sentinel
    refuse("sentinel count", b);
    b = good;
    poke<uint32_t>(b, ob + 4 * (n - 1), 1u << 27);
    refuse("symbol beyond 2^26", b);
    b = good;
    poke<uint64_t>(b, oi, n);                                 // isa[0] = n: a row past the end
    refuse("ISA sample out of range", b);
    b = good;
    poke<uint32_t>(b, os, (uint32_t)fmidx::file_samp_count(n));
    refuse("SA sample out of range", b);
    b = good;
    {
      uint64_t w0 = 0;
      std::memcpy(&w0, good.data() + om, 8);
      poke<uint64_t>(b, om, w0 ^ 2ull);                        // one mark too many or too few
      if (n > 1) refuse("mark count", b);
    }
    if (n % 64) {
      b = good;
      const size_t last = om + 8 * (fmidx::file_mark_words(n) - 1);
      uint64_t w = 0;
      std::memcpy(&w, good.data() + last, 8);
      poke<uint64_t>(b, last, w | (1ull << 63));
      refuse("mark beyond the last row", b);
    }
  }
  // version 1 with a full SA: a non-permutation is refused
  {
    const auto t = make_text(rng, 300, 50, 0);
    std::vector<int64_t> sa;
    fmidx::suffix_array<int64_t>(t.data(), 300, 51, sa);
    std::vector<unsigned char> b(24 + 300 * 4 + 300 * 8);
    std::memcpy(b.data(), fmidx::kFileMagic, 8);
    poke<uint32_t>(b, 8, 1);
    poke<uint32_t>(b, 12, 1);
    poke<uint64_t>(b, 16, 300);
    for (uint64_t i = 0; i < 300; ++i) {
      const uint64_t p = (uint64_t)sa[i];
      poke<uint32_t>(b, 24 + 4 * i, t[p == 0 ? 299 : p - 1]);
      poke<uint64_t>(b, 24 + 1200 + 8 * i, p);
    }
    const std::string p = dir + "/v1.fmidx";
    spit(p, b);
    fmidx::IndexFile g;
    CHECK(fmidx::read_index_file(p.c_str(), g, err), "valid version-1 file refused: %s", err.c_str());
    poke<uint64_t>(b, 24 + 1200 + 8 * 5, (uint64_t)sa[6]);   // a duplicate position
    spit(p, b);
    CHECK(!fmidx::read_index_file(p.c_str(), g, err), "version-1 SA duplicate accepted");
    ++refused;
  }
  {
    fmidx::IndexFile g;
    CHECK(!fmidx::read_index_file((dir + "/missing.fmidx").c_str(), g, err), "a missing file read");
    CHECK(!fmidx::read_index_file(nullptr, g, err), "a null path read");
  }
  std::printf("fileformat: %d corrupt files refused\n", refused);
}

static void check_cpu_ref() {
  std::mt19937_64 rng(11);
  const uint64_t n = 2500;
  auto t = make_text(rng, n, 60, 0);
  std::vector<int64_t> sa;
  fmidx::suffix_array<int64_t>(t.data(), (int64_t)n, 61, sa);
  std::vector<uint32_t> bwt(n);
  for (uint64_t i = 0; i < n; ++i) bwt[i] = t[sa[i] == 0 ? n - 1 : sa[i] - 1];
  const uint32_t L = 6;                                 // symbols < 64
  const uint64_t wpl = (n + 63) / 64;
  std::vector<uint64_t> words(L * wpl, 0);
  std::vector<uint32_t> seq = bwt;
  for (uint32_t lev = 0; lev < L; ++lev) {
    if (lev) std::stable_sort(seq.begin(), seq.end(), [&](uint32_t a, uint32_t b) {
      return (a >> (L - lev)) < (b >> (L - lev));
    });
    for (uint64_t i = 0; i < n; ++i)
      if ((seq[i] >> (L - 1 - lev)) & 1) words[lev * wpl + (i >> 6)] |= 1ull << (i & 63);
  }
  std::vector<uint64_t> C((1u << L) + 1, 0);
  uint64_t sigma = 0;
  {
    std::vector<uint64_t> cnt(1u << L, 0);
    for (uint32_t c : bwt) cnt[c]++;
    for (uint32_t c = 0; c < (1u << L); ++c) {
      C[c + 1] = C[c] + cnt[c];
      sigma += cnt[c] > 0;
    }
  }
  void* h = cr_build(words.data(), n, L, C.data(), sigma);
  CHECK(h != nullptr, "cr_build");
  int checked = 0;
  for (int q = 0; q < 400; ++q) {
    uint64_t a = rng() % n, b = a + rng() % (n - a);
    const uint32_t c = (uint32_t)(rng() % 64);
    uint64_t out[2];
    cr_backward_search_step(h, c, a, b, out);
    // by definition: rows of [C[c], C[c+1]) whose previous row-symbol count ... = occurrences of c in BWT[a, b]
    uint64_t before = 0, inside = 0;
    for (uint64_t i = 0; i < a; ++i) before += bwt[i] == c;
    for (uint64_t i = a; i <= b; ++i) inside += bwt[i] == c;
    const bool known = c == 0 || C[c + 1] > C[c];
    if (known && inside) {
      CHECK(out[0] == C[c] + before && out[1] == C[c] + before + inside, "backward_search_step (%u, %llu, %llu)", c,
            (unsigned long long)a, (unsigned long long)b);
    } else {
      CHECK(out[0] == 0 && out[1] == 0, "empty backward_search_step");
    }
    std::vector<uint64_t> dc(2 * 64);
    const uint64_t k = cr_distinct_count(h, a, b + 1, dc.data(), dc.size());
    std::vector<uint64_t> cnt(64, 0);
    for (uint64_t i = a; i <= b; ++i) cnt[bwt[i]]++;
    uint64_t j = 0;
    bool ok = true;
    for (uint32_t s = 0; s < 64; ++s)
      if (cnt[s]) {
        ok = ok && j < k && dc[2 * j] == s && dc[2 * j + 1] == cnt[s];
        ++j;
      }
    CHECK(ok && j == k, "distinct_count [%llu, %llu)", (unsigned long long)a, (unsigned long long)(b + 1));
    ++checked;
  }
  // decode_step: one LF step + mask row, 2 threads
  const uint64_t B = 64, V = 70;
  std::vector<int64_t> tok(B);
  std::vector<uint64_t> lo(B), hi(B);
  std::vector<uint8_t> mask(B * V);
  for (uint64_t r = 0; r < B; ++r) {
    lo[r] = rng() % n;
    hi[r] = std::min<uint64_t>(n, lo[r] + rng() % 300);
    tok[r] = r % 9 == 0 ? -1 : (int64_t)(rng() % 60) - 10;
  }
  auto lo0 = lo, hi0 = hi;
  cr_decode_step(h, tok.data(), 10, 0, lo.data(), hi.data(), B, mask.data(), V, 2);
  for (uint64_t r = 0; r < B; ++r) {
    uint64_t el = 0, eh = n;
    if (tok[r] >= 0) {
      const uint32_t c = (uint32_t)(tok[r] + 10);
      uint64_t before = 0, inside = 0;
      for (uint64_t i = 0; i < lo0[r]; ++i) before += bwt[i] == c;
      for (uint64_t i = lo0[r]; i < hi0[r]; ++i) inside += bwt[i] == c;
      el = inside ? C[c] + before : 0;
      eh = inside ? C[c] + before + inside : 0;
    }
    CHECK(lo[r] == el && hi[r] == eh, "decode_step range row %llu", (unsigned long long)r);
    bool ok = true;
    for (uint64_t v = 0; v < V; ++v) {
      bool in = false;
      for (uint64_t i = el; i < eh && !in; ++i) in = bwt[i] == v + 10;
      ok = ok && mask[r * V + v] == (in ? 1 : 0);
    }
    CHECK(ok, "decode_step mask row %llu", (unsigned long long)r);
  }
  cr_free(h);
  std::printf("cpu_ref: %d queries + %llu decode rows\n", checked, (unsigned long long)B);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  check_sais();
  check_fileformat(dir);
  check_cpu_ref();
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("all host checks passed\n");
  return 0;
}
