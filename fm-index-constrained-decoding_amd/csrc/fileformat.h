// fileformat.h -- the engine's own index file (fm_save / fm_load), host only.
//
// Layout (little endian): magic "FMIDXAMD", u32 version, u32 flags, u64 n,
// then BWT (n x u32);
//   version 2, flags & 4: SA samples = mark bits (ceil(n/64) x u64, bit i set
//     iff SA[i] % 32 == 0), sa_samp (ceil(n/32) x u32: SA / 32 of the marked
//     rows in row order), isa_samp ((n-1)/64 + 1 x u64: the row of text
//     position 64 k);
//   version 1, flags & 1: the full SA (n x u64), reduced to samples on load;
//   flags & 2: T' (n x u32; indexes built without a suffix array).
// It replaces the sdsl store_to_file / load_from_file pair of
// cpp_modules_linux/fm_index.cpp:196-209 (the reference's .fmi, whose sdsl
// layout fmidx/sdsl_fmi.py reads).
//
// Everything read is checked before it sizes an allocation or reaches the
// device: the file size must equal the size the header implies, n < 2^34, the
// BWT must hold exactly one sentinel and symbols below 2^kFileSymBits, the
// sample arrays must be consistent (marked-row count = ceil(n/32), no mark
// beyond row n - 1, every sample in range, a full SA a permutation).  A
// corrupt file is an error return, never a bad_alloc or an out-of-range row
// handed to the LF-walk kernels.  Host C++ only (no HIP), so the sanitizer
// build of tests/native/host_checks.cpp exercises it directly.
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace fmidx {

constexpr char kFileMagic[8] = {'F', 'M', 'I', 'D', 'X', 'A', 'M', 'D'};
constexpr uint64_t kFileSaRate = 32;
constexpr uint64_t kFileIsaRate = 64;
constexpr uint64_t kFileMaxRows = 1ull << 34;   // row positions are packed in 34 bits
constexpr int kFileSymBits = 26;                // = kMaxSymBits (fmidx_internal.h)

struct IndexFile {
  uint32_t version = 2;
  uint32_t flags = 0;
  uint64_t n = 0;
  std::vector<uint32_t> bwt, samp, text;
  std::vector<uint64_t> sa, mark, isa;
};

inline uint64_t file_mark_words(uint64_t n) { return (n + 63) / 64; }
inline uint64_t file_samp_count(uint64_t n) { return (n + kFileSaRate - 1) / kFileSaRate; }
inline uint64_t file_isa_count(uint64_t n) { return (n - 1) / kFileIsaRate + 1; }

// Bytes a file with this header must have (n < 2^34, so nothing overflows).
inline uint64_t file_expected_bytes(uint32_t version, uint32_t flags, uint64_t n) {
  uint64_t b = 24 + 4 * n;
  if (version == 1 && (flags & 1)) b += 8 * n;
  if (version == 2 && (flags & 4)) b += 8 * file_mark_words(n) + 4 * file_samp_count(n) + 8 * file_isa_count(n);
  if (flags & 2) b += 4 * n;
  return b;
}

namespace file_detail {

inline bool fail(std::string& err, const char* path, const char* what) {
  err = std::string(path ? path : "(null)") + ": " + what;
  return false;
}

template <typename T>
inline bool read_vec(std::FILE* f, std::vector<T>& v, uint64_t count) {
  v.resize(count);
  return count == 0 || std::fread(v.data(), sizeof(T), count, f) == count;
}

inline uint64_t popcount64(uint64_t x) {
  uint64_t c = 0;
  for (; x; x &= x - 1) ++c;
  return c;
}

}  // namespace file_detail

// Content checks shared by the reader and the writer.
inline bool validate_index_file(const IndexFile& x, const char* path, std::string& err) {
  using file_detail::fail;
  const uint64_t n = x.n;
  if (n == 0 || n >= kFileMaxRows) return fail(err, path, "row count out of range (0 < n < 2^34)");
  if (x.bwt.size() != n) return fail(err, path, "BWT length differs from n");
  uint64_t zeros = 0;
  for (uint32_t c : x.bwt) {
    if (c >> kFileSymBits) return fail(err, path, "BWT symbol beyond 2^26");
    zeros += c == 0;
  }
  if (zeros != 1) return fail(err, path, "BWT must hold exactly one sentinel 0");
  if (!x.sa.empty()) {
    if (x.sa.size() != n) return fail(err, path, "suffix array length differs from n");
    std::vector<uint64_t> seen(file_mark_words(n), 0);
    for (uint64_t p : x.sa) {
      if (p >= n) return fail(err, path, "suffix array value out of range");
      uint64_t& w = seen[p >> 6];
      if ((w >> (p & 63)) & 1) return fail(err, path, "suffix array is not a permutation");
      w |= 1ull << (p & 63);
    }
  }
  if (!x.mark.empty() || !x.samp.empty() || !x.isa.empty()) {
    const uint64_t nw = file_mark_words(n), ns = file_samp_count(n), ni = file_isa_count(n);
    if (x.mark.size() != nw || x.samp.size() != ns || x.isa.size() != ni)
      return fail(err, path, "sample arrays have the wrong length");
    uint64_t marked = 0;
    for (uint64_t w = 0; w < nw; ++w) marked += file_detail::popcount64(x.mark[w]);
    if (n & 63) {
      if (x.mark[nw - 1] >> (n & 63)) return fail(err, path, "mark bit set beyond the last row");
    }
    if (marked != ns) return fail(err, path, "marked rows differ from ceil(n / 32)");
    for (uint32_t s : x.samp)
      if ((uint64_t)s >= ns) return fail(err, path, "SA sample out of range");
    for (uint64_t r : x.isa)
      if (r >= n) return fail(err, path, "ISA sample (a row) out of range");
  }
  if (!x.text.empty() && x.text.size() != n) return fail(err, path, "text length differs from n");
  return true;
}

inline bool read_index_file(const char* path, IndexFile& x, std::string& err) {
  using file_detail::fail;
  if (!path) return fail(err, path, "null path");
  std::FILE* f = std::fopen(path, "rb");
  if (!f) return fail(err, path, "cannot open");
  struct Closer {
    std::FILE* f;
    ~Closer() { std::fclose(f); }
  } closer{f};
  if (std::fseek(f, 0, SEEK_END) != 0) return fail(err, path, "cannot seek");
  const long long size = std::ftell(f);
  if (size < 0 || std::fseek(f, 0, SEEK_SET) != 0) return fail(err, path, "cannot seek");
  char magic[8];
  uint32_t version = 0, flags = 0;
  uint64_t n = 0;
  if (std::fread(magic, 1, 8, f) != 8 || std::fread(&version, 4, 1, f) != 1 || std::fread(&flags, 4, 1, f) != 1 ||
      std::fread(&n, 8, 1, f) != 1 || std::memcmp(magic, kFileMagic, 8) != 0)
    return fail(err, path, "not an fmidx index file");
  if (version != 1 && version != 2) return fail(err, path, "unsupported version");
  const uint32_t allowed = version == 1 ? 3u : 6u;
  if (flags & ~allowed) return fail(err, path, "unknown flags");
  if (n == 0 || n >= kFileMaxRows) return fail(err, path, "row count out of range (0 < n < 2^34)");
  if ((uint64_t)size != file_expected_bytes(version, flags, n))
    return fail(err, path, "file size differs from the size its header implies (truncated or corrupt)");
  x = IndexFile{};
  x.version = version;
  x.flags = flags;
  x.n = n;
  bool ok = file_detail::read_vec(f, x.bwt, n);
  if (ok && version == 1 && (flags & 1)) ok = file_detail::read_vec(f, x.sa, n);
  if (ok && version == 2 && (flags & 4))
    ok = file_detail::read_vec(f, x.mark, file_mark_words(n)) && file_detail::read_vec(f, x.samp, file_samp_count(n)) &&
         file_detail::read_vec(f, x.isa, file_isa_count(n));
  if (ok && (flags & 2)) ok = file_detail::read_vec(f, x.text, n);
  if (!ok) return fail(err, path, "short read");
  return validate_index_file(x, path, err);
}

// Writes version 2 (flags from the arrays present: samples 4, text 2).
inline bool write_index_file(const char* path, IndexFile x, std::string& err) {
  using file_detail::fail;
  x.version = 2;
  x.sa.clear();
  x.flags = (!x.mark.empty() ? 4u : 0u) | (x.mark.empty() && !x.text.empty() ? 2u : 0u);
  if (!(x.flags & 2)) x.text.clear();
  if (!validate_index_file(x, path, err)) return false;
  std::FILE* f = path ? std::fopen(path, "wb") : nullptr;
  if (!f) return fail(err, path, "cannot write");
  bool ok = std::fwrite(kFileMagic, 1, 8, f) == 8 && std::fwrite(&x.version, 4, 1, f) == 1 &&
            std::fwrite(&x.flags, 4, 1, f) == 1 && std::fwrite(&x.n, 8, 1, f) == 1 &&
            std::fwrite(x.bwt.data(), 4, x.n, f) == x.n;
  if (ok && (x.flags & 4))
    ok = std::fwrite(x.mark.data(), 8, x.mark.size(), f) == x.mark.size() &&
         std::fwrite(x.samp.data(), 4, x.samp.size(), f) == x.samp.size() &&
         std::fwrite(x.isa.data(), 8, x.isa.size(), f) == x.isa.size();
  if (ok && (x.flags & 2)) ok = std::fwrite(x.text.data(), 4, x.n, f) == x.n;
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) return fail(err, path, "write failed");
  return true;
}

}  // namespace fmidx
