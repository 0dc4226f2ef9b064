// sais.h -- host suffix-array construction by induced sorting (SA-IS) over an
// integer alphabet.  Replaces the construction half of sdsl ``construct`` /
// ``construct_im`` used by the reference (cpp_modules_linux/fm_index.cpp:37,44):
// the text passed in already ends with the unique minimal sentinel 0, so the
// suffix array -- and everything derived from it -- is uniquely defined.
//
// Index type I must be signed (the empty-slot marker is -1).  O(n) time,
// n*sizeof(I) extra bytes for the reduced problem plus a bit vector of types.
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace fmidx {
namespace sais_detail {

template <typename I, typename C>
static void bucket_bounds(const C* s, I n, I K, std::vector<I>& bkt, bool ends) {
  bkt.assign(static_cast<size_t>(K), 0);
  for (I i = 0; i < n; ++i) bkt[static_cast<size_t>(s[i])]++;
  I run = 0;
  for (I c = 0; c < K; ++c) {
    run += bkt[c];
    bkt[c] = ends ? run : run - bkt[c];
  }
}

// L-type suffixes are induced left-to-right from bucket heads, S-type
// right-to-left from bucket tails.
template <typename I, typename C>
static void induce(const C* s, I* SA, I n, I K, const std::vector<bool>& stype, std::vector<I>& bkt) {
  bucket_bounds(s, n, K, bkt, false);
  for (I i = 0; i < n; ++i) {
    I j = SA[i] - 1;
    if (SA[i] > 0 && !stype[static_cast<size_t>(j)]) SA[bkt[static_cast<size_t>(s[j])]++] = j;
  }
  bucket_bounds(s, n, K, bkt, true);
  for (I i = n - 1; i >= 0; --i) {
    I j = SA[i] - 1;
    if (SA[i] > 0 && stype[static_cast<size_t>(j)]) SA[--bkt[static_cast<size_t>(s[j])]] = j;
  }
}

template <typename I, typename C>
static void sais_rec(const C* s, I* SA, I n, I K) {
  if (n == 1) {
    SA[0] = 0;
    return;
  }
  std::vector<bool> stype(static_cast<size_t>(n));
  stype[static_cast<size_t>(n - 1)] = true;
  for (I i = n - 2; i >= 0; --i)
    stype[static_cast<size_t>(i)] =
        s[i] < s[i + 1] || (s[i] == s[i + 1] && stype[static_cast<size_t>(i + 1)]);
  auto lms = [&](I i) {
    return i > 0 && stype[static_cast<size_t>(i)] && !stype[static_cast<size_t>(i - 1)];
  };

  std::vector<I> bkt;
  // 1. seed LMS positions at bucket tails, induce -> LMS substrings sorted
  bucket_bounds(s, n, K, bkt, true);
  std::fill(SA, SA + n, I(-1));
  for (I i = 1; i < n; ++i)
    if (lms(i)) SA[--bkt[static_cast<size_t>(s[i])]] = i;
  induce(s, SA, n, K, stype, bkt);

  // 2. compact sorted LMS substrings into SA[0, n1), then name them
  I n1 = 0;
  for (I i = 0; i < n; ++i)
    if (lms(SA[i])) SA[n1++] = SA[i];
  std::fill(SA + n1, SA + n, I(-1));
  I names = 0;
  I prev = -1;
  for (I i = 0; i < n1; ++i) {
    const I pos = SA[i];
    bool differ = false;
    for (I d = 0;; ++d) {
      if (prev < 0 || pos + d >= n || prev + d >= n || s[pos + d] != s[prev + d] ||
          stype[static_cast<size_t>(pos + d)] != stype[static_cast<size_t>(prev + d)]) {
        differ = true;
        break;
      }
      if (d > 0 && (lms(pos + d) || lms(prev + d))) break;
    }
    if (differ) {
      ++names;
      prev = pos;
    }
    SA[n1 + pos / 2] = names - 1;
  }
  for (I i = n - 1, j = n - 1; i >= n1; --i)
    if (SA[i] >= 0) SA[j--] = SA[i];

  // 3. sort the reduced string (recursively when names repeat)
  I* SA1 = SA;
  I* s1 = SA + n - n1;
  if (names < n1) {
    sais_rec<I, I>(s1, SA1, n1, names);
  } else {
    for (I i = 0; i < n1; ++i) SA1[s1[i]] = i;
  }

  // 4. map reduced ranks back to text positions and induce the final order
  for (I i = 1, j = 0; i < n; ++i)
    if (lms(i)) s1[j++] = i;
  for (I i = 0; i < n1; ++i) SA1[i] = s1[SA1[i]];
  std::fill(SA + n1, SA + n, I(-1));
  bucket_bounds(s, n, K, bkt, true);
  for (I i = n1 - 1; i >= 0; --i) {
    const I j = SA[i];
    SA[i] = -1;
    SA[--bkt[static_cast<size_t>(s[j])]] = j;
  }
  induce(s, SA, n, K, stype, bkt);
}

}  // namespace sais_detail

// Suffix array of text[0, n) (text[n-1] must be the unique minimum, 0).
// Symbols must be < K.  Returns positions as uint64.
template <typename I>
inline void suffix_array(const uint32_t* text, int64_t n, uint32_t K, std::vector<I>& sa) {
  if (n <= 0) throw std::invalid_argument("empty text");
  sa.resize(static_cast<size_t>(n));
  sais_detail::sais_rec<I, uint32_t>(text, sa.data(), static_cast<I>(n), static_cast<I>(K));
}

}  // namespace fmidx
