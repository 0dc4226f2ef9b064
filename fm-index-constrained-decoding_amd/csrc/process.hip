// process.hip -- the per-row bookkeeping of the logits processors on the
// device (fm_processor_step; fm_processor_call runs it and the two launches
// after it in one host call), so a processor call has no per-row host work:
//   k_prep      one wave per row: remove_end_marker, finished_thinking,
//               remove_system_tokens, the trailing n-gram rule, the eos / pad
//               / stop_at_count rules and the pattern's range
//               (document_constrained_generation_causal_qwen.py:44-99,
//               :101-214; document_constrained_generation_causal.py:62-180);
//               FM_PREP_HARD: the hard-mask variants (vllm.py:46-137,
//               seq.py:35-123) -- pattern from `skip` on, no trailing n-gram
//               rule, stop_at_count on the count of the pattern without its
//               last token; writes the epilogue's fm_row_params
//   fm_allowed_mask_batch(packed)   the allowed bits of the rows that need them
//   fm_apply_boosts                 scores + mask in the scores dtype
// The pattern's range is ONE LF step from the previous call's range when the
// row's pattern extends a pattern of the previous call (same beam group,
// compared token by token: the beam search may reorder rows), exactly
// get_range's left-to-right loop (index.py:103-114) resumed; otherwise the
// whole force_decoding_from + sent is searched.
#include "fmidx_internal.h"
#include "../../include/fmidx.h"

namespace fmidx {

namespace {

constexpr int64_t kStageBatch = 512;           // row tokens staged per batch (8 loads per lane in flight)
constexpr int64_t kMaxStaged = 6144;           // rows up to this many tokens are staged in LDS (48 KB)
enum Kind : uint32_t { kNone = 0, kUni = 1, kSpecial = 2, kBits = 3 };

// all 64 lanes: a[j] == b[j] for j < len
__device__ __forceinline__ bool wave_equal(const int64_t* a, const int64_t* b, int64_t len) {
  const uint32_t lane = threadIdx.x & 63u;
  bool ok = true;
  for (int64_t j0 = 0; j0 < len; j0 += 64) {
    const int64_t j = j0 + lane;
    const bool diff = j < len && a[j] != b[j];
    if (__ballot(diff)) {
      ok = false;
      break;
    }
  }
  return ok;
}

__device__ __forceinline__ float pow_at(const float* tab, uint64_t len, int64_t k, uint32_t& bad) {
  if (k < 0 || (uint64_t)k >= len) {
    bad |= FM_PREP_BAD_POW;
    return 0.0f;
  }
  const float x = tab[k];
  if (x != x) bad |= FM_PREP_BAD_POW;
  return x;
}

// Round trips: the row's ids (staged into LDS when they fit) and the row's
// previous state are loaded together first; the end marker, think pair and
// system prefix are then scanned in LDS.  The LF step from the previous range
// is issued speculatively together with the token compare that validates it,
// and the C lookup (count([last]) == 0) is made only for eos / pad rows and
// rows whose range came out empty -- a non-empty range implies count > 0.
template <bool STAGED>
__global__ void __launch_bounds__(64) k_prep(DevView v, fm_prep_config cfg, const int64_t* __restrict__ ids,
                                             uint64_t B, uint64_t Lt, uint64_t ld, const int64_t* __restrict__ fdf,
                                             uint64_t fdf_len, const float* __restrict__ pow_tab, uint64_t pow_len,
                                             const int64_t* __restrict__ prev_ids, uint64_t prev_ld,
                                             uint64_t prev_B, const int64_t* __restrict__ prev_state,
                                             fm_row_params* __restrict__ rows, uint64_t* __restrict__ mlo,
                                             uint64_t* __restrict__ mhi, int64_t* __restrict__ state,
                                             uint32_t* __restrict__ status, int64_t* __restrict__ ids_copy,
                                             uint64_t copy_ld, int32_t* __restrict__ facts,
                                             uint32_t* __restrict__ rowcase) {
  extern __shared__ int64_t srow[];   // STAGED: [npad] the row, then [4] its previous state
  const uint64_t row = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  const int64_t* g = ids + row * ld;
  const int64_t n = (int64_t)Lt;
  const int64_t npad = (n + kStageBatch - 1) / kStageBatch * kStageBatch;
  const bool have_prev = prev_ids && row < prev_B;
  int64_t ps[4] = {-1, -1, 0, 0};   // previous (start, len, lo, hi) of this row
  if (STAGED) {
    // every load issued before any is stored: clamped, unconditional
    int64_t y = -1;
    if (have_prev && lane < 4) y = prev_state[lane * prev_B + row];
    for (int64_t i0 = 0; i0 < n; i0 += kStageBatch) {
      int64_t x[kStageBatch / 64];
#pragma unroll
      for (int u = 0; u < kStageBatch / 64; ++u) x[u] = g[min(i0 + u * 64 + (int64_t)lane, n - 1)];
#pragma unroll
      for (int u = 0; u < kStageBatch / 64; ++u) srow[i0 + u * 64 + lane] = x[u];
    }
    if (lane < 4) srow[npad + lane] = y;
    __syncthreads();
    if (have_prev) {
#pragma unroll
      for (int k = 0; k < 4; ++k) ps[k] = srow[npad + k];
    }
  } else if (have_prev) {
#pragma unroll
    for (int k = 0; k < 4; ++k) ps[k] = prev_state[k * prev_B + row];
  }
  const int64_t* r = STAGED ? srow : g;
  // this call's row, kept for the next call's incremental ranges (prev_ids then)
  if (ids_copy)
    for (int64_t i = lane; i < n; i += 64) ids_copy[row * copy_ld + i] = r[i];
  uint32_t bad = 0;
  // remove_end_marker (causal_qwen.py:44-56): the tokens after the marker
  const bool hard = (cfg.flags & FM_PREP_HARD) != 0;
  // FM_PREP_SHARD (a doc-range shard of the corpus): the index-dependent decisions of the soft
  // variants -- count([last]) > 0, the pattern's range non-empty, its distinct set non-empty --
  // are recorded as this shard's facts (facts [3][B]) with the row's case and pattern length
  // (rowcase); fm_processor_shard_finish decides them from the facts summed over the shards
  const bool shard = facts != nullptr;
  uint32_t rcase = 0;          // 0: index-independent, 1: eos / pad last token, 2: pattern search
  int64_t ls_case = 0;
  int32_t f_cnt1 = 0, f_range = 0, f_dist = 0;
  int64_t searched_len = 0;    // force_decoding_from + sent of a searched row (the halo check)
  const int64_t M = hard ? 0 : cfg.marker_len;
  int64_t first = -1;
  uint32_t hits = hard ? 1u : 0u;
  for (int64_t i0 = 0; M > 0 && i0 + M <= n; i0 += 64) {
    const int64_t i = i0 + lane;
    bool m = i + M <= n;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t x = r[min(i + j, n - 1)];
      m &= (j >= M) | (x == cfg.marker[j]);
    }
    const uint64_t bal = __ballot(m);
    hits += (uint32_t)__popcll(bal);
    if (bal && first < 0) first = i0 + __ffsll((long long)bal) - 1;
  }
  if (hits != 1) bad |= FM_PREP_BAD_MARKER;
  int64_t start = hard ? min((int64_t)max(cfg.skip, 0), n) : (first < 0 ? 0 : first + M);
  if (lane == 0) {
    atomicMin(&status[1], (uint32_t)start);
    atomicMax(&status[2], (uint32_t)start);
  }
  int64_t L = n - start;
  fm_row_params p;
  p.base = cfg.base;
  p.v_dist = p.v_uni = p.v_eos = 0.0f;
  p.flags = 0;
  p.reserved = 0;
  p.special = 0;
  uint32_t kind = kUni;
  int64_t s0 = start, ls = L;
  uint64_t lo = 0, hi = 0;
  bool pattern = false;
  bool forced = false;
  if (cfg.flags & FM_PREP_SKIP_FIRST) {   // causal.py:80-85
    if (L == 0) forced = true;
    else {
      ++start;
      --L;
      s0 = start;
      ls = L;
    }
  }
  if (forced) {
    p.flags = FM_ROW_SPECIAL;
    p.special = cfg.forced_bos;
    p.v_dist = cfg.v_forced;
  } else {
    if (cfg.flags & FM_PREP_THINK) {
      // finished_thinking (causal_qwen.py:74-82) over the whole sent
      bool ft = false;
      for (int64_t i0 = start; i0 + 1 < n; i0 += 64) {
        const int64_t i = i0 + lane;
        const int64_t a = r[min(i, n - 1)], b = r[min(i + 1, n - 1)];
        const bool m = (i + 1 < n) & (a == cfg.think[0]) & (b == cfg.think[1]);
        if (__ballot(m)) {
          ft = true;
          break;
        }
      }
      if (!ft) {
        kind = kNone;
      } else {
        // remove_system_tokens (causal_qwen.py:58-72)
        const int64_t k = L < 4 ? L : 4;
        bool pre = true;   // n >= 2 here (the think pair was found)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t x = r[min(start + j, n - 1)];
          pre &= (j >= k) | (x == cfg.sys[j]);
        }
        if (pre && L < 4) ls = 0;
        else if (pre) {
          s0 += 4;
          ls -= 4;
        }
      }
    }
    if (kind != kNone && ls > 0) {
      // get_trailing_corpus_ngram: only count([last]) matters (causal_qwen.py:95-99)
      const int64_t last = r[s0 + ls - 1];
      const int64_t c = last + cfg.shift;
      bool counted = false;   // cnt1 known
      uint64_t cnt1 = 0;
      if (last == cfg.eos || last == cfg.pad) {
        // hard variants: no trailing n-gram rule, the eos / pad rule applies as is
        cnt1 = hard ? 1 : ((c >= 0 && (uint64_t)c <= v.max_sym) ? v.C[c + 1] - v.C[c] : 0);
        counted = true;
        if (shard && !hard) {
          rcase = 1;
          ls_case = ls;
          f_cnt1 = cnt1 > 0;
        }
      }
      if (counted && cnt1 == 0) {
        ls = 0;
      } else if (counted) {   // count 0 (causal_qwen.py:125-128, 161-174)
        kind = kSpecial;
        p.special = (cfg.stop_at_count > 0) ? cfg.eos : cfg.pad;
      } else {
        // the range of force_decoding_from + sent: one LF step from the previous
        // call's range of a row (same beam group) whose pattern is this one's
        // pattern without its last token, else a full search
        searched_len = (int64_t)fdf_len + ls;
        bool found = false;
        uint64_t pw = 0;   // count of the pattern without its last token (the hard variants' stop rule)
        if (prev_ids && ls >= 2) {
          const uint64_t beams = cfg.num_beams > 0 ? (uint64_t)cfg.num_beams : 1;
          const uint64_t g0 = row / beams * beams;
          // the row itself first: the LF step from its previous range is issued
          // with the first chunk of the token compare that validates it
          if (have_prev && ps[1] == ls - 1 && ps[0] >= 0) {
            const int64_t* pr = prev_ids + row * prev_ld + ps[0];
            const int64_t x = lane < ls - 1 ? pr[lane] : 0;
            uint64_t l2 = (uint64_t)ps[2], h2 = (uint64_t)ps[3];
            const uint32_t* cbm;
            int64_t one;
            lf_step_decode(v, c, l2, h2, cbm, one);
            bool eq = !__ballot(lane < ls - 1 && x != r[s0 + lane]);
            if (eq && ls - 1 > 64) eq = wave_equal(pr + 64, r + s0 + 64, ls - 1 - 64);
            if (eq) {
              lo = l2;
              hi = h2;
              pw = (uint64_t)(ps[3] - ps[2]);
              found = true;
            }
          }
          for (uint64_t k = 1; k < beams && !found; ++k) {
            const uint64_t b2 = g0 + k - 1 < row ? g0 + k - 1 : g0 + k;
            if (b2 >= prev_B || b2 >= g0 + beams) continue;
            const int64_t pstart = prev_state[b2], plen = prev_state[prev_B + b2];
            if (plen != ls - 1 || pstart < 0) continue;
            if (wave_equal(prev_ids + b2 * prev_ld + pstart, r + s0, ls - 1)) {
              lo = (uint64_t)prev_state[2 * prev_B + b2];
              hi = (uint64_t)prev_state[3 * prev_B + b2];
              pw = hi - lo;
              const uint32_t* cbm;
              int64_t one;
              lf_step_decode(v, c, lo, hi, cbm, one);
              found = true;
            }
          }
        }
        if (!found) {
          lo = 0;
          hi = v.n;
          for (int64_t j = 0; j < (int64_t)fdf_len + ls; ++j) {
            if (j == (int64_t)fdf_len + ls - 1) pw = hi - lo;
            // both candidates loaded from their own address spaces (a select of
            // the pointers would make one generic pointer and FLAT loads)
            const int64_t jf = j < (int64_t)fdf_len ? j : 0, jr = j < (int64_t)fdf_len ? 0 : j - (int64_t)fdf_len;
            const int64_t tf = fdf_len ? fdf[jf] : 0, tr = r[s0 + jr];
            const int64_t t = j < (int64_t)fdf_len ? tf : tr;
            const uint32_t* cbm;
            int64_t one;
            lf_step_decode(v, t + cfg.shift, lo, hi, cbm, one);
            if (lo == 0 && hi == 0) break;   // index.py:111-112
          }
        }
        // a non-empty range implies count([last]) > 0; an empty one asks C
        // (the hard variants have no trailing n-gram rule)
        if (hi <= lo && !hard) cnt1 = (c >= 0 && (uint64_t)c <= v.max_sym) ? v.C[c + 1] - v.C[c] : 0;
        if (shard && !hard) {   // this shard's facts; the decision below is provisional
          rcase = 2;
          ls_case = ls;
          f_range = hi > lo;
          f_cnt1 = hi > lo || cnt1 > 0;
          f_dist = !(hi == lo || (hi - lo == 1 && bwt_sym(v, lo) == 0));
        }
        if (hi <= lo && !hard && cnt1 == 0) {
          ls = 0;
          lo = hi = 0;
        } else {
          pattern = true;
          const uint64_t count = hard ? pw : hi - lo;
          if (cfg.stop_at_count > 0 && count <= (uint64_t)cfg.stop_at_count) {
            kind = kSpecial;
            p.special = cfg.eos;
          } else {
            kind = kBits;
          }
        }
      }
    }
    if (kind != kNone && ls == 0) kind = kUni;
    if (kind == kUni) {
      p.flags = FM_ROW_UNIGRAM;
      p.v_uni = cfg.v_uni_full;
    } else if (kind == kSpecial || kind == kBits) {
      // a shard's provisional decision must not flag a boost the summed facts may not need
      p.v_dist = rcase ? 0.0f : pow_at(pow_tab, pow_len, ls, bad);
      bool empty = false;
      if (hard) {   // vllm.py:118-131: the distinct set only, on -inf
        p.flags = kind == kBits ? FM_ROW_BITS : FM_ROW_SPECIAL;
      } else if (kind == kBits) {
        // distinct (sentinel dropped, index.py:170) is empty iff the range is
        // empty or its one row holds the sentinel
        empty = hi == lo || (hi - lo == 1 && bwt_sym(v, lo) == 0);
        p.flags = FM_ROW_BITS | FM_ROW_UNIGRAM;
      } else {
        p.flags = FM_ROW_SPECIAL | FM_ROW_UNIGRAM;
      }
      p.v_uni = (empty && !(cfg.flags & FM_PREP_UNI_HALF)) ? cfg.v_uni_full : cfg.v_uni_half;
    }
    // the eos boost (causal_qwen.py:206-212 / causal.py:173-178)
    if ((cfg.flags & FM_PREP_EOS) && kind != kNone &&
        ((cfg.flags & FM_PREP_EOS_ALL) || L >= cfg.min_new_tokens)) {
      p.flags |= FM_ROW_EOS;
      p.v_eos = pow_at(pow_tab, pow_len, L, bad);
    }
  }
  if (lane == 0) {
    rows[row] = p;
    // a shard's pattern rows keep their (possibly empty) local range: the bits of every shard
    // are ORed, and an empty range stays empty under the next call's LF step
    const bool searched = rcase == 2;
    const bool bits = searched || (kind == kBits && !forced);
    mlo[row] = bits ? lo : 0;
    mhi[row] = bits ? hi : 0;
    state[row] = (pattern || searched) ? s0 : -1;
    state[B + row] = searched ? ls_case : pattern ? ls : -1;
    state[2 * B + row] = (int64_t)lo;
    state[3 * B + row] = (int64_t)hi;
    if (bad) atomicOr(&status[0], bad);
    if (shard) {
      facts[row] = f_cnt1;
      facts[B + row] = f_range;
      facts[2 * B + row] = f_dist;
      rowcase[row] = rcase | ((uint32_t)ls_case << 2);
      // the longest searched pattern: the host checks it against the shards' halo
      if (searched_len) atomicMax(&status[3], (uint32_t)searched_len);
    }
  }
}

// Phase 2 of a doc-sharded processor call: the rows whose decision depends on
// the index (rowcase 1 / 2), decided from the shards' facts summed over the
// ranks (> 0: some shard has it) exactly as k_prep decides them on one index.
__global__ void __launch_bounds__(256) k_prep_finish(fm_prep_config cfg, uint64_t B, const int32_t* __restrict__ fsum,
                                                     const uint32_t* __restrict__ rowcase,
                                                     const float* __restrict__ pow_tab, uint64_t pow_len,
                                                     fm_row_params* __restrict__ rows, uint32_t* __restrict__ status) {
  const uint64_t row = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= B) return;
  const uint32_t rc = rowcase[row];
  const uint32_t c = rc & 3u;
  if (!c) return;
  const int64_t ls = (int64_t)(rc >> 2);
  const bool g_cnt1 = fsum[row] > 0, g_range = fsum[B + row] > 0, g_dist = fsum[2 * B + row] > 0;
  fm_row_params p = rows[row];
  const uint32_t eosf = p.flags & FM_ROW_EOS;
  uint32_t bad = 0;
  p.special = 0;
  p.v_dist = 0.0f;
  if (c == 1 ? !g_cnt1 : (!g_range && !g_cnt1)) {   // count([last]) == 0: all unigrams
    p.flags = FM_ROW_UNIGRAM | eosf;
    p.v_uni = cfg.v_uni_full;
  } else if (c == 1) {                               // eos / pad rule (stop_at_count is 0 here)
    p.flags = FM_ROW_SPECIAL | FM_ROW_UNIGRAM | eosf;
    p.special = cfg.pad;
    p.v_dist = pow_at(pow_tab, pow_len, ls, bad);
    p.v_uni = cfg.v_uni_half;
  } else {
    p.flags = FM_ROW_BITS | FM_ROW_UNIGRAM | eosf;
    p.v_dist = pow_at(pow_tab, pow_len, ls, bad);
    p.v_uni = (!g_dist && !(cfg.flags & FM_PREP_UNI_HALF)) ? cfg.v_uni_full : cfg.v_uni_half;
  }
  rows[row] = p;
  if (bad) atomicOr(&status[0], bad);
}

}  // namespace

int launch_prep_finish(const fm_prep_config& cfg, uint64_t B, const int32_t* fsum, const uint32_t* rowcase,
                       const float* pow_tab, uint64_t pow_len, fm_row_params* rows, uint32_t* status, hipStream_t s) {
  if (!B) return 0;
  if (!fsum || !rowcase || !pow_tab || !rows || !status) {
    set_error("processor shard finish: bad arguments");
    return -1;
  }
  k_prep_finish<<<(unsigned)((B + 255) / 256), 256, 0, s>>>(cfg, B, fsum, rowcase, pow_tab, pow_len, rows, status);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_processor_step(const DevView& v, const fm_prep_config& cfg, const int64_t* ids, uint64_t B, uint64_t L,
                          uint64_t ld, const int64_t* fdf, uint64_t fdf_len, const float* pow_tab, uint64_t pow_len,
                          const int64_t* prev_ids, uint64_t prev_ld, uint64_t prev_B, const int64_t* prev_state,
                          fm_row_params* rows, uint64_t* mlo, uint64_t* mhi, int64_t* state, uint32_t* status,
                          int64_t* ids_copy, uint64_t copy_ld, bool init_status, hipStream_t s, int32_t* facts,
                          uint32_t* rowcase) {
  if (!(cfg.flags & FM_PREP_HARD) && (cfg.marker_len < 1 || cfg.marker_len > 8)) {
    set_error("processor step: marker length %d not in 1..8", cfg.marker_len);
    return -1;
  }
  if (facts && (!rowcase || cfg.stop_at_count > 0)) {
    // stop_at_count compares a count, and a shard's counts include its halo's duplicates
    set_error("processor step over a shard: stop_at_count must be 0 (counts are not exact under sharding)");
    return -1;
  }
  if (ld < L || (fdf_len && !fdf) || !pow_tab || (prev_ids && !prev_state)) {
    set_error("processor step: bad arguments");
    return -1;
  }
  if (ids_copy && copy_ld < L) {
    set_error("processor step: ids copy row of %llu < %llu", (unsigned long long)copy_ld, (unsigned long long)L);
    return -1;
  }
  // k_prep reads prev_ids (and ids) in the same kernel that writes ids_copy, all
  // __restrict__: a copy buffer overlapping either would race with those reads
  if (ids_copy && B) {
    auto overlaps = [&](const int64_t* p, uint64_t rows, uint64_t pld, uint64_t cols) {
      if (!p || !rows) return false;
      const char* a0 = reinterpret_cast<const char*>(ids_copy);
      const char* a1 = reinterpret_cast<const char*>(ids_copy + (B - 1) * copy_ld + L);
      const char* b0 = reinterpret_cast<const char*>(p);
      const char* b1 = reinterpret_cast<const char*>(p + (rows - 1) * pld + cols);
      return a0 < b1 && b0 < a1;
    };
    if (overlaps(prev_ids, prev_B, prev_ld, prev_ld) || overlaps(ids, B, ld, L)) {
      set_error("processor step: ids_copy must not overlap prev_ids or ids");
      return -1;
    }
  }
  if (init_status) {   // a caller that never reads the status (fm_processor_call without a host copy) skips this
    FM_HIP(hipMemsetAsync(status, 0, 16, s));
    FM_HIP(hipMemsetAsync(status + 1, 0xFF, 4, s));
  }
  if (B == 0) return 0;
  if (L <= (uint64_t)kMaxStaged) {
    const size_t lds = ((L + kStageBatch - 1) / kStageBatch * kStageBatch + 4) * sizeof(int64_t);
    k_prep<true><<<(unsigned)B, 64, lds, s>>>(v, cfg, ids, B, L, ld, fdf, fdf_len, pow_tab, pow_len, prev_ids,
                                              prev_ld, prev_B, prev_state, rows, mlo, mhi, state, status, ids_copy,
                                              copy_ld, facts, rowcase);
  } else {
    k_prep<false><<<(unsigned)B, 64, 0, s>>>(v, cfg, ids, B, L, ld, fdf, fdf_len, pow_tab, pow_len, prev_ids,
                                             prev_ld, prev_B, prev_state, rows, mlo, mhi, state, status, ids_copy,
                                             copy_ld, facts, rowcase);
  }
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
