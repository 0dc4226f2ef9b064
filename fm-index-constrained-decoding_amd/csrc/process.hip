// process.hip -- the per-row bookkeeping of the soft logits processors on the
// device (fm_processor_step), so a processor call is three launches and no
// per-row host work:
//   k_prep      one wave per row: remove_end_marker, finished_thinking,
//               remove_system_tokens, the trailing n-gram rule, the eos / pad
//               / stop_at_count rules and the pattern's range
//               (document_constrained_generation_causal_qwen.py:44-99,
//               :101-214; document_constrained_generation_causal.py:62-180),
//               writing the epilogue's fm_row_params
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

constexpr int kThreads = 256;   // 4 rows per workgroup, one wave each
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

__global__ void __launch_bounds__(kThreads) k_prep(DevView v, fm_prep_config cfg, const int64_t* __restrict__ ids,
                                                   uint64_t B, uint64_t Lt, uint64_t ld, const int64_t* __restrict__ fdf,
                                                   uint64_t fdf_len, const float* __restrict__ pow_tab, uint64_t pow_len,
                                                   const int64_t* __restrict__ prev_ids, uint64_t prev_ld,
                                                   uint64_t prev_B, const int64_t* __restrict__ prev_state,
                                                   fm_row_params* __restrict__ rows, uint64_t* __restrict__ mlo,
                                                   uint64_t* __restrict__ mhi, int64_t* __restrict__ state,
                                                   uint32_t* __restrict__ status) {
  const uint64_t row = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (row >= B) return;
  const int64_t* r = ids + row * ld;
  const int64_t n = (int64_t)Lt;
  uint32_t bad = 0;
  // remove_end_marker (causal_qwen.py:44-56): the tokens after the marker
  const int64_t M = cfg.marker_len;
  int64_t first = -1;
  uint32_t hits = 0;
  for (int64_t i0 = 0; i0 + M <= n; i0 += 64) {
    // all 8 candidate tokens loaded at once (clamped, unconditional) and
    // compared after: a short-circuit compare issued one load per round trip
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
  int64_t start = first < 0 ? 0 : first + M;
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
      const uint64_t cnt1 = (c >= 0 && (uint64_t)c <= v.max_sym) ? v.C[c + 1] - v.C[c] : 0;
      if (cnt1 == 0) {
        ls = 0;
      } else if (last == cfg.eos || last == cfg.pad) {   // count 0 (causal_qwen.py:125-128, 161-174)
        kind = kSpecial;
        p.special = (cfg.stop_at_count > 0) ? cfg.eos : cfg.pad;
      } else {
        // the range of force_decoding_from + sent: one LF step from the previous
        // call's range of a row (same beam group) whose pattern is this one's
        // pattern without its last token, else a full search
        bool found = false;
        if (prev_ids && ls >= 2) {
          const uint64_t beams = cfg.num_beams > 0 ? (uint64_t)cfg.num_beams : 1;
          const uint64_t g0 = row / beams * beams;
          for (uint64_t k = 0; k < beams && !found; ++k) {
            const uint64_t b2 = k == 0 ? row : (g0 + k - 1 < row ? g0 + k - 1 : g0 + k);
            if (b2 >= prev_B || b2 >= g0 + beams) continue;
            const int64_t pstart = prev_state[b2], plen = prev_state[prev_B + b2];
            if (plen != ls - 1 || pstart < 0) continue;
            if (wave_equal(prev_ids + b2 * prev_ld + pstart, r + s0, ls - 1)) {
              lo = (uint64_t)prev_state[2 * prev_B + b2];
              hi = (uint64_t)prev_state[3 * prev_B + b2];
              const uint32_t* cbm;
              int64_t one;
              lf_step_decode(v, last + cfg.shift, lo, hi, cbm, one);
              found = true;
            }
          }
        }
        if (!found) {
          lo = 0;
          hi = v.n;
          for (int64_t j = 0; j < (int64_t)fdf_len + ls; ++j) {
            const int64_t t = j < (int64_t)fdf_len ? fdf[j] : r[s0 + j - (int64_t)fdf_len];
            const uint32_t* cbm;
            int64_t one;
            lf_step_decode(v, t + cfg.shift, lo, hi, cbm, one);
            if (lo == 0 && hi == 0) break;   // index.py:111-112
          }
        }
        pattern = true;
        const uint64_t count = hi - lo;
        if (cfg.stop_at_count > 0 && count <= (uint64_t)cfg.stop_at_count) {
          kind = kSpecial;
          p.special = cfg.eos;
        } else {
          kind = kBits;
        }
      }
    }
    if (kind != kNone && ls == 0) kind = kUni;
    if (kind == kUni) {
      p.flags = FM_ROW_UNIGRAM;
      p.v_uni = cfg.v_uni_full;
    } else if (kind == kSpecial || kind == kBits) {
      p.v_dist = pow_at(pow_tab, pow_len, ls, bad);
      bool empty = false;
      if (kind == kBits) {
        // distinct (sentinel dropped, index.py:170) is empty iff the range is
        // empty or its one row holds the sentinel
        empty = hi == lo || (hi - lo == 1 && v.bwt[lo] == 0);
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
    const bool bits = kind == kBits && !forced;
    mlo[row] = bits ? lo : 0;
    mhi[row] = bits ? hi : 0;
    state[row] = pattern ? s0 : -1;
    state[B + row] = pattern ? ls : -1;
    state[2 * B + row] = (int64_t)lo;
    state[3 * B + row] = (int64_t)hi;
    if (bad) atomicOr(&status[0], bad);
  }
}

}  // namespace

int launch_processor_step(const DevView& v, const fm_prep_config& cfg, const int64_t* ids, uint64_t B, uint64_t L,
                          uint64_t ld, const int64_t* fdf, uint64_t fdf_len, const float* pow_tab, uint64_t pow_len,
                          const int64_t* prev_ids, uint64_t prev_ld, uint64_t prev_B, const int64_t* prev_state,
                          fm_row_params* rows, uint64_t* mlo, uint64_t* mhi, int64_t* state, uint32_t* status,
                          hipStream_t s) {
  if (cfg.marker_len < 1 || cfg.marker_len > 8) {
    set_error("processor step: marker length %d not in 1..8", cfg.marker_len);
    return -1;
  }
  if (ld < L || (fdf_len && !fdf) || !pow_tab || (prev_ids && !prev_state)) {
    set_error("processor step: bad arguments");
    return -1;
  }
  FM_HIP(hipMemsetAsync(status, 0, 16, s));
  FM_HIP(hipMemsetAsync(status + 1, 0xFF, 4, s));
  if (B == 0) return 0;
  k_prep<<<(unsigned)((B * 64 + kThreads - 1) / kThreads), kThreads, 0, s>>>(
      v, cfg, ids, B, L, ld, fdf, fdf_len, pow_tab, pow_len, prev_ids, prev_ld, prev_B, prev_state, rows, mlo, mhi,
      state, status);
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
