// query.hip -- batched hot-path kernels for gfx950.
//
//  k_lf          one backward-search (LF) step per row: the loop body of
//                index.py:109-112 / fm_index.cpp:67-97, through the shared
//                lf_step_decode: C lookup, E scan (<= 512 rows), transition
//                probe, or the 2-level wavelet-matrix descent.
//  k_search      get_range over CSR patterns with the reference's early exit.
//  (the allowed-token mask / fused decode step lives in decode.hip)
//  k_distinct    interval_symbols with counts ([sdsl] wt_int::interval_symbols)
//                as a level-synchronous BFS of the wavelet matrix, one
//                workgroup per row, ascending symbol order.
//  k_step_raw / k_raw_multi: the scalar SWIG entry points with sdsl's unsigned
//                arithmetic (fm_index.cpp:55-97).
#include "fmidx_internal.h"

#include <algorithm>
#include <cstdlib>

namespace fmidx {

namespace {

constexpr int kLfThreads = 256;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// ------------------------------------------------------------------ LF
// One wave per row (kLfThreads / 64 rows per block), 2-level wavelet matrix.
__global__ void __launch_bounds__(kLfThreads) k_lf(DevView v, const int64_t* __restrict__ tok,
                                                  int64_t shift, int64_t reset_below,
                                                  const uint64_t* lo_in, const uint64_t* hi_in,
                                                  uint64_t* lo_out, uint64_t* hi_out, uint64_t m) {
  FM_PRELOAD_VIEW(v);
  const uint64_t i = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (i >= m) return;
  const int64_t t = (int64_t)row_load_u64(tok, m, i);
  uint64_t l = row_load_u64(lo_in, m, i), h = row_load_u64(hi_in, m, i);
  // Every row runs lf_step_decode, a reset row with symbol -1 so it leaves at
  // the dead check (its stale range costs no probe or descent), and its result
  // is replaced after it: with a branch on the token, the compiler sank the
  // (lo, hi) loads into the non-reset side, behind the token's round trip.
  const uint32_t* cbm;
  int64_t one;
  lf_step_decode(v, t < reset_below ? -1 : t + shift, l, h, cbm, one);
  if (t < reset_below) {
    l = 0;
    h = v.n;
  }
  if (lane == 0) {
    lo_out[i] = l;
    hi_out[i] = h;
  }
}

__global__ void __launch_bounds__(kLfThreads) k_search(DevView v, const int64_t* __restrict__ tok,
                                                      const int64_t* __restrict__ off, uint64_t m,
                                                      int64_t shift, const uint64_t* lo_in,
                                                      const uint64_t* hi_in, uint64_t* lo_out,
                                                      uint64_t* hi_out) {
  const uint64_t i = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (i >= m) return;
  uint64_t l = lo_in ? lo_in[i] : 0;
  uint64_t h = hi_in ? hi_in[i] : v.n;
  const int64_t a = off[i], b = off[i + 1];
  for (int64_t j = a; j < b; ++j) {
    const uint32_t* cbm;
    int64_t one;
    lf_step_decode(v, tok[j] + shift, l, h, cbm, one);
    if (l == 0 && h == 0) break;       // index.py:111-112
  }
  if (lane == 0) {
    lo_out[i] = l;
    hi_out[i] = h;
  }
}

// ------------------------------------------------------------ grouped LF
// Throughput form of k_lf / k_search for launches with more rows than the chip
// has wave slots (256 CUs x 32 waves): a wave is latency-bound on its dependent
// round trips, so at one row per wave the rows in flight per CU cap the rate
// (Little's law: 32 rows x ~3 cold hops).  Here a group of G lanes owns a row,
// 64 / G rows per wave: a full range takes its C lookup, a range of <= 128
// rows its E scan in a scan packed over the whole wave (group_step), and the
// rest -- wider ranges (transition probe / wavelet descent / wave-wide E
// scan) -- are taken one at a time by the whole wave through lf_step_decode.

// Rows of at most this many entries take their LF step from E inside the
// wave-packed scan of group_step (one load per entry actually needed).
constexpr uint64_t kPackMax = 128;

// Transition probe of a wave's cached rows eight at a time (8 lanes per row): lane sl of a row's
// segment loads slot sl of its bucket A and slot sl of its bucket B (16-B slots: the two 128-B
// lines) and (CE) slot sl of the range's own range-cache run -- the parent's cache id, which the
// slots' keys hold.  Used by get_range (group_step<P8>) and the LF sweep (sweep_head).
constexpr uint32_t kProbeLanes = 8;
constexpr uint32_t kProbeRows = 64 / kProbeLanes;

// Transition probe of up to eight rows (8 lanes each; row k of the batch =
// the wave's lane src[k], src < 0: none) -- loads only; probe_finish consumes.
struct ProbeLoads {
  uint4 ca, cb;           // slot sl of bucket A, slot sl of bucket B
  uint4 ce;               // the range's own range-cache slot sl
};
template <bool CE = true>
__device__ __forceinline__ ProbeLoads probe_issue(const DevView& v, uint64_t l, uint64_t h, uint64_t c) {
  const uint32_t sl = (threadIdx.x & 63u) % kProbeLanes;
  const TransHome th = trans_home(l, h, c, v.trans_cap);
  const uint4* tt = reinterpret_cast<const uint4*>(v.trans_tab);
  ProbeLoads p;
  p.ca = tt[th.a + sl];
  p.cb = tt[th.b + sl];
  // the range's own range-cache run (8 slots, one per lane)
  if (CE) {
    const uint64_t cs = (cache_hash(l, h) + sl) & v.cache_mask;
    p.ce = v.cache_mask ? reinterpret_cast<const uint4*>(v.cache_tab)[cs] : make_uint4(~0u, ~0u, 0, 0);
  } else {
    p.ce = make_uint4(~0u, ~0u, 0, 0);
  }
  return p;
}

// -> per lane: hit (and the child range on the row's first lane), or the
// range's cache id + 1 (0: not found) for the tail entry of a miss.  Without
// the range's cache id among the 8 run slots read no key can match: a miss.
template <bool CE = true>
__device__ __forceinline__ void probe_finish(const DevView& v, uint64_t l, uint64_t h, uint64_t c, bool act,
                                            const ProbeLoads& p, uint4* /*s_run*/, bool& hit_row, uint64_t& clo,
                                            uint64_t& chi, uint64_t& pid1) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t seg = lane / kProbeLanes;
  const uint64_t klo = (uint64_t)p.ce.x | ((uint64_t)p.ce.y << 32);
  const uint64_t khi = (uint64_t)p.ce.z | ((uint64_t)p.ce.w << 32);
  const bool pc = CE && v.cache_mask && klo == l && (khi & kMask34) == h;
  const uint64_t segm = 0xFFull << (kProbeLanes * seg);
  const uint64_t pb = __ballot(act && pc) & segm;
  const int pl = pb ? __ffsll((long long)pb) - 1 : (int)lane;
  const uint64_t pid = pb ? (__shfl(khi, pl, 64) >> kCacheIdShift) : kTPidNone;
  const uint64_t key = trans_key(pid, c);
  const uint64_t a0 = (uint64_t)p.ca.x | ((uint64_t)p.ca.y << 32), a1 = (uint64_t)p.ca.z | ((uint64_t)p.ca.w << 32);
  const uint64_t b0 = (uint64_t)p.cb.x | ((uint64_t)p.cb.y << 32), b1 = (uint64_t)p.cb.z | ((uint64_t)p.cb.w << 32);
  // (a parent id of 2^20 - 1 or more is never a key: trans_key would spill into the symbol bits)
  const bool keyed = pid < kTPidNone && c < kTSymLimit;
  const bool ma = keyed && trans_match(a0, key), mb = keyed && trans_match(b0, key);
  const uint64_t w0 = ma ? a0 : b0, w1 = ma ? a1 : b1;
  const uint64_t hb = __ballot(act && (ma || mb)) & segm;
  const int hl = hb ? __ffsll((long long)hb) - 1 : (int)lane;
  const uint64_t hw0 = __shfl(w0, hl, 64), hw1 = __shfl(w1, hl, 64);
  // a miss beside a free slot of either bucket: c is absent from the range (kProbeComplete) --
  // settled here as the empty range, not handed to the tail
  const uint64_t eb = __ballot(act && keyed && (a0 == kTransEmpty || b0 == kTransEmpty)) & segm;
  const bool absent = !hb && eb && (v.probe_first & kProbeComplete);
  hit_row = hb != 0 || absent;
  clo = absent ? 0 : trans_clo(hw0, hw1);
  chi = absent ? 0 : clo + trans_cw(hw1);
  pid1 = pb ? pid + 1 : 0;
}


// One LF step for every group of the wave.  `live` = the group takes a step
// (false: the row is left as it is).  The loads are shaped for request
// efficiency (the random-line rate of HBM counts requests -- one per (load
// instruction, line) -- not bytes: csrc/probe.hip measures 3.1 TB/s of 64-B
// lines when 4 lanes share a line against 1.3 TB/s when every lane reads its
// own):
//  * the C lookup is made only by full-range rows (the others all read C[0],
//    one shared line);
//  * rows of <= kPackMax entries are scanned from E by the whole wave at once:
//    the rows' entry counts are prefix-summed across the wave, and each pass
//    gives every lane the next entry of the packed list (its row found by a
//    binary search over the rows' offsets), so a row costs a load per entry it
//    has -- consecutive entries of a row land in one request -- instead of 8 G
//    clamped loads (a 1-entry row used to issue 8 requests for its one line);
//    matches go to per-row LDS slots (min / max LF: LF is increasing over a
//    symbol's rows, so they are the LF of the first and last match).
// Every lane executes the same loads (unconditional, clamped or dummy index:
// a guarded load is sunk into a branch with a vmcnt(0) behind it).
constexpr uint64_t kLfWideTag = 1ull << 63;
#ifndef FMIDX_E_PASS
#define FMIDX_E_PASS 1
#endif
constexpr int kEPass = FMIDX_E_PASS;   // wave-packed E scan: 64-entry passes per round trip

// Whether a row's LF step is "wide" in group_step's sense: live, not dead, not
// the full range, and not a <= kPackMax-row E scan.  The split launch
// (k_lf_group in D mode, then k_lf_wide) must agree on it exactly.
__device__ __forceinline__ bool lf_wide(const DevView& v, bool live, int64_t sym, uint64_t l, uint64_t h) {
  if (h > v.n) h = v.n;
  const bool dead = !live || l >= h || sym < 0 || (uint64_t)sym > v.max_sym;
  const bool full = !dead && l == 0 && h == v.n;
  const bool narrow = !dead && !full && v.E && h - l <= kPackMax;
  return !dead && !full && !narrow;
}

// D (defer): the wide rows are not stepped at all (no probe, no descent, none of
// their code in the kernel, so it keeps few registers and many waves); their
// lo / hi come out unspecified and k_lf_wide steps them.
// P8 (get_range, G = 1): cached wide rows probe the transition table eight at
// a time (probe_issue / probe_finish) before the one-at-a-time loop.
template <int G, bool GP, bool Q, bool D = false, bool P8 = false>
__device__ __forceinline__ void group_step(const DevView& v, bool live, int64_t sym, uint64_t l, uint64_t h,
                                           uint64_t& lo, uint64_t& hi) {
  constexpr int R = 64 / G;                 // rows per wave
  __shared__ uint64_t s_lf[kLfThreads / 64][2][R];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t j = lane & (G - 1);
  const uint32_t slot = lane / G;
  const uint64_t h0 = h;
  if (h > v.n) h = v.n;
  const bool dead = !live || l >= h || sym < 0 || (uint64_t)sym > v.max_sym;
  const bool full = !dead && l == 0 && h == v.n;
  const bool narrow = !dead && !full && v.E && h - l <= kPackMax;
  bool wide = live && !dead && !full && !narrow;
  const uint64_t c = dead ? 0 : (uint64_t)sym;
  // C lookup (full-range rows only) and (GP) the group's transition probe, issued together
  const uint64_t cf = full ? c : 0;
  const uint64_t ca = v.C[cf], cb = v.C[cf + 1];
  uint64_t pw[GP ? 2 * (16 / G) : 1];
  uint64_t pe[GP ? 2 * (16 / G) : 1];
  const bool probe = GP && wide && v.trans_cap && v.cache_mask && h - l >= v.cache_min;
  if (GP) {
    // the 16-slot probe of lf_step_decode, 16 / G slots (2 words each) per lane, and as many slots
    // of the range's own range-cache run (the parent's cache id, which the keys hold);
    // unconditional loads (slot 0 for rows that do not probe; C[0..1] when the index has no
    // transition table or cache)
    const uint64_t* tt = probe ? v.trans_tab : v.C;
    const uint64_t* ct = probe ? v.cache_tab : v.C;
    const TransHome th = probe ? trans_home(l, h, c, v.trans_cap) : TransHome{0, 0};
    const uint64_t ch = probe ? cache_hash(l, h) : 0;
#pragma unroll
    for (int k = 0; k < 16 / G; ++k) {
      const uint64_t slot_k = probe ? trans_slot(th, j * (16 / G) + k) : 0;
      const uint64_t cs_k = probe ? ((ch + j * (16 / G) + k) & v.cache_mask) : 0;
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        pw[2 * k + w] = tt[2 * slot_k + w];
        pe[2 * k + w] = ct[2 * cs_k + w];
      }
    }
  }
  // ---- the wave-packed E scan of the narrow rows
  const uint32_t cnt = (narrow && j == 0) ? (uint32_t)(h - l) : 0u;
  uint32_t inc = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += y;
  }
  const uint32_t excl = inc - cnt;
  const uint32_t total = __shfl(inc, 63, 64);
  if (j == 0) {
    s_lf[wv][0][slot] = ~0ull;
    s_lf[wv][1][slot] = 0;
  }
  __builtin_amdgcn_wave_barrier();
  // kEPass passes of 64 entries per iteration, every pass's E load issued
  // before any is consumed.  Measured at C3 (2^19 cold pairs / 2^18 patterns):
  // 1 pass 76.1 / 420 us, 4 passes 80.2 / 504, 8 passes 81.6 / 520 -- a wave's
  // narrow rows rarely need a second pass, and the extra unconditional loads
  // and registers cost more than the round trips they would save.
  for (uint32_t t0 = 0; t0 < total; t0 += 64 * kEPass) {   // wave-uniform
    uint64_t xs[kEPass], rcs[kEPass];
    uint32_t rs[kEPass];
#pragma unroll
    for (int k = 0; k < kEPass; ++k) {
      const uint32_t e = t0 + 64u * k + lane;
      const bool valid = e < total;
      uint32_t r = 0;                                    // the last row whose offset is <= e
#pragma unroll
      for (int step = R / 2; step > 0; step >>= 1) {
        const uint32_t x = __shfl(excl, (int)((r + step) * G), 64);
        if (x <= e) r += step;
      }
      const uint64_t base = __shfl(l, (int)(r * G), 64);
      rcs[k] = __shfl(c, (int)(r * G), 64);
      const uint32_t off = e - __shfl(excl, (int)(r * G), 64);
      xs[k] = v.E[valid ? base + off : 0];
      rs[k] = valid ? r : ~0u;
    }
#pragma unroll
    for (int k = 0; k < kEPass; ++k) {
      if (rs[k] != ~0u && (xs[k] >> kESymShift) == rcs[k]) {
        atomicMin(&s_lf[wv][0][rs[k]], (unsigned long long)(xs[k] & kELfMask));
        atomicMax(&s_lf[wv][1][rs[k]], (unsigned long long)(xs[k] & kELfMask));
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  const uint64_t fmin = s_lf[wv][0][slot], fmax = s_lf[wv][1][slot];
  const bool found = fmin != ~0ull;
  if (!live) {
    lo = l;
    hi = h0;
  } else if (dead) {
    lo = 0;
    hi = 0;
  } else if (full) {
    lo = ca < cb ? ca : 0;
    hi = ca < cb ? cb : 0;
  } else if (narrow) {
    lo = found ? fmin : 0;
    hi = found ? fmax + 1 : 0;
  }
  if (D) return;
  if (P8) {
    // cached wide rows eight per round trip; a hit settles the row, a miss (a
    // symbol the range lacks, or a key the table left out) stays wide
    const uint32_t seg = lane / kProbeLanes;
    uint64_t pm = __ballot(wide && j == 0 && v.trans_cap && h - l >= v.cache_min);
    while (pm) {   // wave-uniform
      int src = -1;
      for (uint32_t k = 0; k < kProbeRows && pm; ++k) {
        const int s_ = __ffsll((long long)pm) - 1;
        pm &= pm - 1;
        if (seg == k) src = s_;
      }
      const bool act = src >= 0;
      const int ps = act ? src : 0;
      const uint64_t pl = __shfl(l, ps, 64), ph = __shfl(h, ps, 64), pc = __shfl(c, ps, 64);
      const ProbeLoads pld = probe_issue<true>(v, pl, ph, pc);
      bool hit;
      uint64_t clo, chi, p1;
      probe_finish<true>(v, pl, ph, pc, act, pld, nullptr, hit, clo, chi, p1);
#pragma unroll
      for (uint32_t k = 0; k < kProbeRows; ++k) {
        const int sk = __shfl(src, (int)(k * kProbeLanes), 64);
        const uint64_t xl = __shfl(clo, (int)(k * kProbeLanes), 64), xh = __shfl(chi, (int)(k * kProbeLanes), 64);
        const int xhit = __shfl((int)hit, (int)(k * kProbeLanes), 64);
        if (sk >= 0 && xhit && (lane / G) == ((uint32_t)sk / G)) {
          lo = xl;
          hi = xh;
          wide = false;
        }
      }
    }
  }
  if (GP) {   // a probe hit (at most one slot of the group holds the key) ends a wide row's step
    // the parent's cache id from the group's run slots (id + 1; 0: not among them -- no hit)
    uint64_t pid1 = 0;
#pragma unroll
    for (int k = 0; k < 16 / G; ++k)
      pid1 |= (probe && pe[2 * k] == l && (pe[2 * k + 1] & kMask34) == h) ? (pe[2 * k + 1] >> kCacheIdShift) + 1 : 0;
#pragma unroll
    for (int d = 1; d < G; d <<= 1) pid1 |= __shfl_xor(pid1, d, 64);
    const uint64_t key = trans_key(pid1 ? pid1 - 1 : kTPidNone, c);
    uint64_t hit = 0, clo = 0, cw = 0;
#pragma unroll
    for (int k = 0; k < 16 / G; ++k) {
      const bool m = probe && pid1 && pid1 - 1 < kTPidNone && c < kTSymLimit && trans_match(pw[2 * k], key);
      hit |= m ? 1u : 0u;
      clo |= m ? trans_clo(pw[2 * k], pw[2 * k + 1]) : 0;
      cw |= m ? trans_cw(pw[2 * k + 1]) : 0;
    }
#pragma unroll
    for (int d = 1; d < G; d <<= 1) {
      hit |= __shfl_xor(hit, d, 64);
      clo |= __shfl_xor(clo, d, 64);
      cw |= __shfl_xor(cw, d, 64);
    }
    if (hit) {
      lo = clo;
      hi = clo + cw;
      wide = false;
    }
  }
  uint64_t wb;
  if (Q) {
    // Wide rows four at a time, 16 lanes each: a cached parent's transition
    // probe (its 16 slots, one per lane) or the E scan of a range <= 128 rows
    // (8 entries per lane), one round trip per four rows.  Rows neither settles
    // (a probe miss, an uncached range > 128 rows) go to the serial loop below.
    const uint32_t seg = lane >> 4, sl = lane & 15u;
    const bool elig = wide && ((v.E && h - l <= 128) || (v.trans_cap && h - l >= v.cache_min));
    uint64_t qb = __ballot(elig && j == 0);
    uint64_t keep = __ballot(wide && !elig && j == 0);
    const uint64_t* tt = v.trans_cap ? v.trans_tab : v.C;   // C[0..1]: a valid dummy address
    const uint64_t* ct = v.cache_mask ? v.cache_tab : v.C;
    while (qb) {
      int sv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sv[k] = qb ? __ffsll((long long)qb) - 1 : -1;
        if (qb) qb &= qb - 1;
      }
      const int my = seg == 0 ? sv[0] : (seg == 1 ? sv[1] : (seg == 2 ? sv[2] : sv[3]));
      const bool act = my >= 0;
      const int srcl = act ? my : 0;
      const uint64_t ql = __shfl(l, srcl, 64), qh = __shfl(h, srcl, 64);
      const int64_t qs = __shfl(sym, srcl, 64);
      const uint64_t qc = act ? (uint64_t)qs : 0;
      const bool qscan = act && v.E && qh - ql <= 128;
      const bool qprobe = act && !qscan && v.trans_cap && qh - ql >= v.cache_min;
      const uint64_t slot = qprobe ? trans_slot(trans_home(ql, qh, qc, v.trans_cap), sl) : 0;
      const uint64_t p0 = tt[2 * slot], p1 = tt[2 * slot + 1];
      // slot sl of the range's own range-cache run: the parent's cache id
      const uint64_t cslot = (qprobe && v.cache_mask) ? ((cache_hash(ql, qh) + sl) & v.cache_mask) : 0;
      const uint64_t e0 = ct[2 * cslot], e1 = ct[2 * cslot + 1];
      uint64_t qe[8];
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) {
        const uint64_t idx = ql + sl + 16ull * k;
        const uint64_t x = v.E ? v.E[qscan ? (idx < qh ? idx : qh - 1) : 0] : 0;
        qe[k] = (qscan && idx < qh) ? x : ~0ull;
      }
      uint64_t fmn = ~0ull, fmx = 0, lmn = 0, lmx = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) {
        if (qe[k] != ~0ull && (qe[k] >> kESymShift) == qc) {
          const uint64_t r = sl + 16ull * k + 1;
          if (r < fmn) {
            fmn = r;
            lmn = qe[k] & kELfMask;
          }
          fmx = r;
          lmx = qe[k] & kELfMask;
        }
      }
#pragma unroll
      for (int d = 1; d < 16; d <<= 1) {
        const uint64_t om = __shfl_xor(fmn, d, 64), ol = __shfl_xor(lmn, d, 64);
        const uint64_t xm = __shfl_xor(fmx, d, 64), xl = __shfl_xor(lmx, d, 64);
        if (om < fmn) {
          fmn = om;
          lmn = ol;
        }
        if (xm > fmx) {
          fmx = xm;
          lmx = xl;
        }
      }
      const uint64_t segm = 0xFFFFull << (16 * seg);
      const uint64_t pb = __ballot(qprobe && v.cache_mask && e0 == ql && (e1 & kMask34) == qh) & segm;
      const uint64_t qpid = pb ? (__shfl(e1, __ffsll((long long)pb) - 1, 64) >> kCacheIdShift) : kTPidNone;
      const uint64_t hb = __ballot(qprobe && pb && qpid < kTPidNone && qc < kTSymLimit &&
                                   trans_match(p0, trans_key(qpid, qc))) & segm;
      const int hl = hb ? __ffsll((long long)hb) - 1 : 0;
      const uint64_t w0 = __shfl(p0, hl, 64), w1 = __shfl(p1, hl, 64);
      uint64_t rlo = 0, rhi = 0;
      int done = 0;
      if (qscan) {
        rlo = fmx ? lmn : 0;
        rhi = fmx ? lmx + 1 : 0;
        done = 1;
      } else if (qprobe && hb) {
        rlo = trans_clo(w0, w1);
        rhi = rlo + trans_cw(w1);
        done = 1;
      }
      // hand each row's result to its group (the loop and sv[] are wave-uniform)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int sk = sv[k];
        if (sk < 0) break;
        const uint64_t xl = __shfl(rlo, 16 * k, 64), xh = __shfl(rhi, 16 * k, 64);
        const int xd = __shfl(done, 16 * k, 64);
        if (xd && (lane / G) == ((uint32_t)sk / G)) {
          lo = xl;
          hi = xh;
        }
        if (!xd) keep |= 1ull << sk;
      }
    }
    wb = keep;
  } else {
    wb = __ballot(wide && j == 0);
  }
  // the remaining wide rows: one at a time by the whole wave (wave-uniform loop)
  while (wb) {
    const int src = __ffsll((long long)wb) - 1;
    wb &= wb - 1;
    uint64_t wl = __shfl(l, src, 64), wh = __shfl(h, src, 64);
    const int64_t ws = __shfl(sym, src, 64);
    const uint32_t* cbm;
    int64_t one;
    lf_step_decode(v, ws, wl, wh, cbm, one);
    if ((lane / G) == ((uint32_t)src / G)) {
      lo = wl;
      hi = wh;
    }
  }
}

#ifndef FMIDX_GROUP_WPE
#define FMIDX_GROUP_WPE 0
#endif
#if FMIDX_GROUP_WPE > 0
#define FMIDX_GROUP_ATTR __attribute__((amdgpu_waves_per_eu(FMIDX_GROUP_WPE, FMIDX_GROUP_WPE)))
#else
#define FMIDX_GROUP_ATTR
#endif
template <int G, bool GP, bool Q>
__global__ void __launch_bounds__(kLfThreads) FMIDX_GROUP_ATTR k_lf_group(DevView v, const int64_t* __restrict__ tok,
                                                        int64_t shift, int64_t reset_below,
                                                        const uint64_t* lo_in, const uint64_t* hi_in,
                                                        uint64_t* lo_out, uint64_t* hi_out, uint64_t m) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 6;
  if (wave * (64 / G) >= m) return;      // wave-uniform
  const uint64_t i = wave * (64 / G) + lane / G;
  const bool valid = i < m;
  const uint64_t ii = valid ? i : m - 1;
  const int64_t t = (int64_t)row_load_u64(tok, m, ii);
  const uint64_t l = row_load_u64(lo_in, m, ii), h = row_load_u64(hi_in, m, ii);
  uint64_t nl, nh;
  // a reset row takes no step (never joins the wide-row ballots); it is replaced below
  group_step<G, GP, Q>(v, valid && t >= reset_below, t + shift, l, h, nl, nh);
  if (t < reset_below) {
    nl = 0;
    nh = v.n;
  }
  if (valid && (lane & (G - 1)) == 0) {
    lo_out[i] = nl;
    hi_out[i] = nh;
  }
}

// The split launch of a large LF batch (fm_lf_step_batch above
// FMIDX_LF_GROUP_MIN rows): this pass steps the cheap rows -- reset, dead, full
// range, <= kPackMax-row E scans -- with no wide-row code at all (few VGPRs:
// many waves per SIMD, the whole batch's random E reads in flight), and leaves
// the wide rows to k_lf_wide (tagged in the outputs).  A wave whose rows are all cheap was
// held up before by any one wide row among its 64 / G (a probe, a descent,
// stepped one at a time by the whole wave).
template <int G>
__global__ void __launch_bounds__(kLfThreads) k_lf_cheap(DevView v, const int64_t* __restrict__ tok,
                                                        int64_t shift, int64_t reset_below,
                                                        const uint64_t* lo_in, const uint64_t* hi_in,
                                                        uint64_t* lo_out, uint64_t* hi_out, uint64_t m) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 6;
  if (wave * (64 / G) >= m) return;      // wave-uniform
  const uint64_t i = wave * (64 / G) + lane / G;
  const bool valid = i < m;
  const uint64_t ii = valid ? i : m - 1;
  const int64_t t = (int64_t)row_load_u64(tok, m, ii);
  const uint64_t l = row_load_u64(lo_in, m, ii), h = row_load_u64(hi_in, m, ii);
  const bool live = valid && t >= reset_below;
  uint64_t nl, nh;
  group_step<G, false, false, true>(v, live, t + shift, l, h, nl, nh);
  if (t < reset_below) {
    nl = 0;
    nh = v.n;
  }
  if (valid && (lane & (G - 1)) == 0) {
    // a wide row is handed to k_lf_wide through the output buffers: its input
    // range, tagged (n < 2^34, so no result has bit 63).  Through the outputs,
    // not the inputs: an in-place launch has overwritten the cheap rows' inputs.
    const bool wide = lf_wide(v, live, t + shift, l, h);
    lo_out[i] = wide ? l : nl;
    hi_out[i] = wide ? (h < v.n ? h : v.n) | kLfWideTag : nh;
  }
}

// The split launch's second pass: only the wide rows step (group_step's probe
// stage four at a time, then one at a time by the whole wave); the others are
// not written.
template <int G, bool Q>
__global__ void __launch_bounds__(kLfThreads) k_lf_wide(DevView v, const int64_t* __restrict__ tok,
                                                       int64_t shift, uint64_t* lo_out, uint64_t* hi_out,
                                                       uint64_t m) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 6;
  if (wave * (64 / G) >= m) return;      // wave-uniform
  const uint64_t i = wave * (64 / G) + lane / G;
  const bool valid = i < m;
  const uint64_t ii = valid ? i : m - 1;
  const uint64_t hw = hi_out[ii];
  const bool wide = valid && (hw & kLfWideTag);
  if (!__ballot(wide)) return;           // wave-uniform: no wide row here
  const int64_t t = (int64_t)row_load_u64(tok, m, ii);
  const uint64_t l = lo_out[ii], h = hw & ~kLfWideTag;
  uint64_t nl, nh;
  group_step<G, false, Q>(v, wide, t + shift, l, h, nl, nh);
  if (wide && (lane & (G - 1)) == 0) {
    lo_out[i] = nl;
    hi_out[i] = nh;
  }
}

template <int G, bool GP, bool Q, bool P8 = false>
__global__ void __launch_bounds__(kLfThreads, P8 ? 4 : 1) k_search_group(DevView v, const int64_t* __restrict__ tok,
                                                            const int64_t* __restrict__ off, uint64_t m,
                                                            int64_t shift, const uint64_t* lo_in,
                                                            const uint64_t* hi_in, uint64_t* lo_out,
                                                            uint64_t* hi_out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 6;
  if (wave * (64 / G) >= m) return;      // wave-uniform
  const uint64_t i = wave * (64 / G) + lane / G;
  const bool valid = i < m;
  const uint64_t ii = valid ? i : m - 1;
  uint64_t l = lo_in ? lo_in[ii] : 0;
  uint64_t h = hi_in ? hi_in[ii] : v.n;
  int64_t j = off[ii];
  const int64_t b = valid ? off[ii + 1] : j;
  bool active = j < b;
  while (__ballot(active)) {           // wave-uniform: until every group's pattern is done
    const int64_t t = tok[active ? j : 0];   // some group is active: tok has an element
    uint64_t nl, nh;
    group_step<G, GP, Q, false, P8>(v, active, t + shift, l, h, nl, nh);
    if (active) {
      l = nl;
      h = nh;
      ++j;
      if ((l == 0 && h == 0) || j >= b) active = false;   // index.py:111-112
    }
  }
  if (valid && (lane & (G - 1)) == 0) {
    lo_out[i] = l;
    hi_out[i] = h;
  }
}

// ------------------------------------------------------------ worklist LF
// (opt-in, FMIDX_LF_WORK=1: exact -- the LF parity test runs it -- but measured
// no faster than the grouped kernel at C3, 2^19 cold pairs: k_lf_sweep 45 us +
// k_lf_tail 25 us + the counter memset and two dependent launches, 92 us per
// call against 76; warm 26 + 18.  profiles/r03_rank/worklist/.)
// Throughput form of fm_lf_step_batch above FMIDX_LF_GROUP_MIN rows, in two
// launches that keep every lane of a wave on one kind of work.  (The grouped
// kernels above serialise a wave's wide rows behind each other, so a wave of
// 32 mostly-narrow rows lives as long as its slowest wide rows' chains.)
//   k_lf_sweep  one lane per row: reset / dead rows, the full range (C
//               lookup), every range of <= kSweepScan rows -- its E entries
//               scanned packed end to end over the wave, so a load
//               instruction touches about one line per row -- and every
//               cached range's transition probe, eight rows at a time with 8
//               lanes each (the 16-slot run staged through LDS from 128-B-wide
//               loads, the range's own range-cache run alongside), issued in
//               the same round trip as the E scan.  Everything else -- ranges
//               of 65..512 rows, uncached wide ranges, probe misses -- goes to
//               the tail list: one atomic per workgroup (returning device
//               atomics are the expensive part of an append: two per wave cost
//               ~30 us over 2^19 rows);
//   k_lf_tail   persistent waves over the tail list, one row per wave: an E
//               scan of <= 512 rows or the 2-level descent (a probe miss
//               starts it with the range's cached bitmap word, so a symbol the
//               range lacks ends after the first level).
// The tail list is split into kWorkRegions regions (region = the appending
// workgroup's index mod kWorkRegions) so the atomics spread over as many
// counters; k_lf_tail's waves are assigned to regions the same way.  Every row
// is written exactly once, by the kernel that settles it, so in-place launches
// (lo_out == lo_in) stay correct.
struct LfWork {
  uint64_t l, h;   // the row's range (h clamped to n)
  uint64_t sym;    // symbol | (cache id + 1 of the range, for a probe miss) << 32
  uint64_t row;
};
constexpr uint32_t kWorkRegions = 64;
constexpr uint64_t kSweepScan = 64;   // widest range k_lf_sweep scans in E
#ifndef FMIDX_SWEEP_PASS
#define FMIDX_SWEEP_PASS 2
#endif
constexpr int kSweepPass = FMIDX_SWEEP_PASS;   // 64-entry passes per round trip of the packed scan (2: 92 VGPRs; 4: 100)
// The 2-level descent / wide E scan, by a whole wave (uniform inputs;
// lo < hi <= n, not the full range, sym valid).  pword = the range's cached
// bitmap word holding bit c (~0 when unknown): a symbol the range lacks ends the
// step after the descent's first level.
__device__ __forceinline__ void lf_step_tail(const DevView& v, uint64_t c, uint32_t pword, uint64_t& lo,
                                             uint64_t& hi) {
  if (v.E && hi - lo <= kENarrow) {
    uint32_t cm = 0;
    lf_step_fast<false>(v, (int64_t)c, lo, hi, nullptr, cm);
    return;
  }
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t q = lane & 31u;
  const bool side = lane >= 32;
  const uint32_t c32 = (uint32_t)c;
  const int64_t dd = v.D2[c32];
  uint64_t z[kW2MaxLevels];
#pragma unroll
  for (int l = 0; l < kW2MaxLevels; ++l)
    z[l] = (l < (int)v.NL2) ? v.w2[l].Z[(c32 >> v.w2[l].shift) & ((1u << v.w2[l].bits) - 1u)] : 0;
  uint64_t pos = side ? hi : lo;
#pragma unroll 1
  for (int l = 0; l < (int)v.NL2; ++l) {
    const uint32_t d = (c32 >> v.w2[l].shift) & ((1u << v.w2[l].bits) - 1u);
    const uint64_t r = rank_w2(v.w2[l], pos, d, q);
    if (l == 0 && !((pword >> (c32 & 31u)) & 1u)) {
      lo = 0;
      hi = 0;
      return;
    }
    pos = z[l] + r;
  }
  const uint64_t other = __shfl_xor(pos, 32, 64);
  const uint64_t l2 = side ? other : pos, h2 = side ? pos : other;
  if (l2 >= h2) {
    lo = 0;
    hi = 0;
    return;
  }
  lo = (uint64_t)((int64_t)l2 + dd);
  hi = (uint64_t)((int64_t)h2 + dd);
}

// The 2-level descent of FOUR ranges at once, one per quarter-wave (lanes
// 16 r .. 16 r + 15: row r; within a quarter, 8 lanes rank the lower end and 8
// the upper, rank_w2_q8 -- at most half a block of digits per rank): the LF
// sweep's tail rows four at a time, so a wave waits one descent's round trips
// for four rows.  Inputs uniform within each quarter (lo < hi <= n, not the
// full range, sym valid); pword as for lf_step_tail -- a symbol the range lacks
// makes the row empty, and when every active row of the wave lacks its symbol
// the second level is skipped.  act = false: the quarter's result is
// unspecified (its inputs must still be a valid range).
__device__ __forceinline__ void lf_descend_quad(const DevView& v, bool act, uint64_t c, uint32_t pword, uint64_t& lo,
                                                uint64_t& hi) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t q = lane & 7u;
  const bool side = ((lane >> 3) & 1u) != 0;
  const uint32_t c32 = (uint32_t)c;
  const int64_t dd = v.D2[c32];
  uint64_t z[kW2MaxLevels];
#pragma unroll
  for (int l = 0; l < kW2MaxLevels; ++l)
    z[l] = (l < (int)v.NL2) ? v.w2[l].Z[(c32 >> v.w2[l].shift) & ((1u << v.w2[l].bits) - 1u)] : 0;
  uint64_t pos = side ? hi : lo;
  const bool absent = !((pword >> (c32 & 31u)) & 1u);
#pragma unroll 1
  for (int l = 0; l < (int)v.NL2; ++l) {
    const uint32_t d = (c32 >> v.w2[l].shift) & ((1u << v.w2[l].bits) - 1u);
    const uint64_t r = rank_w2_q8(v.w2[l], pos, d, q, v.n);
    pos = z[l] + r;
    if (l == 0 && __all(absent || !act)) break;   // wave-uniform
  }
  const uint64_t other = __shfl_xor(pos, 8, 64);
  const uint64_t l2 = side ? other : pos, h2 = side ? pos : other;
  if (absent || l2 >= h2) {
    lo = 0;
    hi = 0;
    return;
  }
  lo = (uint64_t)((int64_t)l2 + dd);
  hi = (uint64_t)((int64_t)h2 + dd);
}

#ifndef FMIDX_SWEEP_TAIL_BATCH
#define FMIDX_SWEEP_TAIL_BATCH 1   // measurement variant 0: the tail rows one at a time (round 3-5's form)
#endif
constexpr int kTailPass = 8;      // 64-entry passes per round trip of the tail rows' packed E scan

// occupancy experiments (make qvariant VFLAGS=-DFMIDX_SWEEP_WPE=6): waves per SIMD forced on the sweep
#ifndef FMIDX_SWEEP_WPE
#define FMIDX_SWEEP_WPE 0
#endif
#if FMIDX_SWEEP_WPE > 0
#define FMIDX_SWEEP_ATTR __attribute__((amdgpu_waves_per_eu(FMIDX_SWEEP_WPE, FMIDX_SWEEP_WPE)))
#else
#define FMIDX_SWEEP_ATTR
#endif
// One wave's 64 rows of the LF sweep up to its tail rows (the head): the row
// state (token, lo, hi: one round trip), the C lookup of full-range rows, the
// narrow rows' E entries packed end to end over the wave, the cached rows'
// transition probes eight at a time -- every row settled except the tail rows
// (E scans of 65..512 rows, uncached wide ranges, probe misses), which come back
// flagged with their (l, h, c, pid1).  i = this lane's row; valid = i < m.
struct SweepRow {
  uint64_t l, h, c;       // the row's range (h clamped to n) and symbol
  uint64_t nl, nh;        // its new range (settled rows)
  uint64_t pid1;          // a probe miss: the range's cache id + 1 (0: unknown)
  bool tail;              // still to step (sweep_tails)
};

__device__ __forceinline__ void sweep_head(const DevView& v, const int64_t* __restrict__ tok, int64_t shift,
                                           int64_t reset_below, const uint64_t* lo_in, const uint64_t* hi_in,
                                           uint64_t m, uint64_t i, bool valid, unsigned long long (*mm)[64],
                                           uint4* run, SweepRow& r) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t seg = lane / kProbeLanes;
  const uint64_t ii = valid ? i : m - 1;
  const int64_t t = (int64_t)row_load_u64(tok, m, ii);
  const uint64_t l = row_load_u64(lo_in, m, ii);
  uint64_t h = row_load_u64(hi_in, m, ii);
  if (h > v.n) h = v.n;
  const int64_t sym = t + shift;
  const bool reset = valid && t < reset_below;
  const bool live = valid && !reset;
  const bool dead = live && (l >= h || sym < 0 || (uint64_t)sym > v.max_sym);
  const bool full = live && !dead && l == 0 && h == v.n;
  const bool step = live && !dead && !full;
  const bool narrow = step && v.E && h - l <= kSweepScan;
  const bool probe = step && !narrow && v.trans_cap && h - l >= v.cache_min;
  bool tail = step && !narrow && !probe;
  const uint64_t c = (uint64_t)sym;
  const uint64_t cf = full ? c : 0;   // the others all read C[0..1]: one shared line
  const uint64_t ca = v.C[cf], cb = v.C[cf + 1];
  // ---- packed E scan: the narrow rows' entries end to end over the wave
  const uint32_t cnt_e = narrow ? (uint32_t)(h - l) : 0u;
  uint32_t inc = cnt_e;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= (uint32_t)d) inc += y;
  }
  const uint32_t excl = inc - cnt_e;
  const uint32_t total = __shfl(inc, 63, 64);
  mm[0][lane] = ~0ull;
  mm[1][lane] = 0;
  __builtin_amdgcn_wave_barrier();
  uint64_t pmask = __ballot(probe);   // probe rows left, batches of kProbeRows
  uint64_t res_lo = 0, res_hi = 0, pid1 = 0;   // a probe row's result (on its own lane)
  bool probed = false;
  for (uint32_t t0 = 0; t0 < total || pmask; t0 += 64 * kSweepPass) {   // wave-uniform
    uint64_t xs[kSweepPass], cs[kSweepPass];
    uint32_t rs[kSweepPass];
#pragma unroll
    for (int k = 0; k < kSweepPass; ++k) {
      const uint32_t e = t0 + 64u * k + lane;
      uint32_t rr = 0;   // the last row whose offset is <= e (rows of no entries are never it)
#pragma unroll
      for (int st = 32; st > 0; st >>= 1) {
        const uint32_t x = __shfl(excl, (int)(rr + st), 64);
        if (x <= e) rr += st;
      }
      const uint64_t base = __shfl(l, (int)rr, 64);
      const uint32_t off = e - __shfl(excl, (int)rr, 64);
      cs[k] = __shfl(c, (int)rr, 64);
      // unconditional (a surplus lane reads E[0]: one shared line)
      xs[k] = v.E[e < total ? base + off : 0];
      rs[k] = e < total ? rr : ~0u;
    }
    // the next batch of probe rows, in the same round trip
    int src = -1;
    {
      uint64_t pm = pmask;
      for (uint32_t k = 0; k < kProbeRows && pm; ++k) {
        const int s = __ffsll((long long)pm) - 1;
        pm &= pm - 1;
        if (seg == k) src = s;
      }
      pmask = pm;
    }
    const bool pact = src >= 0;
    const int ps = pact ? src : 0;
    const uint64_t pl = __shfl(l, ps, 64), ph = __shfl(h, ps, 64), pc = __shfl(c, ps, 64);
    // (no transition table: no row is a probe row and this batch is empty;
    // the loads are skipped wave-uniformly)
    ProbeLoads pld = {};
    if (v.trans_cap) pld = probe_issue(v, pl, ph, pc);
#pragma unroll
    for (int k = 0; k < kSweepPass; ++k) {
      if (rs[k] != ~0u && (xs[k] >> kESymShift) == cs[k]) {
        atomicMin(&mm[0][rs[k]], (unsigned long long)(xs[k] & kELfMask));
        atomicMax(&mm[1][rs[k]], (unsigned long long)(xs[k] & kELfMask));
      }
    }
    if (v.trans_cap && __ballot(pact)) {
      bool hit;
      uint64_t clo, chi, p1;
      probe_finish(v, pl, ph, pc, pact, pld, run, hit, clo, chi, p1);
      // hand each probed row its result (the batch's k-th row sits in segment k)
#pragma unroll
      for (uint32_t k = 0; k < kProbeRows; ++k) {
        const int sk = __shfl(src, (int)(k * kProbeLanes), 64);
        const uint64_t xl = __shfl(clo, (int)(k * kProbeLanes), 64), xh = __shfl(chi, (int)(k * kProbeLanes), 64);
        const uint64_t xp = __shfl(p1, (int)(k * kProbeLanes), 64);
        const int xhit = __shfl((int)hit, (int)(k * kProbeLanes), 64);
        if (sk >= 0 && (int)lane == sk) {
          probed = xhit != 0;
          res_lo = xl;
          res_hi = xh;
          pid1 = xp;
        }
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  // LF is increasing over a symbol's rows: the new range is [min LF, max LF + 1) of the matches
  const uint64_t fmin = mm[0][lane], fmax = mm[1][lane];
  uint64_t nl = 0, nh = 0;
  if (reset) {
    nl = 0;
    nh = v.n;
  } else if (full) {
    nl = ca < cb ? ca : 0;
    nh = ca < cb ? cb : 0;
  } else if (narrow && fmin != ~0ull) {
    nl = fmin;
    nh = fmax + 1;
  } else if (probed) {
    nl = res_lo;
    nh = res_hi;
  }
  r.l = l;
  r.h = h;
  r.c = c;
  r.nl = nl;
  r.nh = nh;
  r.pid1 = pid1;
  r.tail = tail || (probe && !probed);
}

// The wave's tail rows (lanes with r.tail; their (l, h, c, pid1) per lane), stepped together, the
// results into r.nl / r.nh of those lanes (1.8 tail rows per 64 on a decode trace: 0.8 E scans of
// 65..512 rows, 1.0 descents; stepped one at a time they were 37 % of the sweep's time at 2^19
// pairs in round 5):
//  (1) every E-scan tail of the wave in ONE packed scan (their entries end to end over the
//      wave, kTailPass passes per round trip), not one lf_step_fast round trip per row;
//  (2) the descents four at a time, one per quarter-wave (lf_descend_quad).
// A probe miss of a range whose bitmap is cached (pid1): the range's word for c, every such row of
// the wave at once and in the round trip of (1) -- a symbol the range lacks (nearly every miss:
// 0.15 % of the keys are left out of the table) settles the row as empty with no descent.
// mm: the wave's LDS slots, untouched since the head for these rows (or reset by the caller).
__device__ __forceinline__ void sweep_tails(const DevView& v, unsigned long long (*mm)[64], SweepRow& r) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool tail = r.tail;
  const uint64_t l = r.l, h = r.h, c = r.c, pid1 = r.pid1;
  uint64_t nl = r.nl, nh = r.nh;
  const bool pm = tail && pid1 != 0;
  const uint32_t* pwp = pm ? v.cache_bm + (pid1 - 1) * v.bm_words + ((uint32_t)c >> 5)
                           : reinterpret_cast<const uint32_t*>(v.C);
  const uint32_t pword_own = pm ? *pwp : ~0u;
  const bool t1 = tail && v.E && h - l <= kENarrow;
  {
    const uint32_t cnt1 = t1 ? (uint32_t)(h - l) : 0u;
    uint32_t inc1 = cnt1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc1, d, 64);
      if (lane >= (uint32_t)d) inc1 += y;
    }
    const uint32_t excl1 = inc1 - cnt1;
    const uint32_t total1 = __shfl(inc1, 63, 64);
    for (uint32_t t0 = 0; t0 < total1; t0 += 64 * kTailPass) {   // wave-uniform
      uint64_t xs[kTailPass], cs[kTailPass];
      uint32_t rs[kTailPass];
#pragma unroll
      for (int k = 0; k < kTailPass; ++k) {
        const uint32_t e = t0 + 64u * k + lane;
        uint32_t rr = 0;   // the last row whose offset is <= e (rows of no entries are never it)
#pragma unroll
        for (int st = 32; st > 0; st >>= 1) {
          const uint32_t x = __shfl(excl1, (int)(rr + st), 64);
          if (x <= e) rr += st;
        }
        const uint64_t base = __shfl(l, (int)rr, 64);
        const uint32_t off = e - __shfl(excl1, (int)rr, 64);
        cs[k] = __shfl(c, (int)rr, 64);
        xs[k] = v.E[e < total1 ? base + off : 0];   // unconditional (a surplus lane reads E[0])
        rs[k] = e < total1 ? rr : ~0u;
      }
#pragma unroll
      for (int k = 0; k < kTailPass; ++k) {
        if (rs[k] != ~0u && (xs[k] >> kESymShift) == cs[k]) {
          atomicMin(&mm[0][rs[k]], (unsigned long long)(xs[k] & kELfMask));
          atomicMax(&mm[1][rs[k]], (unsigned long long)(xs[k] & kELfMask));
        }
      }
    }
    if (total1) {   // wave-uniform; the slots of these rows were untouched by the narrow scan
      __builtin_amdgcn_wave_barrier();
      const uint64_t f0 = mm[0][lane], f1 = mm[1][lane];
      if (t1) {
        nl = f0 != ~0ull ? f0 : 0;
        nh = f0 != ~0ull ? f1 + 1 : 0;
      }
    }
  }
#ifdef FMIDX_SWEEP_SKIP_TAIL   // measurement variant (wrong results): the launch without its tail rows' steps
  uint64_t tb = 0;
#else
  const bool absent = pm && !((pword_own >> ((uint32_t)c & 31u)) & 1u);   // nl = nh = 0 already
  if (absent) {
    nl = 0;
    nh = 0;
  }
  uint64_t tb = __ballot(tail && !t1 && !absent);
#endif
  while (tb) {   // wave-uniform: up to four rows per round, quarter-wave q takes the q-th
    int sv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      sv[k] = tb ? __ffsll((long long)tb) - 1 : -1;
      if (tb) tb &= tb - 1;
    }
    const uint32_t qw = lane >> 4;
    const int src = qw == 0 ? sv[0] : (qw == 1 ? sv[1] : (qw == 2 ? sv[2] : sv[3]));
    const bool act = src >= 0;
    const int s_ = act ? src : sv[0];   // an idle quarter repeats the first row (valid inputs), its result unused
    uint64_t tl = __shfl(l, s_, 64), th = __shfl(h, s_, 64);
    const uint64_t tc = __shfl(c, s_, 64);
    lf_descend_quad(v, act, tc, __shfl(pword_own, s_, 64), tl, th);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t rl = __shfl(tl, 16 * k, 64), rh = __shfl(th, 16 * k, 64);
      if (sv[k] >= 0 && (int)lane == sv[k]) {
        nl = rl;
        nh = rh;
      }
    }
  }
  r.nl = nl;
  r.nh = nh;
}

template <bool INLINE>
__global__ void __launch_bounds__(kLfThreads) FMIDX_SWEEP_ATTR k_lf_sweep(DevView v, const int64_t* __restrict__ tok, int64_t shift,
                                                        int64_t reset_below, const uint64_t* lo_in,
                                                        const uint64_t* hi_in, uint64_t* lo_out, uint64_t* hi_out,
                                                        uint64_t m, LfWork* lt, uint32_t* cnt, uint64_t cap) {
  __shared__ unsigned long long s_mm[kLfThreads / 64][2][64];
  __shared__ uint32_t s_n[kLfThreads / 64 + 1];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  const uint64_t i = (uint64_t)blockIdx.x * kLfThreads + threadIdx.x;
  // (no early return: every wave of the workgroup reaches the append's barriers)
  const bool valid = i < m;
  SweepRow r;
  sweep_head(v, tok, shift, reset_below, lo_in, hi_in, m, i, valid, s_mm[wv], nullptr, r);
  if (INLINE) {
#if FMIDX_SWEEP_TAIL_BATCH
    sweep_tails(v, s_mm[wv], r);
#else
    // the wave's tail rows one at a time by the whole wave (lf_step_tail), then every row is written
#ifdef FMIDX_SWEEP_SKIP_TAIL   // measurement variant (wrong results): the launch without its tail rows' steps
    uint64_t tb = 0;
#else
    uint64_t tb = __ballot(r.tail);
#endif
    while (tb) {
      const int src = __ffsll((long long)tb) - 1;
      tb &= tb - 1;
      uint64_t tl = __shfl(r.l, src, 64), th = __shfl(r.h, src, 64);
      const uint64_t tc = __shfl(r.c, src, 64), tp = __shfl(r.pid1, src, 64);
      const uint32_t* pw = tp ? v.cache_bm + (tp - 1) * v.bm_words + ((uint32_t)tc >> 5)
                                : reinterpret_cast<const uint32_t*>(v.C);
      const uint32_t pword = tp ? *pw : ~0u;
      lf_step_tail(v, tc, pword, tl, th);
      if ((int)lane == src) {
        r.nl = tl;
        r.nh = th;
      }
    }
#endif
    if (valid) {
      lo_out[i] = r.nl;
      hi_out[i] = r.nh;
    }
    return;
  }
  const bool tail = r.tail;
  if (valid && !tail) {
    lo_out[i] = r.nl;
    hi_out[i] = r.nh;
  }
  // ---- tail rows: one atomic per workgroup (LDS-only barriers: nothing
  // crossing them is global data, so the stores above need not drain)
  const uint64_t tb = __ballot(tail);
  if (lane == 0) s_n[wv] = (uint32_t)__popcll(tb);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  const uint32_t rg = (uint32_t)(blockIdx.x % kWorkRegions);
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (uint32_t w = 0; w < kLfThreads / 64; ++w) tot += s_n[w];
    s_n[kLfThreads / 64] = tot ? atomicAdd(&cnt[rg], tot) : 0u;
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (tail) {
    uint32_t pos = s_n[kLfThreads / 64];
    for (uint32_t w = 0; w < wv; ++w) pos += s_n[w];
    pos += (uint32_t)__popcll(tb & ((1ull << lane) - 1));
    lt[(uint64_t)rg * cap + pos] = LfWork{r.l, r.h, r.c | (r.pid1 << 32), i};
  }
}

// ------------------------------------------------- persistent LF sweep (lf_work 4)
// The in-wave sweep above lives its rows' longest chain: a wave whose 64 rows hold a descent or a
// wide E scan lives 16-27 us where one without lives 10 (round 5's stamps), and a 2^19-pair launch
// is 1.6 residency rounds of such waves, so its last waves start late and end later.  Here the grid
// is the resident wave count W (a multiple of kPParts), and every wave
//   heads  runs the head (sweep_head) of chunks w, w + W, w + 2W, ... (64 rows each), stores the
//          settled rows and APPENDS the tail rows to the tail queue q = chunk mod kPParts (= w mod
//          kPParts: one atomic per chunk reserves the slots; each entry is written write-through
//          and, once performed, its 4-B tag = the launch's epoch); then it counts the chunk in
//          the queue's head count (after its tags are performed);
//   drain  then takes kPClaim slots of its own queue at a time with ONE fetch-and-add on the
//          queue's claim counter (no compare-and-swap: round 6's first two versions claimed only
//          reserved slots by CAS, and 4096 waves retrying CAS on 16 counters made the launch
//          9-15x slower than the in-wave sweep), waits for each slot's tag -- or, once the head
//          count says every chunk of the queue is done, for the slot to lie past the final tail
//          (an empty slot) -- and steps the ready rows together (sweep_tails: E scans packed, the
//          descents one per quarter-wave).  A wave leaves when its claim lies wholly past the
//          final tail.
// A claimed slot may not be reserved yet, so a drainer can wait on another wave's heads: every
// wave of the grid must be resident (the grid is the occupancy x CUs; a launch beside other work
// that keeps waves off the chip can only end by the bounded poll, kPersistSpins, which sets the
// error word -- fm_lf_persist_status reports it).  Counters: two sets (the epoch's parity), each
// counter on its own 128-B line; a launch zeroes the other set for the next launch on the stream.
// Not captured into graphs (the API launches it only on a stream that is not capturing).
constexpr uint32_t kPParts = 64;                  // tail queues
constexpr uint32_t kPClaim = 8;                   // slots per claim
constexpr uint32_t kPStride = 32;                 // words between counters
constexpr uint32_t kPCounters = 3 * kPParts;      // qtail (reserved), qhead (claimed), hdone (chunks done)
constexpr uint32_t kPSetWords = kPCounters * kPStride;
constexpr uint32_t kPersistSpins = 1u << 22;
constexpr int kPSysAux = 16;                      // sc1: entries written through, read past the L1
static_assert(kPCounters <= kLfThreads, "one thread zeroes each counter of the next set");

struct PersistWs {
  uint32_t* ctr;     // 2 x kPSetWords
  LfWork* tq;        // kPParts x qcap
  uint32_t* tag;     // kPParts x qcap
  uint32_t* err;     // a tag poll ran out: the launch's rows are not all stepped
};

__device__ __forceinline__ uint32_t* pctr(uint32_t* set, uint32_t which, uint32_t q) {
  return set + (which * kPParts + q) * kPStride;
}

__global__ void __launch_bounds__(kLfThreads) k_lf_persist(DevView v, const int64_t* __restrict__ tok, int64_t shift,
                                                          int64_t reset_below, const uint64_t* lo_in,
                                                          const uint64_t* hi_in, uint64_t* lo_out, uint64_t* hi_out,
                                                          uint64_t m, PersistWs ws, uint32_t qcap, uint32_t epoch) {
  __shared__ unsigned long long s_mm[kLfThreads / 64][2][64];
  typedef unsigned v4u_ __attribute__((ext_vector_type(4)));
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t* set = ws.ctr + (epoch & 1u) * kPSetWords;
  if (blockIdx.x == 0 && threadIdx.x < kPCounters)   // the next launch's counters
    ws.ctr[((epoch + 1u) & 1u) * kPSetWords + threadIdx.x * kPStride] = 0u;
  const uint64_t nchunks = (m + 63) / 64;
  const uint64_t gw = (uint64_t)blockIdx.x * (kLfThreads / 64) + wv;
  const uint64_t nw = (uint64_t)gridDim.x * (kLfThreads / 64);   // a multiple of kPParts
  const uint32_t q = (uint32_t)(gw % kPParts);
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(ws.tq + (uint64_t)q * qcap, qcap * (uint32_t)sizeof(LfWork));
  uint32_t* qt = pctr(set, 0, q);
  uint32_t* qh = pctr(set, 1, q);
  uint32_t* hd = pctr(set, 2, q);
  // ---- heads: chunks gw, gw + nw, ...
  for (uint64_t chunk = gw; chunk < nchunks; chunk += nw) {   // wave-uniform
    const uint64_t i = chunk * 64 + lane;
    const bool valid = i < m;
    SweepRow r;
    sweep_head(v, tok, shift, reset_below, lo_in, hi_in, m, i, valid, s_mm[wv], nullptr, r);
    const bool tail = valid && r.tail;
    if (valid && !tail) {
      lo_out[i] = r.nl;
      hi_out[i] = r.nh;
    }
    const uint64_t tb = __ballot(tail);
    if (tb) {   // wave-uniform
      uint32_t base = 0;
      if (lane == 0)
        base = __hip_atomic_fetch_add(qt, (uint32_t)__popcll(tb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      base = __shfl(base, 0, 64);
      const uint32_t pos = base + (uint32_t)__popcll(tb & ((1ull << lane) - 1));
      if (tail) {   // pos < qcap: a queue holds every row of its chunks
        const uint64_t sp = r.c | (r.pid1 << 32);
        const v4u_ a = {(uint32_t)r.l, (uint32_t)(r.l >> 32), (uint32_t)r.h, (uint32_t)(r.h >> 32)};
        const v4u_ b = {(uint32_t)sp, (uint32_t)(sp >> 32), (uint32_t)i, (uint32_t)(i >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(a, rq, pos * (uint32_t)sizeof(LfWork), 0, kPSysAux);
        __builtin_amdgcn_raw_buffer_store_b128(b, rq, pos * (uint32_t)sizeof(LfWork) + 16u, 0, kPSysAux);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every entry performed before its tag
      if (tail)
        __hip_atomic_store(ws.tag + (uint64_t)q * qcap + pos, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every tag performed before the chunk counts
    }
    if (lane == 0) __hip_atomic_fetch_add(hd, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // ---- drain: this wave's queue, kPClaim slots per claim
  const uint32_t qchunks = nchunks > q ? (uint32_t)((nchunks - 1 - q) / kPParts + 1) : 0u;
  const bool mine = lane < kPClaim;
  for (;;) {
    uint32_t j0 = 0;
    if (lane == 0) j0 = __hip_atomic_fetch_add(qh, kPClaim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    j0 = __shfl(j0, 0, 64);
    const uint32_t j = j0 + lane;
    // per slot: 1 ready (tagged), 2 empty (past the final tail), 0 not yet known
    uint32_t st = mine ? 0u : 2u;
    uint32_t spin = 0;
    for (; spin < kPersistSpins; ++spin) {
      if (st == 0 && j < qcap &&
          __hip_atomic_load(ws.tag + (uint64_t)q * qcap + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch)
        st = 1;
      if (__all(st != 0)) break;
      uint32_t fin = 0, t = 0;
      if (lane == 0) {
        fin = __hip_atomic_load(hd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == qchunks;
        if (fin) t = __hip_atomic_load(qt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      fin = __shfl(fin, 0, 64);
      t = __shfl(t, 0, 64);
      if (fin && st == 0 && j >= t) st = 2;   // below the final tail, the tag is performed: re-read
      if (__all(st != 0)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (spin == kPersistSpins) {
      if (lane == 0) __hip_atomic_store(ws.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    const bool ready = st == 1;
    if (!__ballot(ready)) break;   // the claim lies past the final tail: the queue is drained
    SweepRow r;
    r.tail = ready;
    r.nl = r.nh = 0;
    const uint32_t jj = ready ? j : j0;
    const v4u_ a = __builtin_amdgcn_raw_buffer_load_b128(rq, jj * (uint32_t)sizeof(LfWork), 0, kPSysAux);
    const v4u_ b = __builtin_amdgcn_raw_buffer_load_b128(rq, jj * (uint32_t)sizeof(LfWork) + 16u, 0, kPSysAux);
    r.l = (uint64_t)a.x | ((uint64_t)a.y << 32);
    r.h = (uint64_t)a.z | ((uint64_t)a.w << 32);
    const uint64_t sp = (uint64_t)b.x | ((uint64_t)b.y << 32);
    r.c = sp & 0xFFFFFFFFull;
    r.pid1 = sp >> 32;
    const uint64_t row = (uint64_t)b.z | ((uint64_t)b.w << 32);
    s_mm[wv][0][lane] = ~0ull;
    s_mm[wv][1][lane] = 0;
    __builtin_amdgcn_wave_barrier();
    sweep_tails(v, s_mm[wv], r);
    if (ready) {
      lo_out[row] = r.nl;
      hi_out[row] = r.nh;
    }
  }
}

// persistent over the tail list: wave w serves region w mod kWorkRegions, one
// row per iteration; the next row's entry is loaded ahead of the current step
__global__ void __launch_bounds__(kLfThreads) k_lf_tail(DevView v, const LfWork* __restrict__ lt,
                                                       const uint32_t* __restrict__ cnt, uint64_t cap,
                                                       uint64_t* lo_out, uint64_t* hi_out, uint32_t waves_per_region) {
  FM_PRELOAD_VIEW(v);
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = ((uint64_t)blockIdx.x * kLfThreads + threadIdx.x) >> 6;
  const uint32_t r = (uint32_t)(wave % kWorkRegions);
  const uint64_t nt = cnt[r];
  const LfWork* st = lt + (uint64_t)r * cap;
  uint64_t j = wave / kWorkRegions;
  if (j >= nt) return;   // wave-uniform
  LfWork it = st[j];
  for (; j < nt; j += waves_per_region) {   // wave-uniform
    const uint64_t jn = j + waves_per_region;
    const LfWork nx = st[jn < nt ? jn : j];
    uint64_t l = it.l, h = it.h;
    const uint32_t c32 = (uint32_t)it.sym;
    const uint64_t pid1 = it.sym >> 32;
    // a probe miss: the range's bitmap word for c (unconditional: C[0] as a dummy)
    const uint32_t* pw = pid1 ? v.cache_bm + (pid1 - 1) * v.bm_words + (c32 >> 5)
                              : reinterpret_cast<const uint32_t*>(v.C);
    const uint32_t pword = pid1 ? *pw : ~0u;
    lf_step_tail(v, c32, pword, l, h);
    if (lane == 0) {
      lo_out[it.row] = l;
      hi_out[it.row] = h;
    }
    it = nx;
  }
}

// (A class-list form of this launch -- k_lf_class settling the one-row / <= 8-row
// rows lane by lane and appending the rest to three per-class lists for a
// persistent k_lf_lists -- was measured in round 5: exact eagerly, no faster
// (37 + 40 us of kernel time against the grouped kernel's 69-71 at 2^19 pairs,
// profiles/r05_rank/), and a run of it inside a captured graph faulted the GPU,
// so it was removed; it is in the history, tuning lf_work 3.)

// [sdsl] backward_search on an inclusive range with unsigned wrap-around.
__device__ void sdsl_backward_search(const DevView& v, uint64_t c, uint64_t l, uint64_t r,
                                     uint64_t& lr, uint64_t& rr) {
  const bool unknown = c > v.max_sym || (c > 0 && v.C[c + 1] == v.C[c]);
  if (unknown) {
    lr = 1;
    rr = 0;
    return;
  }
  uint64_t pl = l > v.n ? v.n : l;
  uint64_t pr = r + 1;
  if (pr > v.n) pr = v.n;
  descend_w2_thread(v, (uint32_t)c, pl, pr);
  lr = pl;
  rr = pr - 1;
}

__global__ void k_step_raw(DevView v, uint64_t sym, uint64_t low, uint64_t high, uint64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (high >= v.n) high = v.n - 1;      // fm_index.cpp:74-76
  if (low > high) {                      // :77-82
    out[0] = 0;
    out[1] = 0;
    return;
  }
  uint64_t lr, rr;
  sdsl_backward_search(v, sym, low, high, lr, rr);
  if (lr > rr) {                         // :87-92
    out[0] = 0;
    out[1] = 0;
    return;
  }
  out[0] = lr;
  out[1] = rr + 1;
}

__global__ void k_raw_multi(DevView v, const uint64_t* q, uint64_t len, uint64_t* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t l = 0, r = v.n - 1;           // fm_index.cpp:58-59
  for (uint64_t i = 0; i < len; ++i) sdsl_backward_search(v, q[i], l, r, l, r);
  out[0] = l;
  out[1] = r + 1;
}

// ------------------------------------------------------------------ distinct
struct Frontier {
  uint64_t* lo[2];
  uint64_t* hi[2];
  uint32_t* pre[2];
};

__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t* lds /*[4]*/, uint32_t& total) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) lds[wave] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint32_t t = lds[w];
    if ((uint32_t)w < wave) base += t;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return base + x - v;
}

// interval_symbols with counts: a level-synchronous BFS over the 2-level
// wavelet matrix, one workgroup (4 waves) per row.  A frontier node (a range
// of level l's sequence) is expanded by ONE wave into all R = 2^bits digit
// children at once: rank_d at both ends for every d = superblock count + block
// header + the digits before the end in its block, the last counted into an
// LDS histogram (lane j takes digits [16 j, 16 j + 16) of each end's block) --
// one round trip per node, 2 levels for a 17-bit alphabet (the 16-ary matrix
// this replaced took 5 levels of 16-way expansion and 14 GiB at C3).  Lane j
// owns digits [j R/64, (j+1) R/64) (or digit j when R < 64), so a wave scan of
// the per-lane child counts orders a node's children by digit; the four waves
// take consecutive nodes and a 4-entry LDS scan orders those.  Children are
// appended in (node, digit) order, so the final frontier is in ascending
// symbol order.  min_count > 1 prunes every prefix node holding fewer
// occurrences (only symbols occurring >= min_count times are reported, in
// O(width / min_count) space); child_lo, when given, receives LF(lo, c) =
// C[c] + rank_c(lo) of every reported symbol (the child range is
// [child_lo, child_lo + count)).
constexpr uint32_t kDistWaves = 4;
constexpr uint32_t kDistMaxR = 512;   // digits of <= 9 bits (device_build_w2)

__global__ void __launch_bounds__(256) k_distinct(DevView v, const uint64_t* __restrict__ lo_a,
                                                 const uint64_t* __restrict__ hi_a, uint64_t m,
                                                 const uint64_t* __restrict__ cap_off,
                                                 uint64_t* __restrict__ syms,
                                                 uint64_t* __restrict__ counts,
                                                 uint64_t* __restrict__ k_out, Frontier fr,
                                                 uint64_t min_count, uint64_t* __restrict__ child_lo,
                                                 bool cached_path) {
  __shared__ uint32_t wave_tot[4];
  __shared__ uint32_t s_hist[kDistWaves][2][kDistMaxR];
  __shared__ uint32_t s_cnt[kDistWaves];
  const uint64_t row = blockIdx.x;
  if (row >= m) return;
  uint64_t lo = lo_a[row], hi = hi_a[row];
  const uint64_t base = cap_off[row];
  const uint64_t cap = cap_off[row + 1] - base;
  // fm_index.cpp:127-133
  bool empty = (lo == hi);
  if (hi > v.n) hi = v.n;
  if (lo >= hi) empty = true;
  if (empty || cap == 0) {
    if (threadIdx.x == 0) k_out[row] = empty ? 0 : ~0ull;
    return;
  }
  if (cached_path && ((lo == 0 && hi == v.n) ? v.bm_full != nullptr : cache_find(v, lo, hi) != nullptr))
    return;   // k_distinct_cached's row
  if (lo == 0 && hi == v.n) {
    // The full range: its symbols and counts are the C array itself (symbol c
    // occurs C[c+1] - C[c] times, its child range starts at C[c]) -- one pass
    // over sigma instead of a BFS whose last level holds every symbol.  Each
    // thread takes a contiguous run of symbols; a block scan orders the output.
    const uint64_t sigma = (uint64_t)v.max_sym + 1;
    const uint64_t per = (sigma + 255) / 256;
    const uint64_t c0 = min<uint64_t>(sigma, threadIdx.x * per), c1 = min<uint64_t>(sigma, c0 + per);
    uint32_t mine = 0;
    for (uint64_t c = c0; c < c1; ++c) mine += (v.C[c + 1] - v.C[c] >= min_count) ? 1u : 0u;
    uint32_t tot;
    uint64_t pos = block_scan_u32(mine, wave_tot, tot);
    if (tot <= cap) {
      for (uint64_t c = c0; c < c1; ++c) {
        const uint64_t a = v.C[c], b = v.C[c + 1];
        if (b - a >= min_count) {
          syms[base + pos] = c;
          counts[base + pos] = b - a;
          if (child_lo) child_lo[base + pos] = a;
          ++pos;
        }
      }
    }
    if (threadIdx.x == 0) k_out[row] = tot <= cap ? tot : ~0ull;
    return;
  }
  uint64_t* alo = fr.lo[0] + base;
  uint64_t* ahi = fr.hi[0] + base;
  uint32_t* apre = fr.pre[0] + base;
  uint64_t* blo = fr.lo[1] + base;
  uint64_t* bhi = fr.hi[1] + base;
  uint32_t* bpre = fr.pre[1] + base;
  if (threadIdx.x == 0) {
    alo[0] = lo;
    ahi[0] = hi;
    apre[0] = 0;
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint64_t fc = 1;
  bool overflow = false;
  for (uint32_t lev = 0; lev < v.NL2; ++lev) {
    const W2Level& L = v.w2[lev];
    const uint32_t bits = L.bits, R = 1u << bits;
    const uint32_t per = R >= 64 ? R / 64 : 1u;   // digits per lane
    const uint32_t d0 = R >= 64 ? lane * per : lane;
    const bool lane_on = d0 < R;
    uint64_t out = 0;
    for (uint64_t t0 = 0; t0 < fc; t0 += kDistWaves) {   // workgroup-uniform
      const uint64_t i = t0 + wv;
      const bool node = i < fc;
      for (uint32_t d = lane; d < R; d += 64) {
        s_hist[wv][0][d] = 0;
        s_hist[wv][1][d] = 0;
      }
      __syncthreads();
      uint32_t p = 0;
      uint64_t sbv[2][8];
      uint32_t hdr[2][8];
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
          sbv[e][u] = 0;
          hdr[e][u] = 0;
        }
      if (node) {
        p = apre[i];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint64_t x = e ? ahi[i] : alo[i];
          const uint32_t k = (uint32_t)(x & (kW2Blk - 1));
          const uint8_t* blk = L.blocks + (x >> kW2BlkLog2) * L.blk_bytes;
          const uint64_t* sbp = L.sb + (x >> kW2SbLog2) * R;
#pragma unroll
          for (uint32_t u = 0; u < 8; ++u) {
            if (lane_on && u < per) {
              sbv[e][u] = sbp[d0 + u];
              hdr[e][u] = reinterpret_cast<const uint16_t*>(blk)[d0 + u];
            }
          }
          // the digits before the end in its block: lane j counts [16 j, 16 j + 16)
          const uint32_t j0 = 16 * lane;
          if (j0 < k) {
            uint32_t w[8];
            if (bits > 8) {
              const uint4* q = reinterpret_cast<const uint4*>(blk + 2 * R) + 2 * lane;
              const uint4 x0 = q[0], x1 = q[1];
              w[0] = x0.x; w[1] = x0.y; w[2] = x0.z; w[3] = x0.w;
              w[4] = x1.x; w[5] = x1.y; w[6] = x1.z; w[7] = x1.w;
            } else {
              const uint4 x0 = reinterpret_cast<const uint4*>(blk + 2 * R)[lane];
              w[0] = x0.x; w[1] = x0.y; w[2] = x0.z; w[3] = x0.w;
              w[4] = w[5] = w[6] = w[7] = 0;
            }
#pragma unroll
            for (uint32_t j = 0; j < 16; ++j) {
              const uint32_t dig = bits > 8 ? (w[j >> 1] >> (16 * (j & 1))) & 0xFFFFu
                                            : (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
              if (j0 + j < k) atomicAdd(&s_hist[wv][e][dig], 1u);
            }
          }
        }
      }
      __syncthreads();
      uint64_t ra[8], rb[8];
      uint32_t nchild = 0;
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        const bool on = node && lane_on && u < per;
        ra[u] = on ? sbv[0][u] + hdr[0][u] + s_hist[wv][0][d0 + u] : 0;
        rb[u] = on ? sbv[1][u] + hdr[1][u] + s_hist[wv][1][d0 + u] : 0;
        nchild += (on && rb[u] >= ra[u] + min_count) ? 1u : 0u;
      }
      // the node's children in digit order (wave scan), the nodes in wave order
      uint32_t inc = nchild;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
      }
      if (lane == 63) s_cnt[wv] = inc;
      __syncthreads();
      uint64_t pos = out + inc - nchild, all = 0;
#pragma unroll
      for (uint32_t w = 0; w < kDistWaves; ++w) {
        const uint32_t cw = s_cnt[w];
        pos += w < wv ? cw : 0u;
        all += cw;
      }
#pragma unroll
      for (uint32_t u = 0; u < 8; ++u) {
        const bool on = node && lane_on && u < per;
        if (on && rb[u] >= ra[u] + min_count) {
          if (pos < cap) {
            const uint64_t z = L.Z[d0 + u];
            blo[pos] = z + ra[u];
            bhi[pos] = z + rb[u];
            bpre[pos] = (p << bits) | (d0 + u);
          }
          ++pos;
        }
      }
      out += all;
      __syncthreads();   // s_hist / s_cnt are reused by the next nodes
    }
    if (out > cap) {
      overflow = true;
      break;
    }
    fc = out;
    uint64_t* t;
    uint32_t* tp;
    t = alo; alo = blo; blo = t;
    t = ahi; ahi = bhi; bhi = t;
    tp = apre; apre = bpre; bpre = tp;
    __threadfence_block();
    __syncthreads();   // this level's frontier writes before the next level reads them
  }
  if (overflow) {
    if (threadIdx.x == 0) k_out[row] = ~0ull;
    return;
  }
  for (uint64_t i = threadIdx.x; i < fc; i += 256) {
    syms[base + i] = apre[i];
    counts[base + i] = ahi[i] - alo[i];
    if (child_lo) child_lo[base + i] = (uint64_t)((int64_t)alo[i] + v.D2[apre[i]]);
  }
  if (threadIdx.x == 0) k_out[row] = fc;
}

// interval_symbols of a cached range or the full range (k_distinct leaves these rows to it):
// its symbols are the set bits of its cached bitmap, already in ascending
// order, and the count of symbol c is the width of the child range the
// transition table holds for (range, c) -- or, for a key the table left out,
// the width of the wavelet-matrix descent of both ends.  A row is split over
// kDcChunks workgroups of 256 words (8192 symbols); a workgroup's output
// offset is the popcount of the bitmap words before its chunk.  Only for
// min_count == 1 with a transition table (not while the table is being built).
constexpr uint32_t kDcWords = 256;

// the child of (lo, hi) by symbol c: a scan of its candidate slots from
// candidate d0 on (the caller has checked the others)
__device__ __forceinline__ void child_of(const DevView& v, uint64_t pid, uint64_t lo, uint64_t hi, uint32_t c,
                                         uint32_t d0, uint64_t& clo, uint64_t& cnt) {
  const uint64_t key = trans_key(pid, c);
  const TransHome th = trans_home(lo, hi, c, v.trans_cap);
  for (uint32_t d = d0; d < kTransProbe && pid < kTPidNone && c < kTSymLimit; ++d) {
    const uint64_t slot = trans_slot(th, d);
    const uint64_t w0 = v.trans_tab[2 * slot], w1 = v.trans_tab[2 * slot + 1];
    if (trans_match(w0, key)) {
      clo = trans_clo(w0, w1);
      cnt = trans_cw(w1);
      return;
    }
    // a bucket fills from its first slot and is never emptied: an empty slot ends it
    if (w0 == kTransEmpty) {
      if (d >= kTransBucket) break;
      d = kTransBucket - 1;
    }
  }
  uint64_t pl = lo, pr = hi;           // a key the table left out: the descent
  descend_w2_thread(v, c, pl, pr);
  clo = pl;
  cnt = pr - pl;
}

__global__ void __launch_bounds__(256) k_distinct_cached(DevView v, const uint64_t* __restrict__ lo_a,
                                                        const uint64_t* __restrict__ hi_a, uint64_t m,
                                                        const uint64_t* __restrict__ cap_off,
                                                        uint64_t* __restrict__ syms, uint64_t* __restrict__ counts,
                                                        uint64_t* __restrict__ k_out,
                                                        uint64_t* __restrict__ child_lo, uint32_t chunks) {
  __shared__ uint32_t wave_tot[4];
  const uint64_t row = blockIdx.x / chunks;
  const uint32_t ch = blockIdx.x % chunks;
  if (row >= m) return;
  uint64_t lo = lo_a[row], hi = hi_a[row];
  if (lo == hi || cap_off[row + 1] == cap_off[row]) return;
  if (hi > v.n) hi = v.n;
  if (lo >= hi) return;
  // the same test as k_distinct's (workgroup-uniform); the full range's bitmap
  // is bm_full and its counts come from C
  const bool fullr = lo == 0 && hi == v.n;
  const uint32_t* bm = fullr ? v.bm_full : cache_find(v, lo, hi);
  if (!bm) return;
  // the range's cache id: the key of its transition slots
  const uint64_t pid = fullr ? kTPidNone : (uint64_t)(bm - v.cache_bm) / v.bm_words;
  const uint64_t base = cap_off[row];
  const uint64_t cap = cap_off[row + 1] - base;
  const uint32_t W = v.bm_words;
  const uint32_t w0 = ch * kDcWords;
  // the row's total and this chunk's output offset (set bits before it); every
  // chunk needs the total: a row over capacity reports k = ~0 and stores
  // nothing (k_distinct's contract, fmidx.h fm_distinct_count_batch)
  uint32_t pre = 0, mine = 0;
  const uint32_t lim = min(w0, W);
  for (uint32_t w = threadIdx.x; w < W; w += 256) {
    const uint32_t c = __popc(bm[w]);
    mine += c;
    pre += w < lim ? c : 0u;
  }
  uint32_t all, before;
  (void)block_scan_u32(mine, wave_tot, all);
  (void)block_scan_u32(pre, wave_tot, before);
  if (ch == 0 && threadIdx.x == 0) k_out[row] = all <= cap ? all : ~0ull;
  if (all > cap) return;                     // workgroup-uniform
  const uint32_t wi = w0 + threadIdx.x;
  const uint32_t word = wi < W ? bm[wi] : 0u;
  uint32_t tot;
  uint64_t pos = base + before + block_scan_u32((uint32_t)__popc(word), wave_tot, tot);
  uint32_t rest = word;
  while (rest) {
    // up to 4 symbols' probes issued together (child_of is inlined per symbol)
    uint32_t cs[4];
    int nb = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (rest) {
        cs[u] = wi * 32u + (uint32_t)(__ffs(rest) - 1);
        rest &= rest - 1;
        nb = u + 1;
      } else {
        cs[u] = 0;
      }
    }
    // the first slot of both buckets of every symbol, issued together
    uint64_t q[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool pr = !fullr && u < nb;
      const TransHome th = pr ? trans_home(lo, hi, cs[u], v.trans_cap) : TransHome{0, 0};
      const uint64_t a = th.a, b = th.b;
      const uint64_t* tt = pr ? v.trans_tab : v.C;   // C[0..1]: a valid dummy address
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        q[u][w] = tt[2 * a + w];
        q[u][2 + w] = tt[2 * b + w];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u < nb) {
        uint64_t clo, cnt;
        if (fullr) {
          clo = v.C[cs[u]];
          cnt = v.C[cs[u] + 1] - clo;
        } else {
          const bool keyed = pid < kTPidNone && cs[u] < kTSymLimit;
          const uint64_t key = trans_key(pid, cs[u]);
          if (keyed && trans_match(q[u][0], key)) {
            clo = trans_clo(q[u][0], q[u][1]);
            cnt = trans_cw(q[u][1]);
          } else if (keyed && trans_match(q[u][2], key)) {
            clo = trans_clo(q[u][2], q[u][3]);
            cnt = trans_cw(q[u][3]);
          } else if (!keyed || (q[u][0] == kTransEmpty && q[u][2] == kTransEmpty)) {
            uint64_t pl = lo, pr2 = hi;    // not in the table (left out): the descent
            descend_w2_thread(v, cs[u], pl, pr2);
            clo = pl;
            cnt = pr2 - pl;
          } else {
            child_of(v, pid, lo, hi, cs[u], 0, clo, cnt);
          }
        }
        if (pos - base < cap) {
          syms[pos] = cs[u];
          counts[pos] = cnt;
          if (child_lo) child_lo[pos] = clo;
        }
        ++pos;
      }
    }
  }
}

// Dense CSR of k_distinct's output for the host API: off[i] = sum of k[< i]
// (an overflowed row, k = ~0, contributes 0), then pairs[2 (off[i] + j)] =
// (symbol, count) -- the interleaved layout of fm_index.cpp:136-143.  One
// workgroup scans k (m is a host batch, thousands of rows at most).
__global__ void __launch_bounds__(1024) k_csr_offsets(const uint64_t* __restrict__ k, uint64_t m,
                                                      uint64_t* __restrict__ off) {
  __shared__ uint64_t part[1024];
  const uint64_t per = (m + 1023) / 1024;
  const uint64_t a = threadIdx.x * per, b = a + per < m ? a + per : m;
  uint64_t s = 0;
  for (uint64_t i = a; i < b; ++i) s += k[i] == ~0ull ? 0 : k[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {   // inclusive Hillis-Steele scan
    const uint64_t y = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += y;
    __syncthreads();
  }
  uint64_t acc = part[threadIdx.x] - s;
  for (uint64_t i = a; i < b; ++i) {
    off[i] = acc;
    acc += k[i] == ~0ull ? 0 : k[i];
  }
  if (threadIdx.x == 1023) off[m] = part[1023];
}

__global__ void __launch_bounds__(256) k_csr_pairs(const uint64_t* __restrict__ k, const uint64_t* __restrict__ cap_off,
                                                   const uint64_t* __restrict__ syms,
                                                   const uint64_t* __restrict__ counts,
                                                   const uint64_t* __restrict__ off, uint64_t* __restrict__ pairs) {
  const uint64_t row = blockIdx.x;
  const uint64_t kk = k[row] == ~0ull ? 0 : k[row];
  const uint64_t src = cap_off[row], dst = 2 * off[row];
  for (uint64_t j = threadIdx.x; j < kk; j += 256) {
    pairs[dst + 2 * j] = syms[src + j];
    pairs[dst + 2 * j + 1] = counts[src + j];
  }
}

// LF / search launch variants, from the process tuning (fm_tuning / fm_set_tuning;
// tests select every variant in one process that way).
//  * lanes per row: 64 (one wave per row) while the rows fit the chip's wave
//    slots (latency: no row waits behind another's wide step), else
//    lf_group lanes (default 2; 64 = never group) above
//    lf_group_min rows (default 8192 = 256 CUs x 32 waves).  Measured on
//    the C3 index (tools/probe_rank.py, 2^19 pairs, cold): one wave per row
//    308 us, G = 16 / 8 / 4 / 2 / 1: 179 / 125 / 99 / 90 / 100 us; get_range of
//    2^18 patterns 2658 us -> 539 us at G = 2.
//  * search_group (default 1): the same for get_range launches
//    (k_search_group).  Since the wave-packed E scan (round 3), 2^18 patterns
//    on the C3 index take 364 / 416 / 527 us cold at G = 1 / 2 / 4 (the LF
//    step kernel: 79.2 / 77.3 / 79.4 us), so get_range groups one lane per row.
//  * search_p8 (default 1): get_range at one lane per row probes its
//    cached wide rows eight per round trip (group_step<P8>, LDS-staged runs,
//    123 VGPRs under a 4-wave cap) before the one-at-a-time loop: 2^18
//    patterns 314-316 vs 367-374 us cold.  (The same stage in place of the
//    four-row one of G = 2 LF launches measured no better: 75-87 vs 72-75 us.)
//  * lf_gprobe (default 1): grouped launches with G >= 4 probe the
//    transition table inside the group, so a cached range's hit needs no
//    wave-wide step.
//  * lf_quad (default 1): G = 2 LF launches settle wide rows four at a
//    time (16 lanes each: a probe or a <= 128-row E scan) before the serial
//    loop: 2^19 cold pairs 87 vs 93 us.  Not in k_search_group, where the extra
//    registers (155 VGPRs: 3 waves per SIMD) cost more than it saves (565 vs
//    548 us).
//  * lf_split (default 0): 1 runs a G = 2 LF launch as two passes,
//    k_lf_cheap (every row but the wide ones: 36 VGPRs, 8 waves per SIMD) then
//    k_lf_wide (the wide rows only).  Exact, but slower at C3: 2^19 cold pairs
//    98.4 vs 76.0 us (the second pass still steps wide rows a few per wave).
//  * lf_work: 0 = the grouped kernel only, 1 / 2 = the worklist sweeps
//    above (k_lf_sweep + k_lf_tail, or tail rows in-wave); -1 = chosen by
//    the launch's row count: the in-wave sweep from lf_sweep_min rows
//    (default 2^18), the grouped kernel below.  Measured on the C3 index, cold
//    / warm us (profiles/r03_rank/worklist/): 2^19 pairs 71.8 / 60.9 grouped vs
//    76.6 / 47.7 in-wave; 2^20 126.6 / 109.5 vs 123.0 / 77.6; 2^21 216.4 / 202.4
//    vs 177.6 / 140.2; round 5, after an eviction that leaves no dirty lines
//    (profiles/r05_rank_temp/): 2^19 72.9 / 63.7 vs 63.1 / 51.5, 2^21 207.3 /
//    205.3 vs 142.8 / 140.5; with its tail rows rewritten (packed E scans,
//    settled misses, quarter-wave descents; profiles/r05_tails/rank_by_launch_size.json)
//    2^17 36.0 / 31.0 vs 44.7 / 30.3, 2^18 57.9 / 44.0 vs 50.2 / 36.9, 2^19 73.0 /
//    63.1 vs 57.6 / 48.4, 2^20 116.8 / 112.1 vs 79.8 / 72.0 -- the sweep from 2^18 rows.
struct LfTuning {
  uint32_t G;
  uint32_t Gs;   // get_range
  uint64_t min_rows;
  bool gprobe;
  bool quad;
  bool split;
  bool work;          // worklist sweeps (k_lf_sweep + k_lf_tail) when a workspace is given
  bool work_inline;   // k_lf_sweep alone, tail rows stepped in-wave
  bool persist;       // k_lf_persist (lf_work 4) from sweep_min rows, when the API gives its workspace
  uint64_t sweep_min; // work_inline from this many rows (lf_work -1: lf_sweep_min; 2: min_rows)
  bool search_p8;     // get_range at one lane per row probes cached rows eight at a time
};

LfTuning load_lf_tuning() {
  const Tuning& p = tuning();
  LfTuning t;
  const uint32_t g = p.lf_group;
  t.G = (g == 1 || g == 2 || g == 4 || g == 8 || g == 16) ? g : 64u;
  const uint32_t gs = p.search_group;
  t.Gs = (gs == 1 || gs == 2 || gs == 4 || gs == 8 || gs == 16) ? gs : 64u;
  t.min_rows = p.lf_group_min;
  t.gprobe = p.lf_gprobe != 0;
  t.quad = p.lf_quad != 0;
  t.split = p.lf_split != 0;
  const bool autow = p.lf_work < 0;
  t.work = p.lf_work == 1;
  t.persist = p.lf_work == 4;
  t.work_inline = autow || p.lf_work == 2 || t.persist;
  t.sweep_min = (autow || t.persist) ? p.lf_sweep_min : 0;
  t.search_p8 = p.search_p8 != 0;
  return t;
}

LfTuning& lf_tuning() {
  static LfTuning t = load_lf_tuning();
  return t;
}

uint32_t lf_group(uint64_t m) { return m > lf_tuning().min_rows ? lf_tuning().G : 64u; }
uint32_t search_group(uint64_t m) { return m > lf_tuning().min_rows ? lf_tuning().Gs : 64u; }
bool lf_gprobe() { return lf_tuning().gprobe; }
bool lf_quad() { return lf_tuning().quad; }
bool lf_split() { return lf_tuning().split; }
bool lf_work() { return lf_tuning().work; }

// worklist geometry for m rows: entries per region, sweep-1 waves
uint64_t lf_work_cap(uint64_t m) {
  return (((m + kLfThreads - 1) / kLfThreads + kWorkRegions - 1) / kWorkRegions) * kLfThreads;
}

}  // namespace

// ------------------------------------------------------------------ launchers
void reload_lf_tuning() { lf_tuning() = load_lf_tuning(); }

size_t lf_ws_bytes(uint64_t m) {
  return m > lf_tuning().min_rows && lf_work() ? kWorkRegions * lf_work_cap(m) * sizeof(LfWork) + kWorkRegions * 4 : 0;
}

int launch_lf_step(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                   const uint64_t* lo, const uint64_t* hi, uint64_t* lo_out, uint64_t* hi_out,
                   uint64_t m, hipStream_t s, void* ws) {
  if (m == 0) return 0;
  if (m > lf_tuning().min_rows && m >= lf_tuning().sweep_min && lf_tuning().work_inline) {
    // one launch, tail rows stepped in-wave
    const unsigned g1 = (unsigned)((m + kLfThreads - 1) / kLfThreads);
    k_lf_sweep<true><<<g1, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m, nullptr,
                                               nullptr, 0);
    FM_HIP(hipGetLastError());
    return 0;
  }
  if (ws && m > lf_tuning().min_rows && lf_work()) {
    const uint64_t cap = lf_work_cap(m);
    LfWork* lt = reinterpret_cast<LfWork*>(ws);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(lt + kWorkRegions * cap);
    FM_HIP(hipMemsetAsync(cnt, 0, kWorkRegions * 4, s));
    const unsigned g1 = (unsigned)((m + kLfThreads - 1) / kLfThreads);
    k_lf_sweep<false><<<g1, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m, lt, cnt, cap);
    // persistent: at most 8192 waves (the chip's slots at 8 waves per SIMD),
    // no more per region than its worst-case row count
    const uint32_t q = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(8192 / kWorkRegions, cap));
    k_lf_tail<<<q * kWorkRegions / (kLfThreads / 64), kLfThreads, 0, s>>>(v, lt, cnt, cap, lo_out, hi_out, q);
    FM_HIP(hipGetLastError());
    return 0;
  }
  const uint32_t G = lf_group(m);
  const unsigned g = (unsigned)(((m + 64 / G - 1) / (64 / G) * 64 + kLfThreads - 1) / kLfThreads);
  if (G == 2 && lf_split()) {
    k_lf_cheap<2><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
    if (lf_quad())
      k_lf_wide<2, true><<<g, kLfThreads, 0, s>>>(v, tok, shift, lo_out, hi_out, m);
    else
      k_lf_wide<2, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, lo_out, hi_out, m);
  } else if (G == 1)
    k_lf_group<1, false, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else if (G == 2 && lf_quad())
    k_lf_group<2, false, true><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else if (G == 2)
    k_lf_group<2, false, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else if (G == 4 && lf_gprobe())
    k_lf_group<4, true, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else if (G == 4)
    k_lf_group<4, false, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else if (G == 8 && lf_gprobe())
    k_lf_group<8, true, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else if (G == 8)
    k_lf_group<8, false, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else if (G == 16)
    k_lf_group<16, false, false><<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  else
    k_lf<<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m);
  FM_HIP(hipGetLastError());
  return 0;
}

bool lf_persist(uint64_t m) {
  return lf_tuning().persist && m > lf_tuning().min_rows && m >= lf_tuning().sweep_min && m < (1ull << 28);
}

// the persistent sweep's workspace: [counters: 2 sets][err word, its own line][tail queues][tags]
static uint64_t lf_persist_qcap(uint64_t m) { return 64 * ((((m + 63) / 64) + kPParts - 1) / kPParts); }

size_t lf_persist_ws_bytes(uint64_t m) {
  const uint64_t qcap = lf_persist_qcap(m);
  return (size_t)2 * kPSetWords * 4 + 128 + (size_t)kPParts * qcap * (sizeof(LfWork) + 4);
}

// the grid: the resident workgroups (every wave a head worker, then a drainer)
static unsigned lf_persist_grid(int dev) {
  static unsigned cached[64] = {};
  if (dev >= 0 && dev < 64 && cached[dev]) return cached[dev];
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lf_persist, kLfThreads, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  constexpr unsigned kBlk = kPParts / (kLfThreads / 64);   // waves a multiple of kPParts: wave w's chunks
  unsigned g = (unsigned)per_cu * (unsigned)cus;          // all in queue w mod kPParts
  g = std::max(kBlk, g / kBlk * kBlk);
  if (dev >= 0 && dev < 64) cached[dev] = g;
  return g;
}

int launch_lf_persist(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below, const uint64_t* lo,
                      const uint64_t* hi, uint64_t* lo_out, uint64_t* hi_out, uint64_t m, hipStream_t s, void* ws,
                      size_t ws_bytes, uint32_t epoch, int dev) {
  if (m == 0) return 0;
  const uint64_t qcap = lf_persist_qcap(m);
  if (!ws || ws_bytes < lf_persist_ws_bytes(m) || qcap * sizeof(LfWork) >= (1ull << 32) || epoch == 0) {
    set_error("lf persist: workspace of %llu bytes, %llu needed", (unsigned long long)ws_bytes,
              (unsigned long long)lf_persist_ws_bytes(m));
    return -1;
  }
  char* b = static_cast<char*>(ws);
  PersistWs w;
  w.ctr = reinterpret_cast<uint32_t*>(b);
  w.err = reinterpret_cast<uint32_t*>(b + 2 * kPSetWords * 4);
  w.tq = reinterpret_cast<LfWork*>(b + 2 * kPSetWords * 4 + 128);
  w.tag = reinterpret_cast<uint32_t*>(w.tq + kPParts * qcap);
  const uint64_t nchunks = (m + 63) / 64;
  constexpr uint64_t kBlk = kPParts / (kLfThreads / 64);
  const unsigned g = (unsigned)std::min<uint64_t>(lf_persist_grid(dev), (nchunks + 4 * kBlk - 1) / (4 * kBlk) * kBlk);
  k_lf_persist<<<g, kLfThreads, 0, s>>>(v, tok, shift, reset_below, lo, hi, lo_out, hi_out, m, w,
                                                               (uint32_t)qcap, epoch);
  FM_HIP(hipGetLastError());
  return 0;
}

size_t lf_persist_err_offset() { return 2 * kPSetWords * 4; }

int launch_search(const DevView& v, const int64_t* tok, const int64_t* off, uint64_t m,
                  int64_t shift, const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out,
                  uint64_t* hi_out, hipStream_t s) {
  if (m == 0) return 0;
  const uint32_t G = search_group(m);
  const unsigned g = (unsigned)(((m + 64 / G - 1) / (64 / G) * 64 + kLfThreads - 1) / kLfThreads);
  if (G == 1 && lf_tuning().search_p8)
    k_search_group<1, false, false, true><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out,
                                                                    hi_out);
  else if (G == 1)
    k_search_group<1, false, false><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  else if (G == 2)
    k_search_group<2, false, false><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  else if (G == 4 && lf_gprobe())
    k_search_group<4, true, false><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  else if (G == 4)
    k_search_group<4, false, false><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  else if (G == 8 && lf_gprobe())
    k_search_group<8, true, false><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  else if (G == 8)
    k_search_group<8, false, false><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  else if (G == 16)
    k_search_group<16, false, false><<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  else
    k_search<<<g, kLfThreads, 0, s>>>(v, tok, off, m, shift, lo_in, hi_in, lo_out, hi_out);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_step_raw(const DevView& v, uint64_t sym, uint64_t low, uint64_t high, uint64_t* out2,
                    hipStream_t s) {
  k_step_raw<<<1, 64, 0, s>>>(v, sym, low, high, out2);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_raw_multi(const DevView& v, const uint64_t* q, uint64_t len, uint64_t* out2,
                     hipStream_t s) {
  k_raw_multi<<<1, 64, 0, s>>>(v, q, len, out2);
  FM_HIP(hipGetLastError());
  return 0;
}

size_t distinct_ws_bytes(uint64_t total_cap) { return (size_t)total_cap * 40 + 256; }

int launch_distinct(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                    const uint64_t* cap_off, uint64_t* syms, uint64_t* counts, uint64_t* k,
                    void* ws, uint64_t total_cap, hipStream_t s, uint64_t min_count, uint64_t* child_lo) {
  if (m == 0) return 0;
  Frontier fr;
  char* p = reinterpret_cast<char*>(ws);
  const uint64_t T = total_cap ? total_cap : 1;
  fr.lo[0] = reinterpret_cast<uint64_t*>(p);
  fr.hi[0] = fr.lo[0] + T;
  fr.lo[1] = fr.hi[0] + T;
  fr.hi[1] = fr.lo[1] + T;
  fr.pre[0] = reinterpret_cast<uint32_t*>(fr.hi[1] + T);
  fr.pre[1] = fr.pre[0] + T;
#ifndef FMIDX_DISTINCT_CACHED
#define FMIDX_DISTINCT_CACHED 1   // measurement variant: 0 = every range through the BFS
#endif
  const bool cached_path = v.trans_cap && v.cache_mask && (min_count ? min_count : 1) == 1 &&
                           FMIDX_DISTINCT_CACHED != 0;
  k_distinct<<<(unsigned)m, 256, 0, s>>>(v, lo, hi, m, cap_off, syms, counts, k, fr,
                                         min_count ? min_count : 1, child_lo, cached_path);
  FM_HIP(hipGetLastError());
  if (cached_path) {
    const uint32_t chunks = (v.bm_words + kDcWords - 1) / kDcWords;
    k_distinct_cached<<<(unsigned)(m * chunks), 256, 0, s>>>(v, lo, hi, m, cap_off, syms, counts, k, child_lo,
                                                             chunks);
    FM_HIP(hipGetLastError());
  }
  return 0;
}

int launch_distinct_csr(const uint64_t* k, const uint64_t* cap_off, const uint64_t* syms, const uint64_t* counts,
                        uint64_t m, uint64_t* off, uint64_t* pairs, hipStream_t s) {
  if (m == 0) return 0;
  k_csr_offsets<<<1, 1024, 0, s>>>(k, m, off);
  k_csr_pairs<<<(unsigned)m, 256, 0, s>>>(k, cap_off, syms, counts, off, pairs);
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
