// decode.hip -- the hot path: allowed-next-token masks, fused with the LF step.
//
// One decode step of the reference processors for every row b (SURVEY §8a
// A2-A8): the backward-search step of the row's range by its new token
// (index.py:109-112 -> fm_index.cpp:67-97), then
//     allowed[b, t] = 1  <=>  t + shift occurs in BWT[lo_b, hi_b)
// -- the boolean core of get_distinct_count_multi (fm_index.cpp:146-166 +
// index.py:161-174, sentinel dropped) that the processors scatter into their
// score masks (document_constrained_generation_causal_qwen.py:185-204).
//
// Geometry (gfx950): one workgroup of kDecThreads threads per (row, vocab
// slice): 1024 (16 waves) and 1 slice per row at B = 256 (measured best at
// C3: 11.7 us/step vs 12.1 for 256 x 4 slices and 13.1 for 512 x 2); 512 or
// 256 threads for larger batches (decode_threads).
//   wave 0        LF step (one round trip for every kind of range: C lookup,
//                 E scan, transition-table probe of a cached range; the
//                 two-level descent only for ranges none of those serves),
//                 then the read plan of the new range
//   all waves     the E scan of an uncached 513..4096-row range
//   waves 1..15   rows whose incoming range is already narrow stay narrow
//                 after the step, so their mask row is zero-filled right away,
//                 overlapping the LF chain
//   all waves     partial ends of the range streamed from the plain BWT into
//                 LDS bits (LDS atomics), whole-block bitmaps ORed in
//   all waves     emit: 16 tokens per lane per store, consecutive lanes on
//                 consecutive 16-B chunks (a wave writes 1 KB contiguous)
#include "fmidx_internal.h"

#include <algorithm>
#include <cstdlib>

namespace fmidx {

namespace {

#ifndef FMIDX_STORE_AUX
#define FMIDX_STORE_AUX 16
#endif
// cache policy of the mask stores (buffer-store aux bits): 16 = sc1, i.e.
// write-through -- the 33 MB of mask a step writes leaves no dirty L2 lines
// for the kernel-end writeback to flush (MI355X_MICROARCH.md "boundary":
// + bytes / 6 TB/s behind a predecessor that leaves bytes dirty); 0 = plain.
constexpr int kStoreAux = FMIDX_STORE_AUX;
#ifndef FMIDX_LATE_AUX
#define FMIDX_LATE_AUX FMIDX_STORE_AUX
#endif
// cache policy of the final emit of rows NOT zero-filled early (the wide rows
// that end the step): a lone CU writes a 128-KB row in 1.0 us with plain
// stores and 1.5 us write-through (tools/micro/cu_store.hip), but the dirty
// lines then cost the kernel end more: C3 cold / warm 13.9 / 10.6 us with
// plain late stores, 14.0 / 11.8 with plain stores everywhere, against 13.5 /
// 9.9 write-through (profiles/r03_latency/store_policy.log)
constexpr int kLateAux = FMIDX_LATE_AUX;
constexpr int kMaxPlan = 160;                 // >= 6 * kMaxBmLevels
constexpr uint32_t kMaxSliceTokens = 262144;  // 32 KB of LDS bits
// LDS window words for a slice of sw tokens: the window starts at most 127
// symbols before the slice (128-bit aligned) and ends 64 after it
__host__ __device__ constexpr uint32_t win_words(uint64_t sw) { return (uint32_t)(sw / 32 + 16); }
#ifndef FMIDX_EARLY_ZERO_WIDTH
#define FMIDX_EARLY_ZERO_WIDTH 64   // measurement variant (make variant VFLAGS=-DFMIDX_EARLY_ZERO_WIDTH=512)
#endif
constexpr uint64_t kEarlyZeroWidth = FMIDX_EARLY_ZERO_WIDTH;   // rows this narrow get their zeros written up front
#ifndef FMIDX_EZ_SLEEP
#define FMIDX_EZ_SLEEP 0   // measurement variant: s_sleep (x 64 clocks) between a thread's early zero stores
#endif
constexpr int kEzSleep = FMIDX_EZ_SLEEP;
constexpr int kUnroll = 4;                    // uint4 loads in flight per thread while streaming
constexpr uint32_t kPayMagic = 0x58534D46u;    // the shard payload's magic (csrc/shard.hip)
constexpr uint32_t kPayMaxWords = 8192;        // W of a payload row: vocab <= 262144

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup
// release/acquire, which on gfx950 also drains every wave's outstanding
// global stores (s_waitcnt vmcnt(0)) -- measured as several us behind the
// early zero-fill of the mask rows.  Nothing crossing these barriers is
// global data, so only LDS (lgkmcnt) is drained.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct Plan {
  uint64_t a0, b0, a1, b1;            // streamed BWT row ranges (partial ends / narrow range)
  uint32_t nb;                        // bitmaps to OR
  const uint32_t* ptr[kMaxPlan];      // those bitmaps
};

// Canonical decomposition of [lo, hi) into two streamed partial ends plus the
// maximal aligned bitmap blocks (B0*4^j rows at level j), computed by wave 0
// with one lane per bitmap level: with a_j / b_j = x / y rounded up / down to
// level-j alignment and `top` the highest level holding a whole block, level
// j < top contributes [a_j, a_{j+1}) and [b_{j+1}, b_j), level top [a_top,
// b_top) -- the same set the greedy left-to-right cover produces (<= 6 per level).
__device__ void plan_range_wave(const DevView& v, uint64_t lo, uint64_t hi, int64_t follow, Plan& p) {
  const uint32_t lane = threadIdx.x;   // called by the 64 lanes of wave 0
  const uint32_t* one = nullptr;
  if (lo == 0 && hi == v.n && v.bm_full)
    one = v.bm_full;                                    // the whole BWT
  else if (follow >= 0 && v.bm_follow)
    one = v.bm_follow + (uint64_t)follow * v.bm_words;  // C-block of symbol `follow`
  if (one) {                                            // one precomputed bitmap
    if (lane == 0) {
      p.nb = 1;
      p.ptr[0] = one;
      p.a0 = p.b0 = p.a1 = p.b1 = 0;
    }
    return;
  }
  const uint32_t lg = v.bm_log2;
  const uint64_t B0 = 1ull << lg;
  bool split = v.bm_levels > 0 && hi - lo > B0;
  uint64_t x = 0, y = 0;
  if (split) {
    x = (lo + B0 - 1) >> lg;
    y = hi >> lg;
    split = x < y;
  }
  if (lane == 0) {
    p.nb = 0;
    p.a0 = lo;
    p.b0 = split ? (x << lg) : hi;
    p.a1 = split ? (y << lg) : 0;
    p.b1 = split ? hi : 0;
  }
  if (!split) return;
  const uint32_t J = v.bm_levels;
  const uint32_t j = lane;
  uint64_t aj = 0, bj = 0, aj1 = 0, bj1 = 0;
  bool valid = false;
  if (j < J) {
    const uint64_t s0 = 1ull << (2 * j), s1 = 1ull << (2 * (j + 1));
    aj = (x + s0 - 1) & ~(s0 - 1);
    bj = y & ~(s0 - 1);
    aj1 = (x + s1 - 1) & ~(s1 - 1);
    bj1 = y & ~(s1 - 1);
    valid = aj < bj;
  }
  const uint64_t vb = __ballot(valid);
  const uint32_t top = 63u - (uint32_t)__clzll(vb);
  uint32_t cnt = 0;
  if (j < top)
    cnt = (uint32_t)(((aj1 - aj) + (bj - bj1)) >> (2 * j));
  else if (j == top)
    cnt = (uint32_t)((bj - aj) >> (2 * j));
  uint32_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += t;
  }
  const uint32_t start = incl - cnt;
  if (cnt) {
    uint64_t off = 0;
    for (uint32_t i = 0; i < j; ++i) off += (v.bm_count[0] >> (2 * i)) * (uint64_t)v.bm_words;
    const uint64_t s0 = 1ull << (2 * j);
    uint32_t k = start;
    if (j < top) {
      for (uint64_t pos = aj; pos < aj1; pos += s0) p.ptr[k++] = v.bm + off + (pos >> (2 * j)) * v.bm_words;
      for (uint64_t pos = bj1; pos < bj; pos += s0) p.ptr[k++] = v.bm + off + (pos >> (2 * j)) * v.bm_words;
    } else {
      for (uint64_t pos = aj; pos < bj; pos += s0) p.ptr[k++] = v.bm + off + (pos >> (2 * j)) * v.bm_words;
    }
  }
  if (j == top) p.nb = start + cnt;
}

__device__ __forceinline__ int64_t floor_div32(int64_t x) { return x >= 0 ? x / 32 : -((-x + 31) / 32); }

__device__ __forceinline__ void set_bit(uint32_t* win, uint32_t sym, int64_t base_bit, int64_t lim) {
  const int64_t rel = (int64_t)sym - base_bit;
  if (rel >= 0 && rel < lim) atomicOr(&win[rel >> 5], 1u << (rel & 31));
}

// Streamed parts of a range: BWT[a0, b0) and BWT[a1, b1).  Each part is an
// unaligned head (< 4 symbols), a 16-B aligned middle read as uint4, and an
// unaligned tail.  The first round's loads -- every head/tail symbol (threads
// 0..11) and kUnroll uint4 per thread of the concatenated middles -- are all
// issued before any is consumed, so a partial end of up to 16K symbols costs
// one memory round trip.  Everything is computed in registers: an aggregate
// selected with a lane-varying index lands in scratch, and a scratch store +
// load ahead of the first BWT load adds a round trip (plus the store's
// acknowledgement, shared vmcnt) to the chain.

// the aligned middle of [a, b) as uint4 indices [q, q + nq)
__device__ __forceinline__ void middle_of(uint64_t a, uint64_t b, uint64_t& q, uint64_t& nq) {
  const uint64_t a4 = (a + 3) & ~3ull, b4 = b & ~3ull;
  const bool has = a < b && a4 < b4;
  q = has ? a4 / 4 : 0;
  nq = has ? (b4 - a4) / 4 : 0;
}

// head (tail = false) or tail piece of [a, b): start position and length (0..3)
__device__ __forceinline__ void piece_of(uint64_t a, uint64_t b, bool tail, uint64_t& pos, uint32_t& len) {
  pos = 0;
  len = 0;
  if (a >= b) return;
  const uint64_t a4 = (a + 3) & ~3ull, b4 = b & ~3ull;
  if (a4 >= b4) {            // fewer than one aligned uint4: up to 6 symbols as head + tail
    const uint32_t hl = (uint32_t)min((uint64_t)3, b - a);
    pos = tail ? a + hl : a;
    len = tail ? (uint32_t)(b - a - hl) : hl;
    return;
  }
  pos = tail ? b4 : a;
  len = tail ? (uint32_t)(b - b4) : (uint32_t)(a4 - a);
}

__device__ __forceinline__ void set_u4(uint32_t* win, const uint4& q, int64_t base_bit, int64_t lim) {
  set_bit(win, q.x, base_bit, lim);
  set_bit(win, q.y, base_bit, lim);
  set_bit(win, q.z, base_bit, lim);
  set_bit(win, q.w, base_bit, lim);
}

// by threads [0, nthr) of the workgroup
__device__ __forceinline__ void stream_symbols(const uint32_t* __restrict__ bwt, uint64_t a0, uint64_t b0,
                                               uint64_t a1, uint64_t b1, int64_t base_bit, int64_t lim,
                                               uint32_t* win, uint32_t nthr) {
  uint64_t q0, n0, q1, n1;
  middle_of(a0, b0, q0, n0);
  middle_of(a1, b1, q1, n1);
  const uint64_t ntot = n0 + n1;
  const uint4* src = reinterpret_cast<const uint4*>(bwt);
  uint32_t hsym = ~0u;          // head/tail symbols: threads 0..11, loaded with the first round
  if (threadIdx.x < 12) {
    const uint32_t pc = threadIdx.x / 3, k = threadIdx.x % 3;
    uint64_t pp;
    uint32_t pl;
    piece_of(pc < 2 ? a0 : a1, pc < 2 ? b0 : b1, (pc & 1) != 0, pp, pl);
    if (k < pl) hsym = bwt[pp + k];
  }
  for (uint64_t base = threadIdx.x; base < ntot; base += (uint64_t)nthr * kUnroll) {
    uint4 q[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      // unconditional load, its result used unconditionally (a surplus lane
      // re-reads element 0 of the middles and ORs in all-ones): a select here
      // let the compiler sink the load into a branch with a vmcnt(0) right
      // after it -- kUnroll round trips instead of one
      const uint64_t j = base + (uint64_t)u * nthr;
      const uint64_t jj = j < ntot ? j : 0;
      const uint4 x = src[jj < n0 ? q0 + jj : q1 + (jj - n0)];
      const uint32_t pad = j < ntot ? 0u : ~0u;
      q[u] = make_uint4(x.x | pad, x.y | pad, x.z | pad, x.w | pad);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      if (q[u].x != ~0u) set_u4(win, q[u], base_bit, lim);
  }
  if (hsym != ~0u) set_bit(win, hsym, base_bit, lim);
}

// The same from E (the plain BWT freed): 16-B loads hold two entries, whose
// symbols are bits 36.. of each; the aligned middle is in entry pairs, the
// head / tail pieces one entry each (threads 0..3).  Same round-trip structure.
__device__ __forceinline__ void stream_symbols_e(const uint64_t* __restrict__ E, uint64_t a0, uint64_t b0,
                                                 uint64_t a1, uint64_t b1, int64_t base_bit, int64_t lim,
                                                 uint32_t* win, uint32_t nthr) {
  auto pairs = [](uint64_t a, uint64_t b, uint64_t& q, uint64_t& nq) {
    const uint64_t a2 = (a + 1) & ~1ull, b2 = b & ~1ull;
    const bool has = a < b && a2 < b2;
    q = has ? a2 / 2 : 0;
    nq = has ? (b2 - a2) / 2 : 0;
  };
  uint64_t q0, n0, q1, n1;
  pairs(a0, b0, q0, n0);
  pairs(a1, b1, q1, n1);
  const uint64_t ntot = n0 + n1;
  const uint4* src = reinterpret_cast<const uint4*>(E);
  uint32_t hsym = ~0u;          // head / tail entries: threads 0..3, loaded with the first round
  if (threadIdx.x < 4) {
    const bool p1 = threadIdx.x >= 2, tail = (threadIdx.x & 1u) != 0;
    const uint64_t a = p1 ? a1 : a0, b = p1 ? b1 : b0;
    uint64_t q, nq;
    pairs(a, b, q, nq);
    uint64_t pos = ~0ull;
    if (a < b) {
      if (nq) pos = tail ? ((b & 1ull) ? b - 1 : ~0ull) : ((a & 1ull) ? a : ~0ull);
      else pos = tail ? (a + 1 < b ? a + 1 : ~0ull) : a;   // no whole pair inside: at most two entries
    }
    if (pos != ~0ull) hsym = (uint32_t)(E[pos] >> kESymShift);
  }
  for (uint64_t base = threadIdx.x; base < ntot; base += (uint64_t)nthr * kUnroll) {
    uint32_t s[kUnroll][2];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      // unconditional load (see stream_symbols): surplus lanes re-read pair 0 and are padded out
      const uint64_t j = base + (uint64_t)u * nthr;
      const uint64_t jj = j < ntot ? j : 0;
      const uint4 x = src[jj < n0 ? q0 + jj : q1 + (jj - n0)];
      const uint32_t pad = j < ntot ? 0u : ~0u;
      s[u][0] = (x.y >> (kESymShift - 32)) | pad;
      s[u][1] = (x.w >> (kESymShift - 32)) | pad;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      if (s[u][0] != ~0u) {
        set_bit(win, s[u][0], base_bit, lim);
        set_bit(win, s[u][1], base_bit, lim);
      }
  }
  if (hsym != ~0u) set_bit(win, hsym, base_bit, lim);
}

// blockIdx -> (row, slice).  Blocks b and b+8 share an XCD under round-robin
// dispatch, so the S slices of a row are given blockIdx values congruent mod 8:
// their redundant reads of the row's rank blocks / BWT / bitmaps share one L2.
// Speed only; any placement is correct.
__device__ __forceinline__ void map_block(uint32_t b, uint32_t S, uint64_t& row, uint32_t& slice) {
  const uint32_t per = 8u * S;
  const uint32_t r = b % per;
  row = (uint64_t)(b / per) * 8 + (r & 7u);
  slice = r >> 3;
}

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// Loads through a bitmap pointer that was handed over in LDS (the plan).  The
// compiler cannot tell such a pointer's address space and emits FLAT loads,
// which count in lgkmcnt as well as vmcnt: the LDS read of the next pointer
// (or any other LDS wait) then drains every earlier load, and a thread's 8-16
// bitmap loads went out one round trip at a time.  As global loads they only
// count in vmcnt and are all in flight together.
typedef const __attribute__((address_space(1))) uint32_t* gptr_u32;
typedef const __attribute__((address_space(1))) v4u* gptr_v4;
__device__ __forceinline__ uint32_t gld(const uint32_t* p, uint32_t i) { return ((gptr_u32)p)[i]; }
__device__ __forceinline__ uint4 gld4(const uint32_t* p, int64_t i) {
  const v4u x = *(gptr_v4)(p + i);
  return make_uint4(x.x, x.y, x.z, x.w);
}




__device__ __forceinline__ void store16(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& x) {
  v4u v = {x.x, x.y, x.z, x.w};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kStoreAux);
}

// the final emit: write-through (kStoreAux) for rows zero-filled early, kLateAux otherwise
__device__ __forceinline__ void store16_emit(__amdgpu_buffer_rsrc_t r, uint32_t off, const uint4& x, bool zeroed) {
  v4u v = {x.x, x.y, x.z, x.w};
  if (kLateAux == kStoreAux || zeroed)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kStoreAux);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kLateAux);
}

// AUX: kStoreAux (sc1, agent-scope write-through) for masks; kPayAux for the peer exchange's payload
template <int AUX = kStoreAux>
__device__ __forceinline__ void store4(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t x) {
  __builtin_amdgcn_raw_buffer_store_b32(x, r, off, 0, AUX);
}

// The peer exchange's payload (PAY) is read by OTHER GPUs over xGMI, straight from this GPU's
// memory (csrc/shard.hip k_or_rows<true>: system-scope loads).  Its stores are system-scope
// write-through (sc0 sc1): every payload byte has left this XCD's L2 when the store is
// acknowledged, so its visibility to a remote reader does not depend on the end-of-kernel
// release (its scope, or which XCDs' L2s it writes back) -- DESIGN.md §5 "Visibility".
constexpr int kPayAux = 1 | 16;
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);   // global_store_dword sc0 sc1
}

// 16 mask bits -> 16 bytes of 0/1
__device__ __forceinline__ uint4 bits16_to_bytes(uint32_t b) {
  uint32_t q[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = (((b >> (4 * j)) & 0xFu) * 0x204081u) & 0x01010101u;
  return make_uint4(q[0], q[1], q[2], q[3]);
}

// One workgroup = one vocab slice of one row.  With DO_LF the row's LF step
// (or restart) is computed first by wave 0 (redundantly per slice; slice 0
// publishes the new state), otherwise [lo_in, hi_in) is the range to mask.
// Mask chunks: CH = 16 tokens (uint8 mask, one uint4 store) or 32 tokens
// (packed, one uint32 store); chunk k of a slice is owned by one thread in
// both the early zero-fill and the final emit.
#ifndef FMIDX_SMALL_WG_WAVES
// waves per SIMD asked of the < 1024-thread variants: 6 fits 80 VGPRs only
// with ~50 B of scratch spills (B = 2048: 46.4 us/step against 48.0), so
// the compiler's own allocation (92 VGPRs, 5 waves) is kept
#define FMIDX_SMALL_WG_WAVES 1
#endif
// PAY (with PACKED and DO_LF, one slice per row): the output is the doc-range
// shards' exchange payload (csrc/shard.hip's layout) with FIXED row slots --
// row b's data at H + b * round4(W) words, W = ceil(vocab / 32) -- so no pack
// pass is needed when the payload is read in place (PeerExchange): a row whose
// new range is streamed whole and narrower than W (every row narrower than W
// when the bitmap blocks and the cache start above W) writes its BWT slice
// (the symbols) and nothing else -- no zero-fill, no bitmap; every other row
// writes its packed bitmap into its slot exactly as PACKED does; the row's
// workgroup writes its desc / off words, row 0's the header.
// The flag barrier's signal fused into the payload decode (PAY with sig.done != null): every
// workgroup, once all its payload stores are acknowledged (system-scope write-through: performed at
// this GPU's memory side), adds one to *sig.done; the workgroup whose add is the grid's last does
// what k_peer_signal (csrc/shard.hip) does as a separate launch -- a system-scope release, the step
// number (*sig.ctr + 1) stored into every rank's flag word for this rank (system-scope stores over
// xGMI), *sig.ctr advanced, *sig.done reset for the next step -- so a flag-barrier step is two
// launches (decode, OR pass), not three.  Every workgroup reads *sig.ctr (the buffer parity)
// before its add, so the advance follows every read of it.
struct PeerSignal {
  const uint64_t* dst;   // [world] the peers' flag-word addresses for this rank
  uint32_t* ctr;         // this rank's device step counter
  uint32_t* done;        // kSigCounters counters, kSigStride words apart (zero between steps)
  uint32_t world;
};
// The count is two-level so that no one word takes every workgroup's add (a word saturates near
// 90 returning atomics per us -- 2048 workgroups on one word cost B = 2048 steps ~13 us): counter r
// (r < 8) counts the workgroups b with b % 8 == r, and the last of each adds to counter 8, whose
// last signals.  Each counter on its own 128-B line.
constexpr uint32_t kSigStride = 32;   // 9 counters: done[0 .. 9 * kSigStride)

// one workgroup's arrival (called by ONE thread, after the workgroup's stores are acknowledged)
__device__ __forceinline__ void peer_signal_arrive(const PeerSignal& sig) {
  const uint32_t b = blockIdx.x, g = gridDim.x, r = b & 7u;
  const uint32_t in_r = (g - r + 7u) / 8u;                 // workgroups with residue r
  uint32_t* cr = sig.done + r * kSigStride;
  if (__hip_atomic_fetch_add(cr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != in_r - 1u) return;
  __hip_atomic_store(cr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // every one of them has added
  uint32_t* top = sig.done + 8u * kSigStride;
  const uint32_t groups = g < 8u ? g : 8u;
  if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != groups - 1u) return;
  __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t value = __hip_atomic_load(sig.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  for (uint32_t k = 0; k < sig.world; ++k)
    __hip_atomic_store(reinterpret_cast<uint32_t*>(sig.dst[k]), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(sig.ctr, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void peer_signal_done(const PeerSignal& sig) {
  // every wave's stores acknowledged, then one arrival per workgroup (all waves reach this point:
  // the callers' exits are workgroup-uniform)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) peer_signal_arrive(sig);
}

// The row-state pointers: __restrict__ (never aliased: the uint8 / packed launches refuse in-place
// state) except in the payload variant, whose flag-barrier step updates the state IN PLACE.  There
// every wave consumes its state load (the early-zero / wg_scan decisions) before the plan barrier,
// and thread 0 stores the new state after it (see the store below).
template <bool PAY> struct StatePtr {
  typedef const uint64_t* __restrict__ in;
  typedef uint64_t* __restrict__ out;
};
template <> struct StatePtr<true> {
  typedef const uint64_t* in;
  typedef uint64_t* out;
};

template <bool PACKED, bool DO_LF, int kDecThreads, bool PAY = false>
// Argument order: the per-row state pointers and the slice geometry come first
// so that, with kernel-argument preloading (Makefile: -amdgpu-kernarg-preload-
// count), they arrive in SGPRs at dispatch and the row-state loads issue
// before any kernel-argument memory load; the large DevView comes last.
// (PAY updates the state in place -- lo_in == lo_out -- so its state pointers carry no
// __restrict__: StateIn / StateOut below.)
__global__ void __launch_bounds__(kDecThreads, kDecThreads >= 1024 ? 1 : FMIDX_SMALL_WG_WAVES) k_decode(const int64_t* __restrict__ tok,
                                                       typename StatePtr<PAY>::in lo_in,
                                                       typename StatePtr<PAY>::in hi_in, uint64_t m,
                                                       uint32_t S, uint32_t SW, uint64_t vocab,
                                                       typename StatePtr<PAY>::out lo_out,
                                                       typename StatePtr<PAY>::out hi_out,
                                                       int64_t shift, int64_t reset_below,
                                                       uint8_t* __restrict__ mask, uint64_t ld,
                                                       uint64_t early_width, uint32_t split_at, DevView v,
                                                       uint32_t* __restrict__ pay,
                                                       uint32_t* __restrict__ pay_alt,
                                                       const uint32_t* __restrict__ pay_sel,
                                                       PeerSignal sig) {
  constexpr uint32_t CH = PACKED ? 32 : 16;
  constexpr int kAux4 = PAY ? kPayAux : kStoreAux;   // the 4-B stores' cache policy
  // first thread of the early zero-fill: wave 0 stays store-free (fewer
  // zero-filling waves -- from thread 256, 512 or 768 -- measured the same)
  constexpr int kEzFirst = 64;
  __shared__ Plan plan;
  __shared__ uint64_t s_lohi[3];              // new range + its only symbol when the transition table knew it (else ~0)
  __shared__ unsigned long long s_scan[2];    // workgroup E scan: first / last occurrence
  FM_STAMP_DECL;
  // sized at launch to the slice (16 KB at a 128k vocabulary instead of the
  // 32 KB maximum): LDS is what bounds the workgroups resident per CU at
  // 256 threads
  extern __shared__ __attribute__((aligned(16))) uint32_t win[];
  uint64_t row;
  uint32_t slice;
  // The static split of the wide rows' emit (split_at != 0: uint8 masks, one slice per row, B <= 256;
  // the grid is 2 x the padded rows).  Workgroup b < grid / 2 is row b's as always; workgroup
  // grid / 2 + b is row b's HELPER.  A row whose incoming range is wide (a restart, or >= cache_min
  // rows: the full range or a cached range -- the rows whose step ends in a 128-KB bitmap emit or a
  // late zero-fill, the step's last to finish) is emitted in two halves: tokens [0, split_at) by its
  // own workgroup, [split_at, V) by its helper, which takes the same LF step (redundantly: the probe
  // lines are then in its XCD's L2 -- grid / 2 is a multiple of 8, so a row and its helper share an
  // XCD) and stores no state.  The helper of any other row exits after the state load.  Decided by
  // the row's own state alone: no schedule, no atomics, no second read of a bitmap half.  (With
  // 89 VGPRs one 1024-thread workgroup fits a CU, so helpers are dispatched as the narrow rows'
  // workgroups retire.)
  const uint32_t half = gridDim.x / 2;
  const bool helper = split_at != 0 && blockIdx.x >= half;
  if (helper) {
    row = blockIdx.x - half;
    slice = 1;
  } else {
    map_block(blockIdx.x, S, row, slice);
  }
  // The row state first, as VECTOR loads (vmcnt) through the preloaded
  // pointers: FM_PRELOAD_VIEW's scalar loads then wait on lgkmcnt alone and do
  // not serialise behind (or in front of) the state's round trip.  (Serving
  // the rows in a "long dependent chain first" order -- every workgroup
  // reading all rows' state and taking the row at its own position -- was
  // measured: 10.7 us/step either way round against 10.3; the bulk of the
  // bytes, not the dispatch position of the slow rows, sets the step.)
  const uint32_t srow = (uint32_t)(row < m ? row : 0);
  const __amdgpu_buffer_rsrc_t r_lo = make_rsrc(lo_in, (uint32_t)(m * 8));
  const __amdgpu_buffer_rsrc_t r_hi = make_rsrc(hi_in, (uint32_t)(m * 8));
  typedef unsigned v2u __attribute__((ext_vector_type(2)));
  const v2u ql = __builtin_amdgcn_raw_buffer_load_b64(r_lo, srow * 8, 0, 0);
  const v2u qh = __builtin_amdgcn_raw_buffer_load_b64(r_hi, srow * 8, 0, 0);
  v2u qt = {0u, 0u};
  if (DO_LF) qt = __builtin_amdgcn_raw_buffer_load_b64(make_rsrc(tok, (uint32_t)(m * 8)), srow * 8, 0, 0);
  FM_STAMP(v, 0);
  const uint64_t st_lo = (uint64_t)ql.x | ((uint64_t)ql.y << 32), st_hi = (uint64_t)qh.x | ((uint64_t)qh.y << 32);
  const int64_t st_tok = (int64_t)((uint64_t)qt.x | ((uint64_t)qt.y << 32));
  if (row >= m) {   // a padding workgroup: nothing stored, still counted by the fused signal (PAY)
    if constexpr (PAY) {
      // (it stored nothing and read no counter: it only arrives)
      if (sig.done && threadIdx.x == 0) peer_signal_arrive(sig);
    }
    return;
  }
  uint64_t t0 = (uint64_t)slice * SW;
  uint64_t t1 = min(vocab, t0 + SW);
  if (split_at) {
    const uint64_t w_in = min(st_hi, v.n) > st_lo ? min(st_hi, v.n) - st_lo : 0;
    const bool wide = st_tok < reset_below || w_in >= v.cache_min;
    if (helper && !wide) return;                 // this row is emitted whole by its own workgroup
    t0 = helper ? split_at : 0;
    t1 = (wide && !helper) ? split_at : vocab;
  }
  if (t0 >= vocab) return;
  const uint64_t ntok = t1 - t0;
  const uint64_t nch = (ntok + CH - 1) / CH;
  uint8_t* out_row = mask + row * ld;
  // Rows whose incoming range is narrow stay narrow after the LF step (it
  // can only shrink a range), so their slice is zero-filled right away --
  // the stores overlap the LF chain -- and the final pass rewrites only the
  // chunks holding an allowed token.
  const bool reset = DO_LF && st_tok < reset_below;
  const uint64_t in_lo = st_lo, in_hi = min(st_hi, v.n);
  const bool early_zero = !PAY && !reset && (in_lo >= in_hi || in_hi - in_lo <= early_width);
  // Incoming ranges of kENarrow+1 .. kEWide rows that the transition table does
  // not serve take their LF step as ONE scan of E[lo, hi) by the whole
  // workgroup (<= kEWide / kDecThreads entries per thread, one round trip)
  // instead of the two-level descent; the other waves are idle until the plan
  // anyway (such rows are not zero-filled early).
  // (at most 4 entries per thread: smaller workgroups serve large batches,
  // where chains overlap anyway, and keep their registers for occupancy)
  constexpr uint32_t kScanMax = kEWide < 4u * kDecThreads ? kEWide : 4u * kDecThreads;
  const bool wg_scan = DO_LF && !reset && v.E && in_lo < in_hi && in_hi - in_lo > kENarrow &&
                       in_hi - in_lo <= kScanMax && !(in_lo == 0 && in_hi == v.n) &&
                       (in_hi - in_lo < v.cache_min || !v.trans_cap);
  FM_PRELOAD_VIEW(v);   // after the state loads are in flight (see above)
  if constexpr (PAY) {
    // the peer exchange's double buffer picked by the device step counter's parity (a
    // captured step replays for every step); only the stores at the end depend on it
    if (pay_sel && (__hip_atomic_load(pay_sel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u)) {
      out_row = reinterpret_cast<uint8_t*>(pay_alt) + (out_row - reinterpret_cast<uint8_t*>(pay));
      pay = pay_alt;
    }
  }
  const bool aligned16 = ((reinterpret_cast<uintptr_t>(out_row + t0) & 15) == 0);
  // the slice's bytes (uint8) or words (packed) as one buffer, offsets relative to token t0
  const __amdgpu_buffer_rsrc_t orsrc =
      make_rsrc(PACKED ? out_row + t0 / 8 : out_row + t0, (uint32_t)(PACKED ? (ntok + 31) / 32 * 4 : ntok));
  FM_STAMP(v, 1);
  // Zero-fill by waves 1.. only: loads and stores share vmcnt in issue order,
  // so a wave with stores in flight cannot wait on a load without also
  // waiting for them -- wave 0 (LF + plan) must stay store-free.
  if (early_zero && threadIdx.x >= kEzFirst) {
    for (uint64_t k = threadIdx.x - kEzFirst; k < nch; k += kDecThreads - kEzFirst) {
      if (kEzSleep && k >= kDecThreads - kEzFirst) __builtin_amdgcn_s_sleep(kEzSleep);
      const uint64_t t = t0 + k * CH;
      if (PACKED) {
        store4<kAux4>(orsrc, (uint32_t)(k * 4), 0u);
      } else if (aligned16 && t + CH <= t1) {
        store16(orsrc, (uint32_t)(k * 16), make_uint4(0, 0, 0, 0));
      } else {
        for (uint64_t j = t; j < min(t1, t + CH); ++j) out_row[j] = 0;
      }
    }
  }
  if (wg_scan) {
    const uint64_t c = (uint64_t)(st_tok + shift);
    constexpr int kU = (kScanMax + kDecThreads - 1) / kDecThreads;
    uint64_t e[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint64_t idx = in_lo + threadIdx.x + (uint64_t)u * kDecThreads;
      e[u] = idx < in_hi ? v.E[idx] : ~0ull;
    }
    if (threadIdx.x == 0) {
      s_scan[0] = ~0ull;
      s_scan[1] = 0;
    }
    lds_barrier();
    // first / last occurrence of c as (relative row + 1) << 36 | LF: min / max
    uint64_t fmin = ~0ull, fmax = 0;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (e[u] != ~0ull && (e[u] >> kESymShift) == c) {
        const uint64_t pk = ((uint64_t)(threadIdx.x + u * kDecThreads + 1) << kESymShift) | (e[u] & kELfMask);
        fmin = min(fmin, pk);
        fmax = max(fmax, pk);
      }
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      fmin = min(fmin, (uint64_t)__shfl_xor(fmin, d, 64));
      fmax = max(fmax, (uint64_t)__shfl_xor(fmax, d, 64));
    }
    if ((threadIdx.x & 63u) == 0 && fmax) {
      atomicMin(&s_scan[0], fmin);
      atomicMax(&s_scan[1], fmax);
    }
    lds_barrier();
  }
  // Wave 0: the LF step (all 64 lanes), then the bitmap plan of the new range
  // (all 64 lanes), published with the range by a single barrier.  A range
  // whose LF step was an E scan gets its content with the scan (E2): wave 0
  // keeps the matched entries' symbols in registers and sets their bits after
  // the barrier -- nothing is planned or streamed for it.
  uint32_t content[kENarrow / 64];
  uint32_t cmask = 0;
  if (threadIdx.x < 64) {
    uint64_t l = st_lo, h = st_hi;
    int64_t follow = -1;
    const uint32_t* tbm = nullptr;   // bitmap of the new range, when the transition table knew it
    int64_t one = -1;                // the new range's only symbol, when the transition table knew it
    if (DO_LF) {
      const int64_t t = st_tok;
      if (t < reset_below) {
        l = 0;
        h = v.n;
      } else {
        // from the full range the LF step lands on symbol c's C-block, whose
        // allowed set is c's precomputed follow-set bitmap
        if (l == 0 && h >= v.n) follow = t + shift;
        if (wg_scan) {
          const uint64_t a = s_scan[0], b = s_scan[1];
          l = b ? (a & kELfMask) : 0;
          h = b ? (b & kELfMask) + 1 : 0;
        } else {
          lf_step_decode<true>(v, t + shift, l, h, tbm, one, content, &cmask);
        }
        if (l >= h) follow = -1;
        // the payload ships a C-block narrower than a bitmap as its slice, not as its follow bitmap
        if (PAY && h - l < (vocab + 31) / 32) follow = -1;
        FM_STAMP(v, 2);
      }
    }
    l = __shfl(l, 0, 64);
    h = __shfl(h, 0, 64);
    follow = __shfl(follow, 0, 64);
    one = __shfl(one, 0, 64);
    if (h > v.n) h = v.n;
    if (threadIdx.x == 0) {
      s_lohi[0] = l;
      s_lohi[1] = h;
      s_lohi[2] = (uint64_t)one;
      plan.nb = 0;
      plan.a0 = plan.b0 = plan.a1 = plan.b1 = 0;
    }
    if (l < h && one < 0 && !(cmask & kContentPath)) {
      // a wide range is looked up in the range-bitmap cache first (one
      // bitmap, nothing streamed); otherwise the aligned-bitmap plan
      const uint32_t* cb = tbm ? tbm : cache_find(v, l, h);
      if (cb) {
        if (threadIdx.x == 0) {
          plan.nb = 1;
          plan.ptr[0] = cb;
        }
      } else {
        plan_range_wave(v, l, h, follow, plan);
      }
    }
  }
  // LDS window over symbol space, 128-bit aligned: words [w_lo, w_lo + nwin)
  const int64_t w_lo = floor_div32((int64_t)t0 + shift) & ~(int64_t)3;
  const int64_t sym_end = (int64_t)t1 + shift + 64;
  const uint32_t nwin = (uint32_t)(((sym_end - w_lo * 32 + 31) / 32 + 3) & ~3ll);
  for (uint32_t w = threadIdx.x; w < nwin; w += kDecThreads) win[w] = 0;
  FM_STAMP_T(v, 5, kDecThreads - 64);   // diagnostic: the last wave's arrival at the plan barrier
  lds_barrier();
  const uint64_t lo = s_lohi[0], hi = s_lohi[1];
  FM_STAMP(v, 3);
  if constexpr (PAY) {
    const uint32_t Wd = (uint32_t)((vocab + 31) / 32);
    const uint64_t W4 = ((uint64_t)Wd + 3) & ~3ull;
    const bool sparse = lo >= hi || (hi - lo < Wd && plan.nb == 0);   // workgroup-uniform
    if (threadIdx.x == 0) {
      const uint64_t H = payload_header_words(m);
      sys_store(&pay[4 + row], sparse ? (uint32_t)(lo < hi ? hi - lo : 0) : (Wd | 0x80000000u));
      sys_store(&pay[4 + m + row], (uint32_t)(H + row * W4));
      if (row == 0) {
        sys_store(&pay[0], (uint32_t)(H + m * W4));
        sys_store(&pay[1], (uint32_t)m);
        sys_store(&pay[2], Wd);
        sys_store(&pay[3], kPayMagic);
      }
    }
    if (sparse) {
      // the slice BWT[lo, hi): every load of the thread in flight together (clamped, masked after)
      const uint32_t w = lo < hi ? (uint32_t)(hi - lo) : 0u;
      for (uint32_t i0 = 0; i0 < w; i0 += 8 * kDecThreads) {
        uint32_t sy[8];
        if (v.bwt) {
#pragma unroll
          for (int u = 0; u < 8; ++u) sy[u] = v.bwt[lo + min(i0 + threadIdx.x + (uint32_t)u * kDecThreads, w - 1)];
        } else {
#pragma unroll
          for (int u = 0; u < 8; ++u)
            sy[u] = (uint32_t)(v.E[lo + min(i0 + threadIdx.x + (uint32_t)u * kDecThreads, w - 1)] >> kESymShift);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const uint32_t i = i0 + threadIdx.x + (uint32_t)u * kDecThreads;
          if (i < w) store4<kAux4>(orsrc, i * 4, sy[u]);
        }
      }
      if (DO_LF && threadIdx.x == 0) {
        lo_out[row] = lo;
        hi_out[row] = hi;
      }
      if (sig.done) peer_signal_done(sig);
      return;
    }
  }
  // Roles.  A wave with stores in flight cannot wait on a load without
  // waiting for its stores too (shared vmcnt), so loads go to store-free waves:
  //   early zero  (narrow input): waves 1.. have zero-filled; wave 0 streams
  //   late zero   (output streamed only, wide input): waves 0-3 stream while
  //               waves 4.. zero-fill now, overlapping the stream round trip
  //   otherwise   every wave gathers (bitmaps + partial ends), every wave emits
  // The zero-filling waves own their chunks in the final emit (program order).
  const bool late_zero = kDecThreads >= 512 && !early_zero && lo < hi && plan.nb == 0;
  const uint32_t e_first = early_zero ? (uint32_t)kEzFirst : (late_zero ? 256u : 0u);   // emit/zero owners: tid >= e_first
  if (late_zero && threadIdx.x >= e_first) {
    for (uint64_t k = threadIdx.x - e_first; k < nch; k += kDecThreads - e_first) {
      const uint64_t t = t0 + k * CH;
      if (PACKED) {
        store4<kAux4>(orsrc, (uint32_t)(k * 4), 0u);
      } else if (aligned16 && t + CH <= t1) {
        store16(orsrc, (uint32_t)(k * 16), make_uint4(0, 0, 0, 0));
      } else {
        for (uint64_t j = t; j < min(t1, t + CH); ++j) out_row[j] = 0;
      }
    }
  }
  // One whole bitmap and nothing streamed (a cached range, the full range or a
  // follow set): emitted straight from the bitmap in memory, no LDS pass.
  const bool single = lo < hi && plan.nb == 1 && plan.a0 >= plan.b0 && plan.a1 >= plan.b1;
  const bool direct = single && kDecThreads >= 1024;
  if (single && !direct) {
    // smaller workgroups: the one bitmap is staged into the LDS window with
    // every load of a batch in flight together (one round trip for a 128k
    // vocabulary at 256 threads), then emitted like any gathered window
    const uint32_t* bm = plan.ptr[0];
    const uint32_t nw4 = nwin / 4;
    for (uint32_t j0 = threadIdx.x; j0 < nw4; j0 += 4 * kDecThreads) {
      uint4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t w4b = j0 + (uint32_t)u * kDecThreads;
        const int64_t gwb = w_lo + 4 * (int64_t)w4b;
        x[u] = (w4b < nw4 && gwb >= 0 && gwb + 4 <= (int64_t)v.bm_words)
                   ? gld4(bm, gwb) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t w4b = j0 + (uint32_t)u * kDecThreads;
        if (w4b < nw4) *reinterpret_cast<uint4*>(&win[4 * w4b]) = x[u];
      }
    }
    lds_barrier();
  } else if (lo < hi && !direct) {
    const int64_t base_bit = w_lo * 32;
    const int64_t lim = (int64_t)nwin * 32;
    const uint32_t nb = plan.nb;
    if (nb == 0) {
      // streamed only
      const uint32_t nthr = early_zero ? 64u : (late_zero ? 256u : (uint32_t)kDecThreads);
      if (threadIdx.x < nthr) {
        if (v.bwt)
          stream_symbols(v.bwt, plan.a0, plan.b0, plan.a1, plan.b1, base_bit, lim, win, nthr);
        else
          stream_symbols_e(v.E, plan.a0, plan.b0, plan.a1, plan.b1, base_bit, lim, win, nthr);
      }
      if (threadIdx.x == 0 && (int64_t)s_lohi[2] >= 0) set_bit(win, (uint32_t)s_lohi[2], base_bit, lim);   // one-row range
      if (cmask & kContentPath) {   // wave 0: the content read with the E scan
#pragma unroll
        for (uint32_t j = 0; j < kENarrow / 64; ++j)
          if ((cmask >> j) & 1u) set_bit(win, content[j], base_bit, lim);
      }
      FM_STAMP(v, 4);
    } else {
      // The first batch of bitmap words (<= 8 per thread) is loaded before the
      // partial ends are streamed, so both are in flight in one round trip.
      const uint32_t nw4 = nwin / 4;
      const uint32_t G = max(1u, (uint32_t)kDecThreads / nw4);   // thread groups splitting the bitmaps
      const uint32_t g = threadIdx.x / nw4;
      uint32_t w4b = threadIdx.x % nw4;
      int64_t gwb = w_lo + 4 * (int64_t)w4b;
      bool own = g < G && w4b < nw4 && gwb >= 0 && gwb + 4 <= (int64_t)v.bm_words;
      uint4 x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t qq = g + (uint32_t)u * G;
        // unconditional (clamped) load, masked afterwards: under a branch the
        // compiler put a vmcnt(0) between the first and second load
        const bool ok = own && qq < nb;
        const uint4 y = gld4(plan.ptr[ok ? qq : 0], ok ? gwb : 0);
        const uint32_t m = ok ? ~0u : 0u;
        x[u] = make_uint4(y.x & m, y.y & m, y.z & m, y.w & m);
      }
      if (v.bwt)
        stream_symbols(v.bwt, plan.a0, plan.b0, plan.a1, plan.b1, base_bit, lim, win, kDecThreads);
      else
        stream_symbols_e(v.E, plan.a0, plan.b0, plan.a1, plan.b1, base_bit, lim, win, kDecThreads);
      FM_STAMP(v, 4);
      // G groups split the bitmaps, each thread owns one uint4 of the window
      // (several when the window is wider than the workgroup); partial ORs
      // merge with LDS atomics.
      bool first = true;
      while (g < G && w4b < nw4) {
        if (own) {
          uint4 acc = make_uint4(0, 0, 0, 0);
          for (uint32_t q = g; q < nb; q += G * 8) {
            if (!first) {
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const uint32_t qq = q + (uint32_t)u * G;
                x[u] = qq < nb ? gld4(plan.ptr[qq], gwb) : make_uint4(0, 0, 0, 0);
              }
            }
            first = false;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              acc.x |= x[u].x;
              acc.y |= x[u].y;
              acc.z |= x[u].z;
              acc.w |= x[u].w;
            }
          }
          if (acc.x) atomicOr(&win[4 * w4b + 0], acc.x);
          if (acc.y) atomicOr(&win[4 * w4b + 1], acc.y);
          if (acc.z) atomicOr(&win[4 * w4b + 2], acc.z);
          if (acc.w) atomicOr(&win[4 * w4b + 3], acc.w);
        }
        first = false;
        w4b += kDecThreads;
        gwb = w_lo + 4 * (int64_t)w4b;
        own = w4b < nw4 && gwb >= 0 && gwb + 4 <= (int64_t)v.bm_words;
      }
    }
    lds_barrier();
  }
  FM_STAMP(v, 6);
  // A zeroed chunk's final store follows its zero store from the same thread
  // to the same address, in program order: per-location coherence orders the
  // two, no wait for the zero stores' acknowledgements is needed.
  const bool zeroed = early_zero || late_zero;
  const int64_t rel0 = (int64_t)t0 + shift - w_lo * 32;   // >= 0
  if (direct) {
    // bits of chunk k = bitmap bits [t0 + CH k + shift, + CH).  All of a
    // thread's chunks (kDirectU per round, one round for a 128k-152k vocab)
    // have their words loaded before any is converted and stored: the emit is
    // one memory round trip.  Chunk ownership as in the zero-fill (threads >=
    // e_first) when the row was zeroed early.
    const uint32_t* bm = plan.ptr[0];
    const uint32_t wlim = v.bm_words;
    const __amdgpu_buffer_rsrc_t brs = make_rsrc(bm, wlim * 4u);
    const uint32_t nt = kDecThreads - e_first;
    const uint32_t nch32 = (uint32_t)nch;
    const uint32_t bit0 = (uint32_t)((int64_t)t0 + shift);   // < 2^27: 32-bit chunk arithmetic
    constexpr int kDirectU = (kDecThreads >= 1024) ? 8 : 4;
    for (uint32_t k0 = threadIdx.x - e_first; threadIdx.x >= e_first && k0 < nch32; k0 += nt * kDirectU) {
      uint32_t wa[kDirectU], wb[kDirectU];
#pragma unroll
      for (int u = 0; u < kDirectU; ++u) {
        const uint32_t k = k0 + (uint32_t)u * nt;
        const uint32_t wi = (bit0 + k * CH) >> 5;
        // buffer loads: the descriptor's range check returns 0 past the
        // bitmap's end, so every load is unconditional and all 2 kDirectU are
        // in flight together (a guarded first load was followed by a vmcnt(0));
        // words of chunks k >= nch are loaded and not used
        wa[u] = __builtin_amdgcn_raw_buffer_load_b32(brs, wi * 4u, 0, 0);
        wb[u] = __builtin_amdgcn_raw_buffer_load_b32(brs, wi * 4u + 4u, 0, 0);
      }
      uint32_t slow = 0;   // chunks needing byte stores (a short last chunk / unaligned row): after the loop
#pragma unroll
      for (int u = 0; u < kDirectU; ++u) {
        const uint32_t k = k0 + (uint32_t)u * nt;
        if (k >= nch32) break;
        const uint32_t o = (bit0 + k * CH) & 31u;
        const uint64_t t = t0 + (uint64_t)k * CH;
        const bool full = t + CH <= t1;
        uint32_t bits = (uint32_t)((((uint64_t)wb[u] << 32) | wa[u]) >> o);
        if (CH == 16) bits &= 0xFFFFu;
        if (PACKED && !full) bits &= (1u << (uint32_t)(t1 - t)) - 1u;
        if (zeroed && bits == 0) continue;
        if (PACKED) {
          store4<kAux4>(orsrc, k * 4, bits);
        } else if (aligned16 && full) {
          store16_emit(orsrc, k * 16, bits16_to_bytes(bits), zeroed);
        } else {
          slow |= 1u << u;
        }
      }
#pragma unroll 1
      for (uint32_t u = 0; !PACKED && slow; ++u, slow >>= 1) {
        if (!(slow & 1u)) continue;
        const uint32_t k = k0 + u * nt;
        const uint32_t wi = (bit0 + k * CH) >> 5, o = (bit0 + k * CH) & 31u;
        const uint32_t a = wi < wlim ? gld(bm, wi) : 0u, b = wi + 1 < wlim ? gld(bm, wi + 1) : 0u;
        const uint32_t bits = (uint32_t)((((uint64_t)b << 32) | a) >> o);
        const uint64_t t = t0 + (uint64_t)k * CH;
        const uint32_t cnt = (uint32_t)min((uint64_t)CH, t1 - t);
        for (uint32_t j = 0; j < cnt; ++j) out_row[t + j] = (uint8_t)((bits >> j) & 1u);
      }
    }
  } else if (threadIdx.x >= e_first) {
    for (uint64_t k = threadIdx.x - e_first; k < nch; k += kDecThreads - e_first) {
      const int64_t rel = rel0 + (int64_t)k * CH;
      const uint32_t wi = (uint32_t)(rel >> 5);
      const uint32_t o = (uint32_t)(rel & 31);
      const uint64_t w2 = (uint64_t)win[wi] | ((uint64_t)win[wi + 1] << 32);
      uint32_t bits = (uint32_t)(w2 >> o);
      const uint64_t t = t0 + k * CH;
      const uint64_t cnt = min((uint64_t)CH, t1 - t);
      if (CH == 16) bits &= 0xFFFFu;
      if (cnt < CH) bits &= (1u << cnt) - 1u;
      if (zeroed && bits == 0) continue;
      if (PACKED) {
        store4<kAux4>(orsrc, (uint32_t)(k * 4), bits);   // t0 and t are multiples of 32
      } else if (aligned16 && cnt == 16) {
        store16_emit(orsrc, (uint32_t)(k * 16), bits16_to_bytes(bits), zeroed);
      } else {
        for (uint64_t j = 0; j < cnt; ++j) out_row[t + j] = (uint8_t)((bits >> j) & 1u);
      }
    }
  }
  // The new row state is stored last: wave 0 loads after its LF step (cache
  // probe, partial ends), and with a store ahead of them in the shared vmcnt
  // queue each of those waits would include the store's acknowledgement.
  if (DO_LF && slice == 0 && threadIdx.x == 0) {
    lo_out[row] = lo;
    hi_out[row] = hi;
  }
  if constexpr (PAY) {
    if (sig.done) peer_signal_done(sig);
  }
  FM_STAMP(v, 7);
  if (!helper) FM_STAMP_FLUSH(v, row);
}

// cache probe per row (one wave each): 1 if [lo, hi) has a cached bitmap
__global__ void __launch_bounds__(256) k_cache_probe(DevView v, const uint64_t* __restrict__ lo,
                                                    const uint64_t* __restrict__ hi, uint64_t m,
                                                    uint8_t* __restrict__ out) {
  const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (i >= m) return;
  const uint64_t l = lo[i], h = min(hi[i], v.n);
  const bool hit = l < h && cache_find(v, l, h) != nullptr;
  if ((threadIdx.x & 63u) == 0) out[i] = hit ? 1 : 0;
}

}  // namespace

// Workgroup size by batch: one 1024-thread workgroup per row while the rows
// fit one per CU (the emit of a row's 128 KB wants all 16 waves' store
// issue); beyond that smaller workgroups, so that several rows' dependent
// chains overlap on each CU (measured at B = 2048: 49.6 us/step with 256
// threads, 60.1 with 512, 79.1 with 1024, 71.4 with 128; B = 512: 15.2 /
// 17.6 / 18.1 / 22.4; B = 256: 1024 and 256 threads x 4 slices tie at 10.4).
// The tuning's dec_threads overrides.
static uint32_t decode_threads(uint64_t m) {
  const uint32_t e = tuning().dec_threads;
  if (e == 256 || e == 512 || e == 1024) return e;
  return m <= 256 ? 1024 : 256;
}

#ifndef FMIDX_DEC_SPLIT
// measurement variant 1: the static split of the wide rows' emit (k_decode) -- exact, but slower at
// C3: 15.9-16.0 us cold per step against 13.7-13.9 (profiles/r06_split/)
#define FMIDX_DEC_SPLIT 0
#endif
constexpr bool kDecSplit = FMIDX_DEC_SPLIT != 0;

#ifndef FMIDX_WAVE_BUDGET
#define FMIDX_WAVE_BUDGET 4096   // measurement variant: resident waves the slice geometry aims at
#endif

// Slice geometry.  Residency budget: kernels of this shape keep about 16 waves
// per CU resident (measured, profiles/r01_tuning); a launch of more waves than
// budget dispatches its tail only as earlier workgroups retire.  So the slices
// per row are chosen to keep rows * S * (threads / 64) waves within the
// budget (default one slice per row at B >= 256), slices a multiple of 64 tokens.
static void mask_geometry(uint64_t m, uint64_t vocab, uint32_t threads, uint32_t& S, uint32_t& SW) {
  uint32_t s = tuning().mask_slices;
  const uint64_t s_min = (vocab + kMaxSliceTokens - 1) / kMaxSliceTokens;
  if (s == 0) {
    const uint64_t rows = (m + 7) / 8 * 8;
    const uint64_t budget = FMIDX_WAVE_BUDGET;
    const uint64_t want = std::max<uint64_t>(1, budget / (rows * (threads / 64)));
    const uint64_t max_s = std::max<uint64_t>(1, (vocab + 8191) / 8192);
    s = (uint32_t)std::min(want, max_s);
  }
  s = (uint32_t)std::max<uint64_t>(s, std::max<uint64_t>(1, s_min));
  uint64_t sw = (vocab + s - 1) / s;
  sw = (sw + 63) & ~63ull;
  if (sw > kMaxSliceTokens) sw = kMaxSliceTokens;
  SW = (uint32_t)sw;
  S = (uint32_t)((vocab + sw - 1) / sw);
}

static int launch_decode_kernel(const DevView& v, const int64_t* tok, int64_t shift,
                                int64_t reset_below, const uint64_t* lo_in, const uint64_t* hi_in,
                                uint64_t* lo_out, uint64_t* hi_out, uint64_t m, uint8_t* mask,
                                uint64_t ld, uint64_t vocab, int packed, bool do_lf, hipStream_t s) {
  if (packed && (ld % 4 != 0 || ld < 4 * ((vocab + 31) / 32) ||
                 (reinterpret_cast<uintptr_t>(mask) & 3))) {
    set_error("packed mask needs 4-byte aligned rows with ld >= 4*ceil(vocab/32)");
    return -1;
  }
  if (!packed && ld < vocab) {
    set_error("mask leading dimension %llu < vocab %llu", (unsigned long long)ld,
              (unsigned long long)vocab);
    return -1;
  }
  const uint32_t T = decode_threads(m);
  uint32_t S, SW;
  mask_geometry(m, vocab, T, S, SW);
  // the wide rows' emit split with a helper workgroup each (see k_decode): the fused uint8 step at
  // one 1024-thread workgroup per row
  const uint32_t split_at = (kDecSplit && do_lf && !packed && T == 1024 && S == 1 && vocab >= 2048)
                                ? (uint32_t)(((vocab / 2) + 63) & ~63ull) : 0u;
  const uint64_t grid = (m + 7) / 8 * 8 * S * (split_at ? 2 : 1);
  if (grid > 0x7fffffffull / T) {
    set_error("too many rows for one launch");
    return -1;
  }
  const unsigned g = (unsigned)grid;
  const uint64_t ew = kEarlyZeroWidth;
  const size_t lds = (size_t)win_words(SW) * 4;
#define FM_LAUNCH(P, L, TT)                                                                                    \
  k_decode<P, L, TT><<<g, TT, lds, s>>>(tok, lo_in, hi_in, m, S, SW, vocab, lo_out, hi_out, shift, reset_below, \
                                        mask, ld, ew, split_at, v, nullptr, nullptr, nullptr, PeerSignal{})
#define FM_LAUNCH_T(P, L)          \
  do {                             \
    if (T == 1024)                 \
      FM_LAUNCH(P, L, 1024);       \
    else if (T == 512)             \
      FM_LAUNCH(P, L, 512);        \
    else                           \
      FM_LAUNCH(P, L, 256);        \
  } while (0)
  if (do_lf) {
    if (packed) FM_LAUNCH_T(true, true);
    else FM_LAUNCH_T(false, true);
  } else {
    if (packed) FM_LAUNCH_T(true, false);
    else FM_LAUNCH_T(false, false);
  }
#undef FM_LAUNCH_T
#undef FM_LAUNCH
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_decode_payload(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                          const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out, uint64_t* hi_out,
                          uint64_t m, uint32_t* pay, uint64_t cap, uint64_t vocab, uint32_t* pay_alt,
                          const uint32_t* pay_sel, hipStream_t s, const uint64_t* sig_dst, uint64_t sig_world,
                          uint32_t* sig_done) {
  if (m == 0) return 0;
  const uint64_t W = (vocab + 31) / 32, W4 = (W + 3) & ~3ull, H = payload_header_words(m);
  if (!pay || !tok || !lo_in || !hi_in || !lo_out || !hi_out || vocab == 0 || W > kPayMaxWords ||
      m >= (1ull << 31) || (reinterpret_cast<uintptr_t>(pay) & 15) || (pay_sel && !pay_alt) ||
      (reinterpret_cast<uintptr_t>(pay_alt) & 15)) {
    set_error("decode payload: bad arguments (vocab %llu <= 262144, 16-B aligned payload)",
              (unsigned long long)vocab);
    return -1;
  }
  if (cap < H + m * W4 || H + m * W4 >= (1ull << 32)) {
    set_error("decode payload: %llu words, %llu needed (< 2^32)", (unsigned long long)cap,
              (unsigned long long)(H + m * W4));
    return -1;
  }
  // the state may be updated in place here (one workgroup per row: its one store follows every
  // read of the row's state behind the workgroup's barriers), so a captured step replays as is;
  // partial overlap is still refused
  if ((lo_in != lo_out && lo_in < lo_out + m && lo_out < lo_in + m) ||
      (hi_in != hi_out && hi_in < hi_out + m && hi_out < hi_in + m)) {
    set_error("decode payload: state in/out buffers overlap without being the same buffer");
    return -1;
  }
  if (sig_done && (!pay_sel || sig_world > 64 || (sig_world && !sig_dst))) {
    set_error("decode payload: the fused signal needs the step counter and 0..64 flag addresses");
    return -1;
  }
  const PeerSignal sig{sig_dst, const_cast<uint32_t*>(pay_sel), sig_done, (uint32_t)sig_world};
  const uint32_t T = decode_threads(m);
  const uint32_t S = 1, SW = (uint32_t)((vocab + 63) & ~63ull);   // one slice per row: whole-row decisions
  const unsigned g = (unsigned)((m + 7) / 8 * 8);
  const size_t lds = (size_t)win_words(SW) * 4;
  uint8_t* mask = reinterpret_cast<uint8_t*>(pay + H);
  const uint64_t ld = W4 * 4;
  if (T == 1024)
    k_decode<true, true, 1024, true><<<g, 1024, lds, s>>>(tok, lo_in, hi_in, m, S, SW, vocab, lo_out, hi_out, shift,
                                                          reset_below, mask, ld, 0, 0u, v, pay, pay_alt, pay_sel, sig);
  else if (T == 512)
    k_decode<true, true, 512, true><<<g, 512, lds, s>>>(tok, lo_in, hi_in, m, S, SW, vocab, lo_out, hi_out, shift,
                                                        reset_below, mask, ld, 0, 0u, v, pay, pay_alt, pay_sel, sig);
  else
    k_decode<true, true, 256, true><<<g, 256, lds, s>>>(tok, lo_in, hi_in, m, S, SW, vocab, lo_out, hi_out, shift,
                                                        reset_below, mask, ld, 0, 0u, v, pay, pay_alt, pay_sel, sig);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_cache_probe(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m, uint8_t* out,
                       hipStream_t s) {
  if (m == 0) return 0;
  k_cache_probe<<<(unsigned)((m * 64 + 255) / 256), 256, 0, s>>>(v, lo, hi, m, out);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_mask(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t m,
                uint8_t* mask, uint64_t ld, uint64_t vocab, int64_t shift, int packed,
                hipStream_t s) {
  if (m == 0 || vocab == 0) return 0;
  return launch_decode_kernel(v, nullptr, shift, 0, lo, hi, nullptr, nullptr, m, mask, ld, vocab, packed,
                              false, s);
}

// Follow-set bitmaps: row c = packed mask (symbol space, shift 0) of the
// C-block [C[c], C[c+1]) -- exactly the bitmap layout plan_range_wave reads.
int launch_follow_bitmaps(const DevView& v, const uint64_t* C, uint64_t nsym, uint32_t* out,
                          hipStream_t s) {
  const uint64_t ld = (uint64_t)v.bm_words * 4;
  const uint64_t chunk = 32768;   // rows per launch
  for (uint64_t c0 = 0; c0 < nsym; c0 += chunk) {
    const uint64_t m = std::min(chunk, nsym - c0);
    if (launch_decode_kernel(v, nullptr, 0, 0, C + c0, C + c0 + 1, nullptr, nullptr, m,
                             reinterpret_cast<uint8_t*>(out + c0 * v.bm_words), ld,
                             (uint64_t)v.bm_words * 32, 1, false, s))
      return -1;
  }
  return 0;
}

int launch_decode(const DevView& v, const int64_t* tok, int64_t shift, int64_t reset_below,
                  const uint64_t* lo_in, const uint64_t* hi_in, uint64_t* lo_out, uint64_t* hi_out,
                  uint64_t m, uint8_t* mask, uint64_t ld, uint64_t vocab, int packed, hipStream_t s) {
  if (m == 0) return 0;
  if (vocab == 0)   // LF only: the per-row kernel is safe in place
    return launch_lf_step(v, tok, shift, reset_below, lo_in, hi_in, lo_out, hi_out, m, s);
  if (lo_in == lo_out || hi_in == hi_out) {
    set_error("fused decode step: state in/out buffers must not alias (ping-pong them)");
    return -1;
  }
  return launch_decode_kernel(v, tok, shift, reset_below, lo_in, hi_in, lo_out, hi_out, m, mask, ld, vocab,
                              packed, true, s);
}

}  // namespace fmidx
