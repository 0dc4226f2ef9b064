// shard.hip -- the exchange step of doc-range sharding: the
// bit-packed allowed-token rows of every shard (gathered over RCCL) are ORed
// into the row of the unsharded index, and optionally expanded to the uint8
// [B, V] mask in the same pass (one read of each shard's words, one write).
//
//   parts   nparts blocks of B rows x words_per_row uint32 (block stride
//           part_stride words), little-endian bit order: token t of row b is
//           bit t % 32 of word t / 32 -- fm_allowed_mask_batch(packed = 1)'s
//           layout, i.e. what each rank's decode step wrote.
//   unpack  0: out = uint32 [B, words_per_row] (ld_out bytes per row), the OR
//           of the words; 1: out = uint8 [B, vocab] 0/1 (ld_out bytes per row).
#include "fmidx_internal.h"

#include <cstdlib>

namespace fmidx {

namespace {

constexpr int kThreads = 256;

// The OR of one word over every part.  The parts' loads are independent, so
// they are issued 8 at a time before any is used (a plain loop over a runtime
// part count put a wait behind every load: one HBM round trip per shard).
// Past the last part the index is clamped (the last part again: harmless for
// an OR), so no load sits under a branch.
__device__ __forceinline__ uint32_t or_parts(const uint32_t* __restrict__ parts, uint32_t nparts,
                                             uint64_t part_stride, uint64_t off) {
  uint32_t x = 0;
  for (uint32_t p0 = 0; p0 < nparts; p0 += 8) {
    uint32_t v[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) v[q] = parts[(uint64_t)min(p0 + q, nparts - 1) * part_stride + off];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) x |= v[q];
  }
  return x;
}

// One wave per tile of kTileWords words (8192 tokens) of one row.  Lane l ORs
// words [4l, 4l + 4) of the tile over every part -- one 16-B load per part,
// so a wave instruction reads 1 KB contiguous (VEC: rows of a multiple of 4
// words; word loads otherwise) -- and the tile's words go through LDS to the
// emit, where store j of lane l writes the 16 tokens of chunk 64 j + l: a
// wave instruction writes 1 KB contiguous.  (One thread per 16 tokens with a
// 4-B load per part, round 3's first version: 2.2 TB/s cold at C4, 8 x 4.1 MB
// in + 33 MB out in 30 us; the 4-B loads, two lanes per word, are
// request-bound.)  Stores write through (sc1) like k_decode's, leaving no
// dirty lines for the kernel-end writeback.
constexpr uint32_t kTileWords = 256;
constexpr int kOrStoreAux = 16;
typedef unsigned or_v4u __attribute__((ext_vector_type(4)));

template <bool VEC>
__global__ void __launch_bounds__(kThreads) k_or_unpack(const uint32_t* __restrict__ parts, uint32_t nparts,
                                                        uint64_t part_stride, uint64_t B, uint64_t wpr,
                                                        uint64_t vocab, uint8_t* __restrict__ out, uint64_t ld) {
  __shared__ uint32_t s_w[kThreads / 64][kTileWords];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t tiles = (wpr + kTileWords - 1) / kTileWords;
  const uint64_t tw = (uint64_t)blockIdx.x * (kThreads / 64) + wv;
  const bool on = tw < B * tiles;                      // wave-uniform
  const uint64_t b = on ? tw / tiles : 0, tile = on ? tw - b * tiles : 0;
  const uint64_t w0 = tile * kTileWords + 4 * lane;    // this lane's first word in the row
  uint32_t x[4] = {0u, 0u, 0u, 0u};
  if (on) {
    if (VEC) {
      const bool inside = w0 < wpr;                    // wpr % 4 == 0: all four words or none
      const uint64_t off = b * wpr + (inside ? w0 : 0);
      for (uint32_t p0 = 0; p0 < nparts; p0 += 8) {
        uint4 v[8];
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q)
          v[q] = *reinterpret_cast<const uint4*>(parts + (uint64_t)min(p0 + q, nparts - 1) * part_stride + off);
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
          x[0] |= v[q].x;
          x[1] |= v[q].y;
          x[2] |= v[q].z;
          x[3] |= v[q].w;
        }
      }
      if (!inside) x[0] = x[1] = x[2] = x[3] = 0u;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool inside = w0 + k < wpr;
        const uint32_t y = or_parts(parts, nparts, part_stride, b * wpr + (inside ? w0 + k : 0));
        x[k] = inside ? y : 0u;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) s_w[wv][4 * lane + k] = x[k];
  __syncthreads();                                     // LDS only: no global store precedes it
  if (!on) return;
  __amdgpu_buffer_rsrc_t r = make_rsrc(out + b * ld, (uint32_t)vocab);
  const uint64_t tok0 = tile * kTileWords * 32;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t c = 64u * j + lane;                 // 16-token chunk of the tile
    const uint64_t t0 = tok0 + 16ull * c;
    if (t0 >= vocab) break;
    const uint32_t bits = (s_w[wv][c >> 1] >> (16 * (c & 1))) & 0xFFFFu;
    uint32_t q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = (((bits >> (4 * i)) & 0xFu) * 0x204081u) & 0x01010101u;
    if (t0 + 16 <= vocab && ((reinterpret_cast<uintptr_t>(out + b * ld + t0) & 15) == 0)) {
      or_v4u v = {q[0], q[1], q[2], q[3]};
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (uint32_t)t0, 0, kOrStoreAux);
    } else {
      uint8_t* o = out + b * ld + t0;
      for (uint64_t i = 0; i < 16 && t0 + i < vocab; ++i) o[i] = (bits >> i) & 1u;
    }
  }
}

// packed output: one thread per 4 words (VEC: 16-B loads and store) or per word
template <bool VEC>
__global__ void __launch_bounds__(kThreads) k_or_words(const uint32_t* __restrict__ parts, uint32_t nparts,
                                                       uint64_t part_stride, uint64_t B, uint64_t wpr,
                                                       uint32_t* __restrict__ out, uint64_t ldw) {
  const uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  if (VEC) {
    const uint64_t q4 = wpr / 4;
    const uint64_t b = g / q4, w = 4 * (g - b * q4);
    if (b >= B) return;
    uint4 x = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t p0 = 0; p0 < nparts; p0 += 8) {
      uint4 v[8];
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q)
        v[q] = *reinterpret_cast<const uint4*>(parts + (uint64_t)min(p0 + q, nparts - 1) * part_stride + b * wpr + w);
#pragma unroll
      for (uint32_t q = 0; q < 8; ++q) {
        x.x |= v[q].x;
        x.y |= v[q].y;
        x.z |= v[q].z;
        x.w |= v[q].w;
      }
    }
    *reinterpret_cast<uint4*>(out + b * ldw + w) = x;
  } else {
    const uint64_t b = g / wpr, w = g - b * wpr;
    if (b >= B) return;
    out[b * ldw + w] = or_parts(parts, nparts, part_stride, b * wpr + w);
  }
}

}  // namespace

int launch_or_bits(const uint32_t* parts, uint64_t nparts, uint64_t part_stride, uint64_t B, uint64_t wpr,
                   uint64_t vocab, void* out, uint64_t ld_out, int unpack, hipStream_t s) {
  if (B == 0 || nparts == 0) return 0;
  if (!parts || !out || wpr * 32 < vocab || part_stride < B * wpr) {
    set_error("or_bits: %llu words per row cannot hold %llu tokens, or parts overlap",
              (unsigned long long)wpr, (unsigned long long)vocab);
    return -1;
  }
  if (unpack) {
    if (ld_out < vocab) {
      set_error("or_bits: output row of %llu bytes < vocab %llu", (unsigned long long)ld_out,
                (unsigned long long)vocab);
      return -1;
    }
    if (vocab >= (1ull << 32)) {
      set_error("or_bits: vocab %llu does not fit one row buffer", (unsigned long long)vocab);
      return -1;
    }
    const uint64_t waves = B * ((wpr + kTileWords - 1) / kTileWords);
    const unsigned grid = (unsigned)((waves + kThreads / 64 - 1) / (kThreads / 64));
    const bool vec = wpr % 4 == 0 && part_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(parts) & 15) == 0;
    if (vec)
      k_or_unpack<true><<<grid, kThreads, 0, s>>>(parts, (uint32_t)nparts, part_stride, B, wpr, vocab,
                                                  static_cast<uint8_t*>(out), ld_out);
    else
      k_or_unpack<false><<<grid, kThreads, 0, s>>>(parts, (uint32_t)nparts, part_stride, B, wpr, vocab,
                                                   static_cast<uint8_t*>(out), ld_out);
  } else {
    if (ld_out % 4 || ld_out < wpr * 4) {
      set_error("or_bits: packed output rows need ld >= 4 * words and a multiple of 4");
      return -1;
    }
    const bool vec = wpr % 4 == 0 && part_stride % 4 == 0 && ld_out % 16 == 0 &&
                     (reinterpret_cast<uintptr_t>(parts) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    const uint64_t threads = vec ? B * (wpr / 4) : B * wpr;
    const unsigned grid = (unsigned)((threads + kThreads - 1) / kThreads);
    if (vec)
      k_or_words<true><<<grid, kThreads, 0, s>>>(parts, (uint32_t)nparts, part_stride, B, wpr,
                                                 static_cast<uint32_t*>(out), ld_out / 4);
    else
      k_or_words<false><<<grid, kThreads, 0, s>>>(parts, (uint32_t)nparts, part_stride, B, wpr,
                                                  static_cast<uint32_t*>(out), ld_out / 4);
  }
  FM_HIP(hipGetLastError());
  return 0;
}


// ---- the sparse exchange (C4): per row either the shard's BWT slice or its bitmap
//
// A rank's payload (uint32 words, every offset a multiple of 4 words):
//   [0] total words (a multiple of 4)   [1] B   [2] words per bitmap row W   [3] kPayloadMagic
//   [4, 4 + B)        desc[b] = count | (dense << 31)
//   [4 + B, 4 + 2B)   off[b]  = word offset of row b's data in this payload
//   [F, F + 3B)       facts[k * B + b], F = payload_facts_at(B): a processor call's per-row facts
//                     (k_prep over the shard: count([last]) > 0, range non-empty, distinct non-empty),
//                     ORed by the OR pass -- so a sharded processor call needs no collective for them
//                     (zeros when the payload carries none)
//   data: row b's `count` words at off[b] (zero-padded to a multiple of 4):
//         dense  -- the W words of its allowed-token bitmap (the decode step's packed row)
//         sparse -- BWT[lo, hi) of the shard (T' symbols; token = symbol - shift when in [0, V)),
//                   chosen when hi - lo < W, i.e. when the slice is smaller than the bitmap.
// Most decode rows are narrow on a shard (median width 1 at C3), so a payload is a few
// hundred KB where the packed rows of every row are B * W * 4 bytes (4.1 MB at B = 256).
namespace {

constexpr uint32_t kPayloadMagic = 0x58534D46u;   // "FMSX"


// One workgroup per row, one launch: the workgroup sums the padded sizes of
// the rows before its own (every thread loads a few (lo, hi) pairs -- B * 16
// bytes, L2-resident after the first workgroup -- then a wave reduction), so
// no separate scan launch precedes the copy: two dependent round trips
// (the states, then the row's source) in all.  Workgroup B - 1 writes the
// header words, workgroup 0 zeroes the header's padding.
constexpr int kPackRowThreads = 256;

__device__ __forceinline__ uint64_t pack_row_words(uint64_t l, uint64_t h, uint64_t n, uint32_t W, uint32_t& desc) {
  h = min(h, n);                                       // a state past the BWT reads none of it
  const uint64_t w = h > l ? h - l : 0;
  const bool dense = w >= W;
  const uint64_t count = dense ? W : w;
  desc = (uint32_t)count | (dense ? 0x80000000u : 0u);
  return (count + 3) & ~3ull;
}

// The payload's stores are system-scope write-through (sc0 sc1): a payload packed into a peer
// exchange's buffer is read by other GPUs over xGMI from this GPU's memory, and no byte of it may
// wait in this XCD's L2 for the end-of-kernel release (DESIGN.md §5 "Visibility").
__device__ __forceinline__ void pay_store(uint32_t* p, uint32_t x) {
  __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(kPackRowThreads) k_pack(DevView v, const uint64_t* __restrict__ lo,
                                                          const uint64_t* __restrict__ hi,
                                                          const uint32_t* __restrict__ bits, uint64_t ldw,
                                                          uint64_t B, uint32_t W, const int32_t* __restrict__ facts,
                                                          uint32_t* __restrict__ pay) {
  __shared__ uint64_t s_part[kPackRowThreads / 64];
  const uint64_t b = blockIdx.x;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint64_t H = payload_header_words(B);
  if (B == 0) {   // the empty payload: its header alone
    if (t < H) pay_store(&pay[t], t == 0 ? (uint32_t)H : t == 2 ? W : t == 3 ? kPayloadMagic : 0u);
    return;
  }
  // the padded sizes of rows [0, b): every load issued before any is used
  uint64_t before = 0;
  for (uint64_t j0 = 0; j0 < b; j0 += 4 * kPackRowThreads) {
    uint64_t l[4], h[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t j = min(j0 + u * kPackRowThreads + t, B - 1);
      l[u] = lo[j];
      h[u] = hi[j];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      uint32_t d;
      const uint64_t words = pack_row_words(l[u], h[u], v.n, W, d);
      before += (j0 + u * kPackRowThreads + t < b) ? words : 0;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o);
  if (lane == 0) s_part[wv] = before;
  const uint64_t l0 = lo[b], h0 = hi[b];
  uint32_t desc;
  const uint64_t words = pack_row_words(l0, h0, v.n, W, desc);
  __syncthreads();
  uint64_t off = H;
#pragma unroll
  for (int k = 0; k < kPackRowThreads / 64; ++k) off += s_part[k];
  if (t < 3) {   // the row's facts (ORed by the readers' OR pass), zeros without any
    const uint64_t F = payload_facts_at(B);
    pay_store(&pay[F + t * B + b], facts ? (uint32_t)(facts[t * B + b] != 0) : 0u);
  }
  if (t == 0) {
    pay_store(&pay[4 + b], desc);
    pay_store(&pay[4 + B + b], (uint32_t)off);
    if (b == B - 1) {
      pay_store(&pay[0], (uint32_t)(off + words));
      pay_store(&pay[1], (uint32_t)B);
      pay_store(&pay[2], W);
      pay_store(&pay[3], kPayloadMagic);
    }
  }
  if (b == 0) {   // the paddings of the desc / off words and of the facts area
    const uint64_t F = payload_facts_at(B);
    for (uint64_t i = 4 + 2 * B + t; i < F; i += kPackRowThreads) pay_store(&pay[i], 0u);
    for (uint64_t i = F + 3 * B + t; i < H; i += kPackRowThreads) pay_store(&pay[i], 0u);
  }
  const uint32_t count = desc & 0x7FFFFFFFu;
  const bool dense = (desc >> 31) != 0;
  const uint64_t s0 = min(l0, v.n - 1);
  uint32_t* dst = pay + off;
  // up to 8 loads per thread in flight before the stores (W <= 8192 words: one pass); a slice's
  // symbols come from the plain BWT when it is kept, else from E's symbol field -- one source per
  // row (workgroup-uniform), chosen outside the loads so none sits under a branch
  const uint32_t* src32 = dense ? bits + b * ldw : (v.bwt ? v.bwt + s0 : nullptr);
  const uint64_t* srcE = v.E + (dense ? 0 : s0);
  for (uint32_t i0 = 0; i0 < (uint32_t)words; i0 += 8 * kPackRowThreads) {
    uint32_t x[8];
    if (src32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = src32[min(i0 + u * kPackRowThreads + t, count ? count - 1 : 0u)];
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        x[u] = (uint32_t)(srcE[min(i0 + u * kPackRowThreads + t, count ? count - 1 : 0u)] >> kESymShift);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t i = i0 + u * kPackRowThreads + t;
      if (i < (uint32_t)words) pay_store(&dst[i], i < count ? x[u] : 0u);
    }
  }
}

// One workgroup (1024 threads) per row.  Every part's (desc, off) for the row
// is staged in LDS (one round trip), then the dense parts' words (16-B loads,
// eight parts per round: all 8 shards of a wide row are dense) and the first
// 4096 sparse symbols (one flat index space over the parts' lists) load
// together; the words are ORed into the LDS bitmap and the symbols' bits set
// with LDS atomics; the row is stored once, each 16-token chunk by one thread.
// Barriers are LDS-only (s_waitcnt lgkmcnt(0); s_barrier).  (A variant whose
// store waves zero-filled the row while the loads were in flight measured
// slower, 17-56 us against 11-31: profiles/r04_or/.)
//
// PEERS = false: part p is parts + p * stride (an all_gather's output).
// PEERS = true:  part p is ptrs[p], a peer rank's payload buffer mapped over
//                xGMI (fm_ipc_open), of cap words; every load of it is a
//                system-scope (sc0 sc1) load, so no line of an earlier step's
//                payload (double-buffered: the same buffer two steps ago) is
//                served from this GPU's caches.
constexpr int kOrRowThreads = 1024;
constexpr int kOrRowMaxWords = 8 * kOrRowThreads;   // V <= 262144
constexpr int kOrMaxParts = 64;
constexpr int kSysLoadAux = 1 | 16;                 // sc0 sc1

typedef const __attribute__((address_space(1))) uint32_t g32_t;

__device__ __forceinline__ void or_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool PEERS>
__device__ __forceinline__ uint32_t part_word(const uint32_t* base, uint64_t i) {
  g32_t* p = (g32_t*)(base + i);   // a global load, not a flat one (the base may come from LDS)
  if constexpr (PEERS) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else return *p;
}

typedef const __attribute__((address_space(1))) or_v4u g128_t;
typedef const __attribute__((address_space(1))) uint64_t g64_t;

// four consecutive words at a 16-B aligned address (PEERS: two system-scope 8-B loads)
template <bool PEERS>
__device__ __forceinline__ uint4 part_quad(const uint32_t* base, uint64_t i) {
  if constexpr (PEERS) {
    g64_t* p = (g64_t*)(base + i);
    const uint64_t x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t y = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
  } else {
    const or_v4u v = *(g128_t*)(base + i);
    return make_uint4(v.x, v.y, v.z, v.w);
  }
}

constexpr uint32_t kFlagSpins = 1u << 20;   // default flag polls before a step is given up (~0.1-1 s)

constexpr int kOrSym0 = 4;   // 16-B symbol loads per thread issued with the dense words (16 K symbols)
constexpr int kOrSymU = 8;   // per later round (32 K symbols)

// PP (per part): a sparse list is loaded through a workgroup-uniform buffer resource over that
// part's list (16-B loads, 4096 symbols per part and round; past the list's end the descriptor's
// range check returns zeros without a memory request), the (part, round) pairs eight at a time,
// instead of over one flat index space searched per load.  In PEERS mode these are 16-B
// system-scope loads where the flat space needs pairs of 8-B ones.
// The flag wait's acquire.  Every read of a peer's payload below is a system-scope load (sc0 sc1:
// part_word / part_quad are system-scope atomic loads, the buffer loads carry kSysLoadAux), each
// coherent for its location at the system's coherence point, and each issued only after wave 0's
// poll has returned the step (the loop's exit depends on the polled values; the other waves pass
// the workgroup barrier after it).  The peers' payload stores were write-through and acknowledged
// before their release and flag store.  So the data is read from where the peer put
// it, and an acquire fence adds only its cache maintenance -- a system-scope `buffer_inv sc0 sc1`
// in every workgroup, invalidating the XCD's L2 each time: 12 µs of a B = 2048 world-1 step
// (69.8 -> 57.8 µs; B = 256 20.2 -> 18.6; profiles/r06_or/).  FMIDX_OR_ACQUIRE=1 restores the fence
// (measurement variant).
#ifndef FMIDX_OR_ACQUIRE
#define FMIDX_OR_ACQUIRE 0
#endif
template <bool PEERS, bool PP, int T>
__global__ void __launch_bounds__(T) k_or_rows(const uint32_t* __restrict__ parts,
                                                            const uint64_t* __restrict__ ptrs, uint32_t nparts,
                                                            uint64_t stride, uint64_t B, uint32_t W, uint64_t vocab,
                                                            int64_t shift, void* __restrict__ out, uint64_t ld,
                                                            int unpack, const uint32_t* __restrict__ flags,
                                                            const uint32_t* __restrict__ ctr, uint32_t spins,
                                                            uint32_t* __restrict__ err, int32_t* __restrict__ facts_out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t s_bits[];   // [round4(W)]
  // per part: its sparse count (0 for dense parts), data offset, and first 16-B slot in the
  // flat space of every sparse list padded to a multiple of 4 words
  __shared__ uint32_t s_cnt[kOrMaxParts], s_off[kOrMaxParts], s_pre[kOrMaxParts + 1], s_dense[kOrMaxParts];
  __shared__ uint64_t s_base[PEERS ? kOrMaxParts : 1];
  __shared__ uint32_t s_nd, s_nq;
  const uint64_t b = blockIdx.x;
  const uint32_t t = threadIdx.x;
  auto base_of = [&](uint32_t p) -> const uint32_t* {
    if constexpr (PEERS) return reinterpret_cast<const uint32_t*>(s_base[p]);
    else return parts + (uint64_t)p * stride;
  };
  const uint32_t W4 = (W + 3) / 4;
  for (uint32_t w4 = t; w4 < W4; w4 += T) reinterpret_cast<uint4*>(s_bits)[w4] = make_uint4(0, 0, 0, 0);
  if (t < 64) {
    const uint64_t* tab = ptrs;
    if (PEERS && flags) {
      // the device-side barrier (PeerExchange "flags"): every rank has stored this step's number
      // into its word of this rank's flag array once its payload was complete (k_peer_signal,
      // after the kernel that wrote it).  The step number is this rank's device counter, which
      // its own signal kernel advanced just before this pass (stream order), so one captured
      // step replays for every step; its parity picks the payload buffer the step wrote
      // (ptrs = buffer 0's addresses, then buffer 1's).  Wave 0 waits for all of them
      // (system-scope loads: the words are written over xGMI), bounded: past `spins` polls the
      // step is recorded in *err (host-visible: a system-scope store) and the pass goes on, so
      // the grid always drains -- the host raises on the recorded step.
      const uint32_t want = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tab = ptrs + ((want - 1u) & 1u) * nparts;
      bool ok = t >= nparts;
      for (uint32_t it = 0; it < spins && !__all(ok); ++it) {
        if (!ok) ok = (int32_t)(__hip_atomic_load(flags + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - want) >= 0;
        if (!__all(ok)) __builtin_amdgcn_s_sleep(4);
      }
      if (!__all(ok) && t == 0) __hip_atomic_store(err, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      // the peers' payload stores, released before their flag stores, are read below by
      // system-scope loads only, issued after this poll (see FMIDX_OR_ACQUIRE)
      if (FMIDX_OR_ACQUIRE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    // wave 0 stages every part's (desc, off) and scans them in registers (nparts <= 64).  A row
    // whose data lies past the part's end (a gather shorter than the payload: the speculative
    // all_gather of SparseExchange, redone in full when it was too short) is read as empty --
    // never beyond the part
    uint32_t d = 0, o = 0, f[3] = {0u, 0u, 0u};
    const uint32_t* pp = nullptr;
    const uint64_t F = payload_facts_at(B);
    if (t < nparts) {
      pp = PEERS ? reinterpret_cast<const uint32_t*>(tab[t]) : parts + (uint64_t)t * stride;
      d = part_word<PEERS>(pp, 4 + b);
      o = part_word<PEERS>(pp, 4 + B + b);
      if (facts_out) {   // the row's facts, in the same round trip (the header is within every part)
#pragma unroll
        for (int k = 0; k < 3; ++k) f[k] = part_word<PEERS>(pp, F + (uint64_t)k * B + b);
      }
      const uint64_t end = (uint64_t)o + (((d & 0x7FFFFFFFu) + 3u) & ~3u);
      if (!(o >= payload_header_words(B) && end <= stride)) d = o = 0;
    }
    if (facts_out) {   // OR over the parts: some shard has it
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const bool any = __ballot(t < nparts && f[k] != 0) != 0;
        if (t == 0) facts_out[(uint64_t)k * B + b] = any ? 1 : 0;
      }
    }
    const bool dense = (d >> 31) != 0;
    const uint32_t q = dense ? 0u : (d + 3u) >> 2;
    uint32_t inc = q;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const uint32_t y = __shfl_up(inc, k, 64);
      if (t >= (uint32_t)k) inc += y;
    }
    const uint64_t dm = __ballot(dense);
    if (t < nparts) {
      s_cnt[t] = dense ? 0u : d;
      s_off[t] = o;
      s_pre[t] = inc - q;
      if (dense) s_dense[__popcll(dm & ((1ull << t) - 1))] = t;
      if constexpr (PEERS) s_base[t] = reinterpret_cast<uint64_t>(pp);
    }
    const uint32_t tot = __shfl(inc, (int)(nparts - 1), 64);
    uint32_t mq = q;                                    // the longest list, in 16-B quads
#pragma unroll
    for (int k = 32; k; k >>= 1) mq = max(mq, (uint32_t)__shfl_xor(mq, k, 64));
    if (t == 0) {
      s_pre[nparts] = tot;
      s_nd = (uint32_t)__popcll(dm);
      s_nq = (mq + T - 1) / T;
    }
  }
  or_lds_barrier();
  const uint32_t nd = s_nd;
  const uint32_t total4 = s_pre[nparts];   // 16-B slots of sparse symbols
  // the 16-B slot j of the flat space: its part and its four symbols
  auto quad_at = [&](uint32_t j, uint32_t& p) -> uint4 {
    p = 0;                                              // the last part whose first slot is <= j
    for (uint32_t step = kOrMaxParts / 2; step; step >>= 1)
      if (p + step <= nparts - 1 && s_pre[p + step] <= j) p += step;
    return part_quad<PEERS>(base_of(p), s_off[p] + 4ull * (j - s_pre[p]));
  };
  auto set_quad = [&](uint32_t j, uint32_t p, const uint4& x) {
    const uint32_t k0 = 4 * (j - s_pre[p]), cnt = s_cnt[p];
    const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t tok = (int64_t)xs[e] - shift;
      if (j < total4 && k0 + e < cnt && tok >= 0 && (uint64_t)tok < vocab)
        atomicOr(&s_bits[tok >> 5], 1u << (tok & 31));
    }
  };
  // PP: (part, round) pair j = k * nparts + p covers quads [k * 1024, (k + 1) * 1024) of part p's list
  const uint32_t npairs = nparts * s_nq;
  auto pair_load = [&](uint32_t j) -> or_v4u {
    const uint32_t k = j / nparts, p = j - k * nparts;
    const uint32_t bytes = j < npairs ? 4u * ((s_cnt[p] + 3u) & ~3u) : 0u;   // dense parts: 0, no request
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(base_of(p) + s_off[p], bytes);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * (t + k * T), 0, PEERS ? kSysLoadAux : 0);
  };
  auto pair_set = [&](uint32_t j, const or_v4u& x) {
    if (j >= npairs) return;                             // workgroup-uniform
    const uint32_t k = j / nparts, p = j - k * nparts;
    const uint32_t i0 = 4 * (t + k * T), cnt = s_cnt[p];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t tok = (int64_t)x[e] - shift;
      if (i0 + e < cnt && tok >= 0 && (uint64_t)tok < vocab) atomicOr(&s_bits[tok >> 5], 1u << (tok & 31));
    }
  };
  constexpr int kPP = T >= 1024 ? 8 : 4;                 // (part, round) pairs per round trip
  or_v4u pq0[PP ? kPP : 1];
  if constexpr (PP) {
#pragma unroll
    for (int u = 0; u < kPP; ++u) pq0[u] = pair_load((uint32_t)u);
  }
  // flat space: the first 16 K sparse symbols, loaded with the first dense round
  uint4 sq0[PP ? 1 : kOrSym0];
  uint32_t sp0[PP ? 1 : kOrSym0];
  if constexpr (!PP) {
#pragma unroll
    for (int u = 0; u < kOrSym0; ++u) {
      sp0[u] = 0;
      sq0[u] = total4 ? quad_at(min(u * T + t, total4 - 1), sp0[u]) : make_uint4(0, 0, 0, 0);
    }
  }
  constexpr int kSlots4 = kOrRowMaxWords / (4 * T);   // W <= 8192 words
  const uint32_t slots = (W4 + T - 1) / T;
  uint4 acc[kSlots4];
#pragma unroll
  for (int k = 0; k < kSlots4; ++k) acc[k] = make_uint4(0u, 0u, 0u, 0u);
  constexpr int kPB = T >= 1024 ? 8 : 1;                // dense parts per round trip (registers: kPB x kSlots4)
  for (uint32_t j0 = 0; j0 < nd; j0 += kPB) {
    uint4 x[kPB][kSlots4];
#pragma unroll
    for (int q = 0; q < kPB; ++q) {
      const uint32_t p = s_dense[min(j0 + q, nd - 1)];   // past the last: the last again (harmless for an OR)
      const uint32_t* src = base_of(p) + s_off[p];
      if constexpr (PEERS) {
        // workgroup-uniform part: one buffer resource over the row's W words
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, 16u * W4);
#pragma unroll
        for (int k = 0; k < kSlots4; ++k) {
          if ((uint32_t)k < slots) {
            const or_v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16u * min(t + k * T, W4 - 1), 0,
                                                                   kSysLoadAux);
            x[q][k] = make_uint4(v.x, v.y, v.z, v.w);
          } else {
            x[q][k] = make_uint4(0, 0, 0, 0);
          }
        }
      } else {
        const uint4* s4 = reinterpret_cast<const uint4*>(src);
#pragma unroll
        for (int k = 0; k < kSlots4; ++k)
          x[q][k] = (uint32_t)k < slots ? s4[min(t + k * T, W4 - 1)] : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < kPB; ++q)
#pragma unroll
      for (int k = 0; k < kSlots4; ++k) {
        acc[k].x |= x[q][k].x;
        acc[k].y |= x[q][k].y;
        acc[k].z |= x[q][k].z;
        acc[k].w |= x[q][k].w;
      }
  }
  if (nd) {
#pragma unroll
    for (int k = 0; k < kSlots4; ++k) {
      const uint32_t w4 = t + k * T;
      if (w4 < W4) reinterpret_cast<uint4*>(s_bits)[w4] = acc[k];
    }
  }
  // the dense words are in place before any symbol's bit is ORed in (other waves' words may
  // share a symbol's word)
  or_lds_barrier();
  if constexpr (PP) {
#pragma unroll
    for (int u = 0; u < kPP; ++u) pair_set((uint32_t)u, pq0[u]);
    for (uint32_t j0 = kPP; j0 < npairs; j0 += kPP) {   // more parts, or lists past 4096 symbols
      or_v4u pq[kPP];
#pragma unroll
      for (int u = 0; u < kPP; ++u) pq[u] = pair_load(j0 + (uint32_t)u);
#pragma unroll
      for (int u = 0; u < kPP; ++u) pair_set(j0 + (uint32_t)u, pq[u]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < kOrSym0; ++u) set_quad(u * T + t, sp0[u], sq0[u]);
    for (uint32_t j0 = kOrSym0 * T; j0 < total4; j0 += kOrSymU * T) {   // long lists
      uint4 sq[kOrSymU];
      uint32_t sp[kOrSymU];
#pragma unroll
      for (int u = 0; u < kOrSymU; ++u) sq[u] = quad_at(min(j0 + u * T + t, total4 - 1), sp[u]);
#pragma unroll
      for (int u = 0; u < kOrSymU; ++u) set_quad(j0 + u * T + t, sp[u], sq[u]);
    }
  }
  or_lds_barrier();
  if (!unpack) {
    uint32_t* o = static_cast<uint32_t*>(out) + b * (ld / 4);
    for (uint32_t w = t; w < W; w += T) o[w] = s_bits[w];
    return;
  }
  uint8_t* row = static_cast<uint8_t*>(out) + b * ld;
  const __amdgpu_buffer_rsrc_t r = make_rsrc(row, (uint32_t)vocab);
  const bool aligned = (reinterpret_cast<uintptr_t>(row) & 15) == 0;
  const uint32_t nch = (uint32_t)((vocab + 15) / 16);
  for (uint32_t c = t; c < nch; c += T) {
    const uint64_t t0 = 16ull * c;
    const uint32_t bits16 = (s_bits[c >> 1] >> (16 * (c & 1))) & 0xFFFFu;
    uint32_t q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = (((bits16 >> (4 * i)) & 0xFu) * 0x204081u) & 0x01010101u;
    if (t0 + 16 <= vocab && aligned) {
      or_v4u vv = {q[0], q[1], q[2], q[3]};
      __builtin_amdgcn_raw_buffer_store_b128(vv, r, (uint32_t)t0, 0, kOrStoreAux);
    } else {
      for (uint64_t i = 0; i < 16 && t0 + i < vocab; ++i) row[t0 + i] = (bits16 >> i) & 1u;
    }
  }
}

}  // namespace

// the OR pass's sparse lists per part (1, the default) or over one flat index space (0): a
// measurement variant (make ... VFLAGS=-DFMIDX_OR_PERPART=0; tools/or_perpart_ab.sh)
#ifndef FMIDX_OR_PERPART
#define FMIDX_OR_PERPART 1
#endif
static bool or_per_part() { return FMIDX_OR_PERPART != 0; }

// Workgroup size of the OR pass by batch, as the decode kernel's (decode_threads): one 1024-thread
// workgroup per row while the rows fit one per CU (the 128-KB uint8 row wants all 16 waves' store
// issue); beyond that 256 threads, so that several rows' round-trip chains -- flag poll, header,
// payload data -- overlap on each CU instead of running one row per CU per round.
// FMIDX_OR_THREADS (measurement variant): 1024 or 256 for every batch.
#ifndef FMIDX_OR_THREADS
#define FMIDX_OR_THREADS 0
#endif
static uint32_t or_threads(uint64_t B) {
  if (FMIDX_OR_THREADS == 1024 || FMIDX_OR_THREADS == 256) return FMIDX_OR_THREADS;
  return B <= 256 ? 1024u : 256u;
}

uint64_t shard_payload_capacity(uint64_t B, uint64_t vocab) {
  const uint64_t W = (vocab + 31) / 32;
  return payload_header_words(B) + B * ((W + 3) & ~3ull);
}

int launch_shard_pack(const DevView& v, const uint64_t* lo, const uint64_t* hi, uint64_t B, const uint32_t* bits,
                      uint64_t ldw, uint64_t vocab, const int32_t* facts, uint32_t* pay, uint64_t cap, hipStream_t s) {
  const uint64_t W = (vocab + 31) / 32;
  if (!lo || !hi || !pay || (B && !bits) || ldw < W || B >= (1ull << 31) ||
      W > (uint64_t)kOrRowMaxWords) {
    set_error("shard_pack: bad arguments (B %llu, vocab %llu, ld %llu words)", (unsigned long long)B,
              (unsigned long long)vocab, (unsigned long long)ldw);
    return -1;
  }
  if (cap < shard_payload_capacity(B, vocab) || cap >= (1ull << 32)) {
    set_error("shard_pack: payload of %llu words, %llu needed (< 2^32)", (unsigned long long)cap,
              (unsigned long long)shard_payload_capacity(B, vocab));
    return -1;
  }
  k_pack<<<(unsigned)(B ? B : 1), kPackRowThreads, 0, s>>>(v, lo, hi, bits, ldw, B, (uint32_t)W, facts, pay);
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_shard_or_rows(const uint32_t* parts, uint64_t nparts, uint64_t stride, uint64_t B, uint64_t vocab,
                         int64_t shift, void* out, uint64_t ld, int unpack, int32_t* facts_out, hipStream_t s) {
  const uint64_t W = (vocab + 31) / 32;
  if (!parts || !out || !nparts || nparts > (uint64_t)kOrMaxParts || W > (uint64_t)kOrRowMaxWords ||
      stride < payload_header_words(B) ||
      (unpack ? ld < vocab : (ld < 4 * W || ld % 4))) {
    set_error("shard_or_rows: bad arguments (parts %llu, stride %llu, vocab %llu, ld %llu)",
              (unsigned long long)nparts, (unsigned long long)stride, (unsigned long long)vocab,
              (unsigned long long)ld);
    return -1;
  }
  if (B == 0) return 0;
  const bool aligned = (reinterpret_cast<uintptr_t>(parts) & 15) == 0 && stride % 4 == 0;
  if (!aligned) {
    set_error("shard_or_rows: the payloads must start on 16-B boundaries (stride a multiple of 4 words)");
    return -1;
  }
#define FM_OR_LAUNCH(PP, TT)                                                                                  \
  k_or_rows<false, PP, TT><<<(unsigned)B, TT, (W + 3) / 4 * 16, s>>>(parts, nullptr, (uint32_t)nparts, stride, B,     \
                                                                     (uint32_t)W, vocab, shift, out, ld, unpack,       \
                                                                     nullptr, nullptr, 0, nullptr, facts_out)
  if (or_threads(B) == 1024) {
    if (or_per_part()) FM_OR_LAUNCH(true, 1024);
    else FM_OR_LAUNCH(false, 1024);
  } else {
    if (or_per_part()) FM_OR_LAUNCH(true, 256);
    else FM_OR_LAUNCH(false, 256);
  }
#undef FM_OR_LAUNCH
  FM_HIP(hipGetLastError());
  return 0;
}

int launch_shard_or_rows_peers(const uint64_t* ptrs, uint64_t nparts, uint64_t cap, uint64_t B, uint64_t vocab,
                               int64_t shift, void* out, uint64_t ld, int unpack, const uint32_t* flags,
                               const uint32_t* ctr, uint32_t spins, uint32_t* err, int32_t* facts_out,
                               hipStream_t s) {
  const uint64_t W = (vocab + 31) / 32;
  if (!ptrs || !out || !nparts || nparts > (uint64_t)kOrMaxParts || W > (uint64_t)kOrRowMaxWords ||
      cap < shard_payload_capacity(B, vocab) || cap >= (1ull << 30) ||
      (unpack ? ld < vocab : (ld < 4 * W || ld % 4))) {
    set_error("shard_or_rows_peers: bad arguments (parts %llu, cap %llu words, vocab %llu, ld %llu)",
              (unsigned long long)nparts, (unsigned long long)cap, (unsigned long long)vocab,
              (unsigned long long)ld);
    return -1;
  }
  if (B == 0) return 0;
  if (flags && (!err || !ctr)) {
    set_error("shard_or_rows_peers: a flag barrier needs a step counter and an error word");
    return -1;
  }
  if (!spins) spins = kFlagSpins;
#define FM_OR_LAUNCH(PP, TT)                                                                                  \
  k_or_rows<true, PP, TT><<<(unsigned)B, TT, (W + 3) / 4 * 16, s>>>(nullptr, ptrs, (uint32_t)nparts, cap, B,           \
                                                                    (uint32_t)W, vocab, shift, out, ld, unpack, flags, \
                                                                    ctr, spins, err, facts_out)
  if (or_threads(B) == 1024) {
    if (or_per_part()) FM_OR_LAUNCH(true, 1024);
    else FM_OR_LAUNCH(false, 1024);
  } else {
    if (or_per_part()) FM_OR_LAUNCH(true, 256);
    else FM_OR_LAUNCH(false, 256);
  }
#undef FM_OR_LAUNCH
  FM_HIP(hipGetLastError());
  return 0;
}

namespace {
// the flag barrier's signal: the step number is this rank's device counter plus one (the
// counter advances here, so a captured step replays for every step); after a system-scope
// release -- the payload the previous kernel on this stream wrote is visible at system scope
// before any flag says so -- lane r stores it into rank r's flag word for this rank (an address
// in rank r's memory, mapped over xGMI) with a system-scope (sc0 sc1) vector store.  world = 0
// advances the counter and posts nothing (the timeout path's tests).
__global__ void __launch_bounds__(64) k_peer_signal(const uint64_t* __restrict__ dst, uint32_t world,
                                                    uint32_t* __restrict__ ctr) {
  const uint32_t t = threadIdx.x;
  const uint32_t value = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (t < world)
    __hip_atomic_store(reinterpret_cast<uint32_t*>(dst[t]), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t == 0) __hip_atomic_store(ctr, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

int launch_peer_signal(const uint64_t* dst, uint64_t world, uint32_t* ctr, hipStream_t s) {
  if (!ctr || (world && !dst) || world > 64) {
    set_error("peer_signal: 0..64 flag addresses and a step counter");
    return -1;
  }
  k_peer_signal<<<1, 64, 0, s>>>(dst, (uint32_t)world, ctr);
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
