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

}  // namespace fmidx
