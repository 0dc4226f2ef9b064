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

// one thread per 16 tokens: half a word of every part, one 16-B store
__global__ void __launch_bounds__(kThreads) k_or_unpack(const uint32_t* __restrict__ parts, uint32_t nparts,
                                                        uint64_t part_stride, uint64_t B, uint64_t wpr,
                                                        uint64_t vocab, uint8_t* __restrict__ out, uint64_t ld) {
  const uint64_t chunks = (vocab + 15) / 16;
  const uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint64_t b = g / chunks, k = g - b * chunks;
  if (b >= B) return;
  const uint64_t w = k >> 1;
  const uint32_t x = or_parts(parts, nparts, part_stride, b * wpr + w);
  const uint32_t bits = (k & 1) ? (x >> 16) : (x & 0xFFFFu);
  uint8_t* o = out + b * ld + k * 16;
  const uint64_t t0 = k * 16;
  if (t0 + 16 <= vocab && ((reinterpret_cast<uintptr_t>(o) & 15) == 0)) {
    uint32_t q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = (((bits >> (4 * j)) & 0xFu) * 0x204081u) & 0x01010101u;
    *reinterpret_cast<uint4*>(o) = make_uint4(q[0], q[1], q[2], q[3]);
  } else {
    for (uint64_t j = 0; j < 16 && t0 + j < vocab; ++j) o[j] = (bits >> j) & 1u;
  }
}

__global__ void __launch_bounds__(kThreads) k_or_words(const uint32_t* __restrict__ parts, uint32_t nparts,
                                                       uint64_t part_stride, uint64_t B, uint64_t wpr,
                                                       uint32_t* __restrict__ out, uint64_t ldw) {
  const uint64_t g = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
  const uint64_t b = g / wpr, w = g - b * wpr;
  if (b >= B) return;
  out[b * ldw + w] = or_parts(parts, nparts, part_stride, b * wpr + w);
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
    const uint64_t threads = B * ((vocab + 15) / 16);
    k_or_unpack<<<(unsigned)((threads + kThreads - 1) / kThreads), kThreads, 0, s>>>(
        parts, (uint32_t)nparts, part_stride, B, wpr, vocab, static_cast<uint8_t*>(out), ld_out);
  } else {
    if (ld_out % 4 || ld_out < wpr * 4) {
      set_error("or_bits: packed output rows need ld >= 4 * words and a multiple of 4");
      return -1;
    }
    const uint64_t threads = B * wpr;
    k_or_words<<<(unsigned)((threads + kThreads - 1) / kThreads), kThreads, 0, s>>>(
        parts, (uint32_t)nparts, part_stride, B, wpr, static_cast<uint32_t*>(out), ld_out / 4);
  }
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
