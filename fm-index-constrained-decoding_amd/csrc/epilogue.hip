// epilogue.hip -- fused logits-processor epilogue.
//
// Replaces the per-row mask assembly of the reference processors
// (document_constrained_generation_causal_qwen.py:151-214, and the hard-mask
// variants ..._vllm.py:102-137, ..._seq.py:268-303):
//     mask = full_like(scores, base)            # 0.0 (soft) or -inf (hard)
//     mask[row, all_unigrams]           = v_uni     (unigram rows / the rest)
//     mask[row, distinct]               = v_dist    (allowed continuations)
//     mask[row, eos]                    = v_eos     (always_allow_eos)
//     return scores + mask
// as one streaming pass over scores: read a row chunk, decide each token's
// mask value from the allowed-token bit row (produced by the decode/mask
// kernel), the all_unigrams bit row and per-row parameters, add in the
// scores dtype, store.  Per-row values are supplied already rounded to the
// scores dtype (as torch rounds a Python float on assignment), and the add is
// done exactly like torch's (fp32 add; bf16/fp16 via fp32 then RNE), so the
// output is bit-identical, -0.0 + 0.0 == +0.0 included.
#include "fmidx_internal.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

namespace fmidx {

namespace {

constexpr int kEpiThreads = 256;

// row flags
constexpr uint32_t kUseBits = 1u;      // allowed tokens from the bit row
constexpr uint32_t kUnigram = 2u;      // all_unigrams get v_uni
constexpr uint32_t kEos = 4u;          // eos gets v_eos (last, overrides)
constexpr uint32_t kSpecial = 8u;      // the single token `special` is the distinct set

struct RowParams {
  float base, v_dist, v_uni, v_eos;
  uint32_t flags;
  int32_t pad;
  int64_t special;
};

template <typename T>
__device__ __forceinline__ float to_f(T x);
template <>
__device__ __forceinline__ float to_f<float>(float x) { return x; }
template <>
__device__ __forceinline__ float to_f<__hip_bfloat16>(__hip_bfloat16 x) { return __bfloat162float(x); }
template <>
__device__ __forceinline__ float to_f<__half>(__half x) { return __half2float(x); }

template <typename T>
__device__ __forceinline__ T from_f(float x);
template <>
__device__ __forceinline__ float from_f<float>(float x) { return x; }
template <>
__device__ __forceinline__ __hip_bfloat16 from_f<__hip_bfloat16>(float x) { return __float2bfloat16(x); }
template <>
__device__ __forceinline__ __half from_f<__half>(float x) { return __float2half(x); }

// mask value of token t = t0 + k (dbits / ubits: the thread's tokens' allowed /
// unigram bits), in the reference's assignment order: base, all_unigrams,
// distinct, eos
__device__ __forceinline__ float mask_value(const RowParams& p, uint32_t k, uint64_t t, uint32_t dbits,
                                            uint32_t ubits, int64_t eos) {
  float m = p.base;
  if ((ubits >> k) & 1u) m = p.v_uni;
  bool dist = (dbits >> k) & 1u;
  if ((p.flags & kSpecial) && (int64_t)t == p.special) dist = true;
  if (dist) m = p.v_dist;
  if ((p.flags & kEos) && (int64_t)t == eos) m = p.v_eos;
  return m;
}

template <typename T>
__device__ __forceinline__ uint32_t add16(uint32_t h, float m) {   // one 16-bit element, as bits
  const T x = __builtin_bit_cast(T, (unsigned short)h);
  return (uint32_t)__builtin_bit_cast(unsigned short, from_f<T>(to_f<T>(x) + m));
}

// One thread = 8 consecutive tokens t0 = 8 j .. t0 + 7 of one row (blockIdx.y
// strides the rows, so no division): their allowed and unigram bits are one
// byte of the rows' bit words, and when both row bases are 16-B aligned the
// scores move as 32 B (f32: two uint4) or 16 B (bf16 / f16: one uint4) per
// thread -- hipcc does not vectorize 16-bit scalar accesses
// (cdna_hip_programming.md Guideline 13).  (32 B per thread for the 16-bit
// types measured slower: 26.4 against 24.5 us at 256 x 128256.)  Row tails and
// unaligned rows take the scalar path.  Same arithmetic either way: the f32
// add, then the dtype's round to nearest even.
template <typename T>
__global__ void __launch_bounds__(kEpiThreads) k_epilogue(const T* __restrict__ scores, T* __restrict__ out,
                                                         uint32_t B, uint32_t V, uint64_t lds, uint64_t ldo,
                                                         const uint32_t* __restrict__ bits, uint64_t ldb,
                                                         const uint32_t* __restrict__ uni,
                                                         const RowParams* __restrict__ rp, int64_t eos) {
  const uint32_t per_row = (V + 7) / 8;
  for (uint32_t b = blockIdx.y; b < B; b += gridDim.y) {
    const RowParams p = rp[b];
    const T* s = scores + (uint64_t)b * lds;
    T* o = out + (uint64_t)b * ldo;
    const uint32_t* brow = ((p.flags & kUseBits) && bits) ? bits + (uint64_t)b * ldb : nullptr;
    const uint32_t* urow = ((p.flags & kUnigram) && uni) ? uni : nullptr;
    const bool vec = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(o)) & 15) == 0;
    for (uint32_t j = blockIdx.x * kEpiThreads + threadIdx.x; j < per_row; j += gridDim.x * kEpiThreads) {
      const uint32_t t0 = 8 * j;
      const uint32_t dbits = brow ? (brow[t0 >> 5] >> (t0 & 31)) & 0xFFu : 0u;
      const uint32_t ubits = urow ? (urow[t0 >> 5] >> (t0 & 31)) & 0xFFu : 0u;
      if (vec && t0 + 8 <= V) {
        if constexpr (sizeof(T) == 4) {
          const uint4 a = *reinterpret_cast<const uint4*>(s + t0);
          const uint4 c = *reinterpret_cast<const uint4*>(s + t0 + 4);
          uint32_t w[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
#pragma unroll
          for (uint32_t k = 0; k < 8; ++k)
            w[k] = __float_as_uint(__uint_as_float(w[k]) + mask_value(p, k, t0 + k, dbits, ubits, eos));
          *reinterpret_cast<uint4*>(o + t0) = make_uint4(w[0], w[1], w[2], w[3]);
          *reinterpret_cast<uint4*>(o + t0 + 4) = make_uint4(w[4], w[5], w[6], w[7]);
        } else {
          const uint4 a = *reinterpret_cast<const uint4*>(s + t0);
          uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
          for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t lo = add16<T>(w[q] & 0xFFFFu, mask_value(p, 2 * q, t0 + 2 * q, dbits, ubits, eos));
            const uint32_t hi = add16<T>(w[q] >> 16, mask_value(p, 2 * q + 1, t0 + 2 * q + 1, dbits, ubits, eos));
            w[q] = lo | (hi << 16);
          }
          *reinterpret_cast<uint4*>(o + t0) = make_uint4(w[0], w[1], w[2], w[3]);
        }
      } else {
        for (uint32_t k = 0; k < 8 && t0 + k < V; ++k)
          o[t0 + k] = from_f<T>(to_f<T>(s[t0 + k]) + mask_value(p, k, t0 + k, dbits, ubits, eos));
      }
    }
  }
}

}  // namespace

int launch_epilogue(int dtype, const void* scores, void* out, uint64_t B, uint64_t V, uint64_t lds,
                    uint64_t ldo, const uint32_t* bits, uint64_t ldb, const uint32_t* uni,
                    const void* row_params, int64_t eos, hipStream_t s) {
  if (B == 0 || V == 0) return 0;
  if (B >= (1ull << 32) || V >= (1ull << 32) - 8) {
    set_error("apply_boosts: B = %llu, V = %llu exceed 2^32", (unsigned long long)B, (unsigned long long)V);
    return -1;
  }
  const uint64_t per_row = (V + 7) / 8;
  const dim3 grid((unsigned)std::min<uint64_t>((per_row + kEpiThreads - 1) / kEpiThreads, 1024),
                  (unsigned)std::min<uint64_t>(B, 65535));
  const RowParams* rp = reinterpret_cast<const RowParams*>(row_params);
  switch (dtype) {
    case 0:
      k_epilogue<float><<<grid, kEpiThreads, 0, s>>>(reinterpret_cast<const float*>(scores),
                                                     reinterpret_cast<float*>(out), B, V, lds, ldo, bits, ldb,
                                                     uni, rp, eos);
      break;
    case 1:
      k_epilogue<__hip_bfloat16><<<grid, kEpiThreads, 0, s>>>(
          reinterpret_cast<const __hip_bfloat16*>(scores), reinterpret_cast<__hip_bfloat16*>(out), B, V, lds, ldo,
          bits, ldb, uni, rp, eos);
      break;
    case 2:
      k_epilogue<__half><<<grid, kEpiThreads, 0, s>>>(reinterpret_cast<const __half*>(scores),
                                                      reinterpret_cast<__half*>(out), B, V, lds, ldo, bits, ldb,
                                                      uni, rp, eos);
      break;
    default:
      set_error("unsupported scores dtype code %d", dtype);
      return -1;
  }
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
