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

__device__ __forceinline__ bool bit_at(const uint32_t* row, uint64_t t) {
  return (row[t >> 5] >> (t & 31)) & 1u;
}

// One thread = 8 consecutive tokens of one row.
template <typename T>
__global__ void __launch_bounds__(kEpiThreads) k_epilogue(const T* __restrict__ scores, T* __restrict__ out,
                                                         uint64_t B, uint64_t V, uint64_t lds, uint64_t ldo,
                                                         const uint32_t* __restrict__ bits, uint64_t ldb,
                                                         const uint32_t* __restrict__ uni,
                                                         const RowParams* __restrict__ rp, int64_t eos) {
  const uint64_t per_row = (V + 7) / 8;
  const uint64_t total = B * per_row;
  for (uint64_t g = (uint64_t)blockIdx.x * kEpiThreads + threadIdx.x; g < total;
       g += (uint64_t)gridDim.x * kEpiThreads) {
    const uint64_t b = g / per_row;
    const uint64_t t0 = (g - b * per_row) * 8;
    const RowParams p = rp[b];
    const T* s = scores + b * lds;
    T* o = out + b * ldo;
    const uint32_t* brow = bits ? bits + b * ldb : nullptr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t t = t0 + j;
      if (t >= V) break;
      float m = p.base;
      if ((p.flags & kUnigram) && uni && bit_at(uni, t)) m = p.v_uni;
      bool dist = false;
      if ((p.flags & kUseBits) && brow) dist = bit_at(brow, t);
      if ((p.flags & kSpecial) && (int64_t)t == p.special) dist = true;
      if (dist) m = p.v_dist;
      if ((p.flags & kEos) && (int64_t)t == eos) m = p.v_eos;
      o[t] = from_f<T>(to_f<T>(s[t]) + m);
    }
  }
}

}  // namespace

int launch_epilogue(int dtype, const void* scores, void* out, uint64_t B, uint64_t V, uint64_t lds,
                    uint64_t ldo, const uint32_t* bits, uint64_t ldb, const uint32_t* uni,
                    const void* row_params, int64_t eos, hipStream_t s) {
  if (B == 0 || V == 0) return 0;
  const uint64_t work = B * ((V + 7) / 8);
  const unsigned grid = (unsigned)std::min<uint64_t>((work + kEpiThreads - 1) / kEpiThreads, 8192);
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
