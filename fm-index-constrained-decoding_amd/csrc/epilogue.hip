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

#include <cstdlib>

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

template <typename T>
__device__ __forceinline__ uint32_t add16(uint32_t h, float m) {   // one 16-bit element, as bits
  const T x = __builtin_bit_cast(T, (unsigned short)h);
  return (uint32_t)__builtin_bit_cast(unsigned short, from_f<T>(to_f<T>(x) + m));
}

// A row's mask values and rules as uniform constants.  The mask value of a
// token follows the reference's assignment order -- base, all_unigrams,
// distinct (the allowed bits, plus `special`), eos -- and is selected with
// bit operations on the four values' f32 bits (a select between struct
// fields was compiled as an LDS copy of the struct and an indexed read per
// token).  eos and `special` are found by chunk index, not by a 64-bit
// compare per token.
struct RowSel {
  uint32_t fb, fu, fd, fe;   // base, v_uni, v_dist, v_eos (f32 bits)
  uint32_t dm, um;           // 0xFF if the allowed / unigram bits apply, else 0
  uint32_t je, eb;           // chunk holding eos and its bit (je = ~0: none)
  uint32_t js, sb;           // the same for `special`
};

__device__ __forceinline__ RowSel row_sel(const RowParams& p, uint32_t V, int64_t eos) {
  RowSel r;
  r.fb = __float_as_uint(p.base);
  r.fu = __float_as_uint(p.v_uni);
  r.fd = __float_as_uint(p.v_dist);
  r.fe = __float_as_uint(p.v_eos);
  r.dm = (p.flags & kUseBits) ? 0xFFu : 0u;
  r.um = (p.flags & kUnigram) ? 0xFFu : 0u;
  const bool he = (p.flags & kEos) && eos >= 0 && eos < (int64_t)V;
  r.je = he ? (uint32_t)(eos >> 3) : ~0u;
  r.eb = he ? 1u << (uint32_t)(eos & 7) : 0u;
  const bool hs = (p.flags & kSpecial) && p.special >= 0 && p.special < (int64_t)V;
  r.js = hs ? (uint32_t)(p.special >> 3) : ~0u;
  r.sb = hs ? 1u << (uint32_t)(p.special & 7) : 0u;
  return r;
}

// Chunk j (tokens 8 j .. 8 j + 7): bit k of H = "token k gets v_dist or
// v_eos", bit k of L = "the upper value of its pair" (v_eos over v_dist,
// v_uni over base).  dw / uw: the bit words holding the chunk's byte.
__device__ __forceinline__ void chunk_codes(const RowSel& r, uint32_t j, uint32_t dw, uint32_t uw, uint32_t& H,
                                            uint32_t& L) {
  const uint32_t sh = (8 * j) & 31u;
  const uint32_t d = ((dw >> sh) & r.dm) | (j == r.js ? r.sb : 0u);
  const uint32_t u = (uw >> sh) & r.um;
  const uint32_t e = j == r.je ? r.eb : 0u;
  H = d | e;
  L = e | (u & ~H);
}

__device__ __forceinline__ uint32_t bit_mask(uint32_t X, uint32_t k) {   // all ones iff bit k of X
  return (uint32_t)((int32_t)(X << (31 - k)) >> 31);
}
__device__ __forceinline__ uint32_t bit_sel(uint32_t M, uint32_t a, uint32_t b) { return (a & M) | (b & ~M); }

__device__ __forceinline__ float mask_at(const RowSel& r, uint32_t H, uint32_t L, uint32_t k) {
  const uint32_t mh = bit_mask(H, k), ml = bit_mask(L, k);
  return __uint_as_float(bit_sel(mh, bit_sel(ml, r.fe, r.fd), bit_sel(ml, r.fu, r.fb)));
}

typedef unsigned epi_v4u __attribute__((ext_vector_type(4)));

// 8 tokens of one chunk in registers (f32: a and b, 16-bit: a): the mask
// value added in f32, then the dtype's round to nearest even
template <typename T>
__device__ __forceinline__ void chunk_apply(epi_v4u& a, epi_v4u& b, const RowSel& r, uint32_t H, uint32_t L) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      a[k] = __float_as_uint(__uint_as_float(a[k]) + mask_at(r, H, L, k));
      b[k] = __float_as_uint(__uint_as_float(b[k]) + mask_at(r, H, L, k + 4));
    }
  } else {
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t lo = add16<T>(a[q] & 0xFFFFu, mask_at(r, H, L, 2 * q));
      const uint32_t hi = add16<T>(a[q] >> 16, mask_at(r, H, L, 2 * q + 1));
      a[q] = lo | (hi << 16);
    }
  }
}

// One thread = U chunks of 8 consecutive tokens of one row, kEpiThreads
// chunks apart (blockIdx.y strides the rows, so no division).  A chunk's
// allowed and unigram bits are one byte of the rows' bit words; when both row
// bases are 16-B aligned its scores move as 32 B (f32: two 16-B loads) or 16 B
// (bf16 / f16: one) -- hipcc does not vectorize 16-bit scalar accesses
// (cdna_hip_programming.md Guideline 13).  All U chunks' loads are issued
// (clamped to the row, so unconditionally) before the first add, and every
// chunk is computed whether or not it is stored (a loaded value consumed only
// under the store's guard had its load sunk into that branch).  The partial
// last chunk and unaligned rows take the scalar path.  Same
// arithmetic either way: the f32 add, then the dtype's round to nearest even.
template <typename T, int U>
__global__ void __launch_bounds__(kEpiThreads) k_epilogue(const T* __restrict__ scores, T* __restrict__ out,
                                                         uint32_t B, uint32_t V, uint64_t lds, uint64_t ldo,
                                                         const uint32_t* __restrict__ bits, uint64_t ldb,
                                                         const uint32_t* __restrict__ uni,
                                                         const RowParams* __restrict__ rp, int64_t eos) {
  const uint32_t per_row = (V + 7) / 8;
  const uint32_t full = V / 8;                       // chunks with all 8 tokens in the row
  const uint32_t j0 = blockIdx.x * (U * kEpiThreads) + threadIdx.x;
  const uint32_t uni_bytes = uni ? (V + 31) / 32 * 4 : 0u;
  for (uint32_t b = blockIdx.y; b < B; b += gridDim.y) {
    const T* s = scores + (uint64_t)b * lds;
    T* o = out + (uint64_t)b * ldo;
    // The bit words come through range-checked buffer loads (a null row reads
    // 0) and the row's flags are applied afterwards, so no load sits under a
    // branch: the scores, bit words and row parameters go out together.
    const __amdgpu_buffer_rsrc_t brs = make_rsrc(bits ? bits + (uint64_t)b * ldb : nullptr,
                                                 bits ? (uint32_t)(ldb * 4) : 0u);
    const __amdgpu_buffer_rsrc_t urs = make_rsrc(uni, uni_bytes);
    const bool vec = full && ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(o)) & 15) == 0;
    uint32_t jtail = 0;
    if (vec) {
      epi_v4u wa[U], wb[U];
      uint32_t dw[U], uw[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t j = j0 + u * kEpiThreads;
        const uint32_t t0 = 8 * (j < full ? j : full - 1);
        const epi_v4u* src = reinterpret_cast<const epi_v4u*>(s + t0);
        wa[u] = src[0];
        if constexpr (sizeof(T) == 4) wb[u] = src[1];
        dw[u] = __builtin_amdgcn_raw_buffer_load_b32(brs, (t0 >> 5) * 4u, 0, 0);
        uw[u] = __builtin_amdgcn_raw_buffer_load_b32(urs, (t0 >> 5) * 4u, 0, 0);
      }
      const RowSel r = row_sel(rp[b], V, eos);   // loaded after the scores: a load before them was
                                                // waited on before the scores went out
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t j = j0 + u * kEpiThreads;
        uint32_t H, L;
        chunk_codes(r, j < full ? j : full - 1, dw[u], uw[u], H, L);
        chunk_apply<T>(wa[u], wb[u], r, H, L);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t j = j0 + u * kEpiThreads;
        if (j < full) {
          epi_v4u* dst = reinterpret_cast<epi_v4u*>(o + 8 * j);
          dst[0] = wa[u];
          if constexpr (sizeof(T) == 4) dst[1] = wb[u];
        }
      }
      jtail = full;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t j = j0 + u * kEpiThreads;
      if (j >= jtail && j < per_row) {
        const RowSel r = row_sel(rp[b], V, eos);
        const uint32_t t0 = 8 * j;
        uint32_t H, L;
        chunk_codes(r, j, __builtin_amdgcn_raw_buffer_load_b32(brs, (t0 >> 5) * 4u, 0, 0),
                    __builtin_amdgcn_raw_buffer_load_b32(urs, (t0 >> 5) * 4u, 0, 0), H, L);
        for (uint32_t k = 0; k < 8 && t0 + k < V; ++k)
          o[t0 + k] = from_f<T>(to_f<T>(s[t0 + k]) + mask_at(r, H, L, k));
      }
    }
  }
}

template <typename T, int U>
void launch_epi_t(const void* scores, void* out, uint64_t B, uint64_t V, uint64_t lds, uint64_t ldo,
                  const uint32_t* bits, uint64_t ldb, const uint32_t* uni, const RowParams* rp, int64_t eos,
                  hipStream_t s) {
  const uint64_t per_row = (V + 7) / 8;
  const dim3 grid((unsigned)((per_row + U * kEpiThreads - 1) / (U * kEpiThreads)),
                  (unsigned)std::min<uint64_t>(B, 65535));
  k_epilogue<T, U><<<grid, kEpiThreads, 0, s>>>(reinterpret_cast<const T*>(scores), reinterpret_cast<T*>(out),
                                               (uint32_t)B, (uint32_t)V, lds, ldo, bits, ldb, uni, rp, eos);
}

// Chunks per thread (FMIDX_EPI_CHUNKS, default 1).  Measured at 256 x 128256
// (tools/sweeps/epi.sh, profiles/r02_processor/epi/): 1 chunk 21.7 us bf16 /
// 40.2 us f32, 2 chunks 24.3 / 44.5, 4 chunks 25.8 / 44.9 -- more waves beat
// more loads per wave; the nontemporal hint was slower in every case (23.0 /
// 51.3 at 1 chunk).  Before the bit-select rewrite: 24.5 / 43.2.
template <typename T>
void launch_epi_dt(uint32_t chunks, const void* scores, void* out, uint64_t B, uint64_t V, uint64_t lds,
                   uint64_t ldo, const uint32_t* bits, uint64_t ldb, const uint32_t* uni, const RowParams* rp,
                   int64_t eos, hipStream_t s) {
  if (chunks >= 4)
    launch_epi_t<T, 4>(scores, out, B, V, lds, ldo, bits, ldb, uni, rp, eos, s);
  else if (chunks == 2)
    launch_epi_t<T, 2>(scores, out, B, V, lds, ldo, bits, ldb, uni, rp, eos, s);
  else
    launch_epi_t<T, 1>(scores, out, B, V, lds, ldo, bits, ldb, uni, rp, eos, s);
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
  // chunks per thread: a measurement variant (make variant VFLAGS=-DFMIDX_EPI_CHUNKS=2); 1 measured fastest
#ifndef FMIDX_EPI_CHUNKS
#define FMIDX_EPI_CHUNKS 1
#endif
  const uint32_t chunks = FMIDX_EPI_CHUNKS;
  const RowParams* rp = reinterpret_cast<const RowParams*>(row_params);
  switch (dtype) {
    case 0: launch_epi_dt<float>(chunks, scores, out, B, V, lds, ldo, bits, ldb, uni, rp, eos, s); break;
    case 1: launch_epi_dt<__hip_bfloat16>(chunks, scores, out, B, V, lds, ldo, bits, ldb, uni, rp, eos, s); break;
    case 2: launch_epi_dt<__half>(chunks, scores, out, B, V, lds, ldo, bits, ldb, uni, rp, eos, s); break;
    default:
      set_error("unsupported scores dtype code %d", dtype);
      return -1;
  }
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
