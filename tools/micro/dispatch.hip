// What sets the start-time spread of a launch's workgroups?  The decode
// kernel's 256 workgroups of 1024 threads start over 1.3-2.3 us (phase stamps,
// DESIGN §6), and every row's chain starts only when its workgroup does.  Here
// an empty-bodied kernel with the decode launch's shape records, per
// workgroup, s_memrealtime (100 MHz) at entry and exit; the spread is the
// last entry minus the first.  Variants: workgroup size at a fixed 4096 waves
// (1024 x 256, 512 x 512, 256 x 1024), kernel-argument size (16 B vs a 768-B
// struct by value, like the DevView the decode kernel takes), dynamic LDS
// (0 vs 20 KB) and register footprint (a kernel holding ~120 VGPRs live).
// Each variant: 12 launches, each after a 1 GiB eviction; median spread.
// build: hipcc --offload-arch=gfx950 -O3 dispatch.hip -o dispatch ; run: ./dispatch
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

struct Big {
  uint64_t w[96];   // 768 B
};

template <bool HEAVY>
__device__ __forceinline__ void body(uint64_t* stamps, const uint64_t* src, uint64_t salt) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  if (HEAVY) {
    // ~120 VGPRs live: 30 uint4 loads held until all are summed
    uint4 x[30];
#pragma unroll
    for (int i = 0; i < 30; ++i) x[i] = reinterpret_cast<const uint4*>(src)[(threadIdx.x * 31 + i) & 4095];
#pragma unroll
    for (int i = 0; i < 30; ++i) acc ^= x[i].x + x[i].y * 3 + x[i].z * 5 + x[i].w * 7;
  }
  if (threadIdx.x == 0) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = (__builtin_amdgcn_s_memrealtime() + (acc == 0x9E3779B9u ? salt : 0)) |
                                 ((uint64_t)(xcc & 0xF) << 60);
  }
}

template <int T, bool HEAVY>
__global__ void __launch_bounds__(T) k_small(uint64_t* stamps, const uint64_t* src) {
  extern __shared__ uint32_t lds[];
  if (threadIdx.x == 1 << 30) lds[0] = 0;
  body<HEAVY>(stamps, src, 0);
}

template <int T, bool HEAVY>
__global__ void __launch_bounds__(T) k_big(uint64_t* stamps, const uint64_t* src, Big b) {
  extern __shared__ uint32_t lds[];
  if (threadIdx.x == 1 << 30) lds[0] = (uint32_t)b.w[95];
  body<HEAVY>(stamps, src, b.w[threadIdx.x & 63]);
}

__global__ void k_flush(uint32_t* buf, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    buf[i] += 1;
}

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

template <int T, bool BIG, bool HEAVY>
int run(const char* name, uint64_t* d_st, const uint64_t* d_src, uint32_t* d_flush, uint64_t nflush, size_t lds,
        unsigned grid = 256u * (1024 / T)) {
  std::vector<uint64_t> st(2 * grid);
  std::vector<double> spread, span;
  Big b{};
  for (int i = 0; i < 96; ++i) b.w[i] = i;
  for (int rep = 0; rep < 12; ++rep) {
    k_flush<<<4096, 256>>>(d_flush, nflush);
    CK(hipDeviceSynchronize());
    if (BIG)
      k_big<T, HEAVY><<<grid, T, lds>>>(d_st, d_src, b);
    else
      k_small<T, HEAVY><<<grid, T, lds>>>(d_st, d_src);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost));
    uint64_t a = ~0ull, z = 0, e = 0;
    uint64_t xa[16], xz[16];
    for (int k = 0; k < 16; ++k) {
      xa[k] = ~0ull;
      xz[k] = 0;
    }
    for (unsigned g = 0; g < grid; ++g) {
      const uint64_t x = st[2 * g + 1] >> 60, end = st[2 * g + 1] & ((1ull << 60) - 1);
      a = std::min(a, st[2 * g]);
      z = std::max(z, st[2 * g]);
      e = std::max(e, end);
      xa[x] = std::min(xa[x], st[2 * g]);
      xz[x] = std::max(xz[x], st[2 * g]);
    }
    if (rep >= 2) {
      spread.push_back((z - a) * 0.01);
      span.push_back((e - a) * 0.01);
    }
    if (rep == 11 && T == 1024 && grid == 256) {   // per-XCD first / last start, relative to the first overall
      std::printf("   per XCC (first..last start, us):");
      for (int k = 0; k < 16; ++k)
        if (xa[k] != ~0ull) std::printf(" %d:%.2f..%.2f", k, (xa[k] - a) * 0.01, (xz[k] - a) * 0.01);
      std::printf("   blockIdx%%8 of the first 16 starts:");
      std::vector<std::pair<uint64_t, unsigned>> o;
      for (unsigned g = 0; g < grid; ++g) o.push_back({st[2 * g], g});
      std::sort(o.begin(), o.end());
      for (int k = 0; k < 16; ++k) std::printf(" %u", o[k].second % 8);
      std::printf("\n");
    }
  }
  std::sort(spread.begin(), spread.end());
  std::sort(span.begin(), span.end());
  std::printf("%-34s grid %5u x %4d  lds %5zu B  start spread median %.2f us (min %.2f max %.2f), span %.2f us\n",
              name, grid, T, lds, spread[spread.size() / 2], spread.front(), spread.back(), span[span.size() / 2]);
  return 0;
}

int main() {
  uint64_t* d_st = nullptr;
  uint64_t* d_src = nullptr;
  uint32_t* d_flush = nullptr;
  const uint64_t nflush = (1ull << 30) / 4;
  CK(hipMalloc(&d_st, 2 * 1024 * 8 * 4));
  CK(hipMalloc(&d_src, 4096 * 16));
  CK(hipMemset(d_src, 1, 4096 * 16));
  CK(hipMalloc(&d_flush, nflush * 4));
  CK(hipMemset(d_flush, 0, nflush * 4));
  const size_t L = 20 * 1024;
  int rc = 0;
  rc |= run<1024, false, false>("1024 thr, 16-B args", d_st, d_src, d_flush, nflush, 0);
  rc |= run<1024, true, false>("1024 thr, 768-B args", d_st, d_src, d_flush, nflush, 0);
  rc |= run<1024, true, false>("1024 thr, 768-B args, 20 KB LDS", d_st, d_src, d_flush, nflush, L);
  rc |= run<1024, true, true>("1024 thr, 768-B args, LDS, ~120 VGPR", d_st, d_src, d_flush, nflush, L);
  rc |= run<512, true, false>("512 thr, 768-B args, 20 KB LDS", d_st, d_src, d_flush, nflush, L);
  rc |= run<256, true, false>("256 thr, 768-B args, 20 KB LDS", d_st, d_src, d_flush, nflush, L);
  rc |= run<256, false, false>("256 thr, 16-B args", d_st, d_src, d_flush, nflush, 0);
  // the spread against the total wave count
  rc |= run<512, true, false>("256 x 512 thr (2048 waves)", d_st, d_src, d_flush, nflush, L, 256);
  rc |= run<256, true, false>("256 x 256 thr (1024 waves)", d_st, d_src, d_flush, nflush, L, 256);
  rc |= run<1024, true, false>("128 x 1024 thr (2048 waves)", d_st, d_src, d_flush, nflush, L, 128);
  rc |= run<64, true, false>("256 x 64 thr (256 waves)", d_st, d_src, d_flush, nflush, L, 256);
  rc |= run<1024, true, false>("512 x 1024 thr (8192 waves)", d_st, d_src, d_flush, nflush, L, 512);
  return rc;
}
