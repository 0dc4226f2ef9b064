// How fast can ONE workgroup (one CU) write a 128-KB mask row, alone on the
// chip and with every CU writing?  The decode kernel's slowest rows end with
// exactly that: one 1024-thread workgroup expanding a bitmap into 128 KB of
// uint8 mask after its LF chain ("Where the cold time goes").
// Each workgroup writes `bytes` with 16-B stores, consecutive lanes on
// consecutive chunks (a wave writes 1 KB per instruction), plain or
// write-through (sc1), and stamps s_memrealtime (100 MHz) before its first
// store and after its last store is acknowledged (vmcnt(0)).
// build: hipcc --offload-arch=gfx950 -O3 cu_store.hip -o cu_store ; run: ./cu_store
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ void __launch_bounds__(1024) k_store(uint8_t* out, uint32_t bytes, uint64_t* stamps) {
  uint8_t* row = out + (uint64_t)blockIdx.x * bytes;
  const uint64_t a = reinterpret_cast<uint64_t>(row);
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                              __builtin_amdgcn_readfirstlane((uint32_t)a)),
      0, bytes, 0x00020000);
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const v4u v = {threadIdx.x, 1u, 2u, 3u};
  for (uint32_t off = threadIdx.x * 16; off < bytes; off += 1024 * 16)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t1;
  }
}

int main() {
  const uint32_t bytes = 128256;               // one uint8 mask row of a 128k vocabulary
  const int max_wg = 1024;
  uint8_t* out;
  uint64_t* st;
  hipError_t e = hipMalloc(&out, (size_t)max_wg * bytes);
  if (e == hipSuccess) e = hipMalloc(&st, 2 * max_wg * 8);
  if (e != hipSuccess) {
    printf("hipMalloc: %s\n", hipGetErrorString(e));
    return 1;
  }
  std::vector<uint64_t> h(2 * max_wg);
  for (int aux : {0, 16}) {
    for (int wgs : {1, 8, 64, 256, 512}) {
      std::vector<double> per, span;
      for (int rep = 0; rep < 20; ++rep) {
        if (aux)
          k_store<16><<<wgs, 1024>>>(out, bytes, st);
        else
          k_store<0><<<wgs, 1024>>>(out, bytes, st);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e == hipSuccess) e = hipMemcpy(h.data(), st, 2 * wgs * 8, hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
          printf("aux %d wgs %d rep %d: %s\n", aux, wgs, rep, hipGetErrorString(e));
          return 2;
        }
        if (rep < 3) continue;
        uint64_t lo = ~0ull, hi = 0;
        double s = 0;
        for (int i = 0; i < wgs; ++i) {
          s += (double)(h[2 * i + 1] - h[2 * i]);
          lo = std::min(lo, h[2 * i]);
          hi = std::max(hi, h[2 * i + 1]);
        }
        per.push_back(s / wgs * 10.0 / 1000.0);     // us per workgroup
        span.push_back((hi - lo) * 10.0 / 1000.0);
      }
      std::sort(per.begin(), per.end());
      std::sort(span.begin(), span.end());
      const double p = per[per.size() / 2], sp = span[span.size() / 2];
      printf("aux %2d  workgroups %4d: per-WG 128 KB write %.2f us (%.1f GB/s per CU), span %.2f us (%.0f GB/s chip)\n",
             aux, wgs, p, bytes / (p * 1e3), sp, (double)wgs * bytes / (sp * 1e3));
    }
  }
  return 0;
}
