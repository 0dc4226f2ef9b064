// Cold dependent hops vs how the buffer was allocated: does a physically
// contiguous allocation (hipExtMallocWithFlags(hipDeviceMallocContiguous))
// shorten a cold random hop -- i.e. is the page-table walk, not HBM, what a
// cold decode step's dependent hops pay?  Each pass: evict the caches (1 GiB
// written), then `chains` lanes each chase `hops` random 64-B lines; the time
// per hop is reported for few hops (dominated by first-touch translation) and
// many (steady state).
// build: hipcc --offload-arch=gfx950 -O3 tlb.hip -o tlb ; run: ./tlb [GiB ...]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      return false;                                                               \
    }                                                                             \
  } while (0)

__device__ __host__ inline uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void fill(uint64_t* buf, uint64_t lines) {   // the first word of every line
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x)
    buf[i * 8] = mix(i);
}

__global__ void bump(uint32_t* f, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    f[i] += 1;
}

__global__ void chase(const uint64_t* __restrict__ buf, uint64_t lines, int hops, uint64_t seed, uint64_t* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t p = mix(tid ^ seed) % lines;
  for (int i = 0; i < hops; ++i) p = mix(p ^ buf[p * 8]) % lines;
  out[tid] = p;
}

static bool run(int kind, double gib, uint32_t* flush, uint64_t nflush, uint64_t* out) {
  const uint64_t bytes = (uint64_t)(gib * (1ull << 30));
  const uint64_t lines = bytes / 64;
  uint64_t* buf = nullptr;
  if (kind == 0) {
    CK(hipMalloc(&buf, bytes));
  } else {
    hipError_t e = hipExtMallocWithFlags((void**)&buf, bytes, hipDeviceMallocContiguous);
    if (e != hipSuccess) {
      printf("%-10s %7.1f GiB: allocation failed (%s)\n", "contiguous", gib, hipGetErrorString(e));
      (void)hipGetLastError();
      return true;
    }
  }
  fill<<<4096, 256>>>(buf, lines);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int hop_list[] = {2, 4, 8, 32, 256};
  for (int chains : {256, 16384}) {
    for (int hops : hop_list) {
      float best = 1e30f, sum = 0;
      const int reps = 5;
      for (int r = 0; r < reps; ++r) {
        bump<<<4096, 256>>>(flush, nflush);
        CK(hipEventRecord(a));
        chase<<<chains / 64, 64>>>(buf, lines, hops, 1000003ull * r + hops + chains, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
        sum += ms;
      }
      printf("%-10s %7.1f GiB chains %5d hops %4d: %7.0f ns/hop (best %7.0f)\n", kind ? "contiguous" : "hipMalloc",
             gib, chains, hops, sum / reps * 1e6 / hops, best * 1e6 / hops);
      fflush(stdout);
    }
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  CK(hipFree(buf));
  return true;
}

int main(int argc, char** argv) {
  const uint64_t nflush = 1ull << 28;   // 1 GiB of uint32
  uint32_t* flush = nullptr;
  uint64_t* out = nullptr;
  if (hipMalloc(&flush, nflush * 4) != hipSuccess || hipMalloc(&out, 16384 * 8) != hipSuccess) return 1;
  hipMemset(flush, 0, nflush * 4);
  for (int i = 1; i < argc || i == 1; ++i) {
    const double gib = argc > 1 ? atof(argv[i]) : 16.0;
    for (int kind = 0; kind < 2; ++kind)
      if (!run(kind, gib, flush, nflush, out)) return 2;
    if (argc <= 1) break;
  }
  hipFree(flush);
  hipFree(out);
  return 0;
}
