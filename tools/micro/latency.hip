// Dependent-load latency on MI355X vs footprint (pointer chase), to separate
// cache, HBM and TLB effects for the decode kernel's random gathers.
//   chase: each hop = splitmix64(previous address ^ loaded value) over the
//   whole footprint (a new random 64-B line, usually a new 2-MB page).
//   paged: hops stay inside a window of 64 pages (2 MB each) for 64 hops,
//   then move -- same number of distinct lines, far fewer page changes.
// build: hipcc --offload-arch=gfx950 -O3 latency.hip -o latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void chase(const uint64_t* __restrict__ buf, uint64_t lines, int steps, int paged, uint64_t* out) {
  uint64_t p = mix(threadIdx.x + 1) % lines;
  uint64_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t base = 0;
  for (int i = 0; i < steps; ++i) {
    const uint64_t v = buf[p * 8];
    acc += v;
    const uint64_t h = mix(p ^ v ^ (uint64_t)i);
    if (paged) {
      if ((i & 63) == 0) base = (h % (lines / 32768 > 64 ? lines / 32768 - 64 : 1)) * 32768;   // 2 MB = 32768 lines
      p = base + (h % (64 * 32768 < lines ? 64 * 32768 : lines));
      if (p >= lines) p %= lines;
    } else {
      p = h % lines;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  out[1 + threadIdx.x] = acc + p;
}

int main() {
  const uint64_t sizes_mb[] = {64, 512, 4096, 16384, 65536};
  uint64_t* out;
  (void)hipMalloc(&out, 4096);
  for (uint64_t mb : sizes_mb) {
    uint64_t* buf;
    const uint64_t bytes = mb << 20;
    if (hipMalloc(&buf, bytes) != hipSuccess) {
      printf("alloc %llu MB failed\n", (unsigned long long)mb);
      continue;
    }
    (void)hipMemset(buf, 0, bytes);
    const uint64_t lines = bytes / 64;
    const int steps = 4000;
    double r[4];
    int k = 0;
    for (int paged = 0; paged < 2; ++paged) {
      for (int lanes : {1, 64}) {
        uint64_t h = 0;
        for (int rep = 0; rep < 2; ++rep) {
          chase<<<1, lanes>>>(buf, lines, steps, paged, out);
          (void)hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
        }
        r[k++] = h * 10.0 / steps;
      }
    }
    printf("footprint %6llu MB: random %.0f ns (1 lane) %.0f ns (64 lanes) | page-local %.0f ns (1) %.0f ns (64)\n",
           (unsigned long long)mb, r[0], r[1], r[2], r[3]);
    (void)hipFree(buf);
  }
  return 0;
}
