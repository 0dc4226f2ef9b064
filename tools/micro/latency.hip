// Dependent-load latency on MI355X vs footprint (pointer chase, one lane).
// Calibrates the "round trip" cost the decode kernel's chains pay.
// build: hipcc --offload-arch=gfx950 -O3 latency.hip -o latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void chase(const uint64_t* __restrict__ buf, uint64_t mask_lines, uint64_t start, int steps,
                      uint64_t* out) {
  uint64_t p = start;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < steps; ++i) {
    const uint64_t v = __builtin_nontemporal_load(buf + p * 8);   // one 64-B line per hop
    p = (v ^ (p * 0x9E3779B97F4A7C15ull)) & mask_lines;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0;
  out[1] = p;
}

// same chase by 64 lanes of one wave, each its own chain (like 64 rows in flight)
__global__ void chase_wave(const uint64_t* __restrict__ buf, uint64_t mask_lines, int steps, uint64_t* out) {
  uint64_t p = (threadIdx.x * 0x632BE59BD9B4E019ull) & mask_lines;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < steps; ++i) {
    const uint64_t v = buf[p * 8];
    p = (v ^ (p * 0x9E3779B97F4A7C15ull)) & mask_lines;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  out[2 + threadIdx.x] = p;
}

__global__ void fill(uint64_t* buf, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    buf[i] = i * 0xD1B54A32D192ED03ull + 12345;
}

int main() {
  const uint64_t sizes_mb[] = {16, 128, 1024, 8192, 32768};
  uint64_t* out;
  hipMalloc(&out, 1024);
  for (uint64_t mb : sizes_mb) {
    const uint64_t bytes = mb << 20;
    uint64_t* buf;
    if (hipMalloc(&buf, bytes) != hipSuccess) { printf("alloc %llu MB failed\n", (unsigned long long)mb); continue; }
    fill<<<4096, 256>>>(buf, bytes / 8);
    const uint64_t lines = bytes / 64;
    uint64_t mask = 1;
    while (mask * 2 <= lines) mask *= 2;
    mask -= 1;
    const int steps = 2000;
    uint64_t h[2];
    for (int rep = 0; rep < 2; ++rep) {
      chase<<<1, 1>>>(buf, mask, 7, steps, out);
      hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    }
    const double ns1 = h[0] * 10.0 / steps;
    chase_wave<<<1, 64>>>(buf, mask, steps, out);
    hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
    const double ns64 = h[0] * 10.0 / steps;
    printf("footprint %6llu MB: dependent load %.0f ns (1 lane), %.0f ns (64 lanes, 64 chains)\n",
           (unsigned long long)mb, ns1, ns64);
    hipFree(buf);
  }
  return 0;
}
