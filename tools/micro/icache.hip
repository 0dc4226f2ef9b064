// Instruction-fetch cost of straight-line code executed once per launch
// (MI355X): a block of 2048 independent v_add (8 KB of code) is run twice in
// the same wave; pass 1 fetches it cold, pass 2 from the instruction cache.
// Reported per launch, over several launches (does the I-cache stay warm
// across kernel launches?).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define A1 "v_add_u32 %0, %0, 1\n"
#define A4 A1 A1 A1 A1
#define A16 A4 A4 A4 A4
#define A64 A16 A16 A16 A16
#define A256 A64 A64 A64 A64
#define A2048 A256 A256 A256 A256 A256 A256 A256 A256

__global__ void k(uint64_t* out, int reps) {
  uint32_t x = threadIdx.x;
  uint64_t t[3];
  t[0] = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < 2; ++r) {
    asm volatile(A2048 : "+v"(x));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    t[r + 1] = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[0] = t[1] - t[0];
    out[1] = t[2] - t[1];
  }
  if (x == 0xFFFFFFFF) out[2] = x;
}

int main() {
  uint64_t* d;
  (void)hipMalloc(&d, 64);
  for (int launch = 0; launch < 4; ++launch) {
    k<<<256, 64>>>(d, 1);
    uint64_t h[2];
    (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("launch %d: 8 KB straight-line code: cold pass %.2f us, warm pass %.2f us\n", launch, h[0] / 100.0,
           h[1] / 100.0);
  }
  return 0;
}
