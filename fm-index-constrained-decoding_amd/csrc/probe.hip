// probe.hip -- measurement kernels for the bench's rank roofline (SURVEY
// §8(d)): the random 64-B gather ceiling of HBM, against which the LF
// (rank) throughput of the index is judged.  Not on any query path.
//
//  k_gather64  every thread loads `loads` random 64-B lines (4 x 16 B from the
//              same line, one request per line) of a buffer far larger than
//              the 256 MB MALL; the line indices come from a hash of
//              (thread, i), so the loads are independent and many are in
//              flight per wave: the throughput ceiling of scattered lines.
//  k_chase64   the dependent form: the next line index is read from the line
//              just loaded (a pointer chase) -- one round trip per hop, the
//              pattern of an LF step's rank lookups; `chains` lanes chase at once.
//  k_gather_coop<LPL, LINE>  lane-cooperative gathers: LPL lanes share one
//              random LINE-byte line, 16 B each (4 lanes per 64-B line, 8 per
//              128-B line), so one wave instruction fetches 64 / LPL whole lines
//              as contiguous 16-B pieces -- the shape of the index's grouped
//              kernels (a row's lanes reading its E window / probe run).
//  k_gather8   every lane its own random 8-B word (the narrowest read an LF
//              step makes: one E entry).
#include "fmidx_internal.h"

namespace fmidx {

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  return x ^ (x >> 33);
}

__global__ void __launch_bounds__(256) k_gather64(const uint4* __restrict__ buf, uint64_t nlines, uint64_t loads,
                                                  uint64_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
  uint64_t i = 0;
  for (; i + 4 <= loads; i += 4) {
    uint4 x[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t line = mix64(tid * 0x9E3779B97F4A7C15ull + i + u) & (nlines - 1);
      const uint4* p = buf + line * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) x[u][q] = p[q];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc ^= x[u][q].x ^ x[u][q].y ^ x[u][q].z ^ x[u][q].w;
  }
  if (acc == 0x9E3779B9u) sink[tid & 1023] = acc;   // keeps the loads live; practically never stores
}

template <int LPL, int LINE>
__global__ void __launch_bounds__(256) k_gather_coop(const uint4* __restrict__ buf, uint64_t nlines, uint64_t loads,
                                                     uint64_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t grp = tid / LPL;
  const uint32_t j = (uint32_t)(tid % LPL);
  uint32_t acc = 0;
  for (uint64_t i = 0; i + 8 <= loads; i += 8) {
    uint4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t line = mix64(grp * 0x9E3779B97F4A7C15ull + i + u) & (nlines - 1);
      x[u] = buf[line * (LINE / 16) + j];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= x[u].x ^ x[u].y ^ x[u].z ^ x[u].w;
  }
  if (acc == 0x9E3779B9u) sink[tid & 1023] = acc;
}

__global__ void __launch_bounds__(256) k_gather8(const uint64_t* __restrict__ buf, uint64_t nwords, uint64_t loads,
                                                 uint64_t* __restrict__ sink) {
  const uint64_t tid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint64_t acc = 0;
  for (uint64_t i = 0; i + 8 <= loads; i += 8) {
    uint64_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = buf[mix64(tid * 0x9E3779B97F4A7C15ull + i + u) & (nwords - 1)];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc ^= x[u];
  }
  if (acc == 0x9E3779B97F4A7C15ull) sink[tid & 1023] = acc;
}

__global__ void __launch_bounds__(64) k_chase64(const uint64_t* __restrict__ buf, uint64_t nlines, uint64_t hops,
                                                uint32_t chains, uint64_t* __restrict__ sink) {
  const uint64_t c = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (c >= chains) return;
  uint64_t line = mix64(c + 1) & (nlines - 1);
  for (uint64_t h = 0; h < hops; ++h) line = buf[line * 8] & (nlines - 1);
  if (line == ~0ull) sink[c & 1023] = line;
}

}  // namespace

int launch_probe_gather(const void* buf, uint64_t bytes, int chase, uint64_t loads, uint32_t threads_or_chains,
                        uint64_t* sink, hipStream_t s) {
  uint64_t nlines = 1;   // a power of two: line = hash & (nlines - 1), no 64-bit division
  while (nlines * 2 * 64 <= bytes) nlines *= 2;
  if (bytes < 64 || !buf || !sink) {
    set_error("probe_gather: empty buffer");
    return -1;
  }
  const uint32_t threads = threads_or_chains ? threads_or_chains : 256 * 2048;
  const unsigned g = (threads + 255) / 256;
  switch (chase) {
    case 1: {
      const uint32_t chains = threads_or_chains ? threads_or_chains : 256;
      k_chase64<<<(chains + 63) / 64, 64, 0, s>>>(static_cast<const uint64_t*>(buf), nlines, loads, chains, sink);
      break;
    }
    case 2:   // 4 lanes per random 64-B line
      k_gather_coop<4, 64><<<g, 256, 0, s>>>(static_cast<const uint4*>(buf), nlines, loads, sink);
      break;
    case 3:   // 8 lanes per random 128-B line
      k_gather_coop<8, 128><<<g, 256, 0, s>>>(static_cast<const uint4*>(buf), nlines / 2, loads, sink);
      break;
    case 4:   // one random 8-B word per lane
      k_gather8<<<g, 256, 0, s>>>(static_cast<const uint64_t*>(buf), nlines * 8, loads, sink);
      break;
    default:  // every lane its own random 64-B line (4 x 16 B)
      k_gather64<<<g, 256, 0, s>>>(static_cast<const uint4*>(buf), nlines, loads, sink);
  }
  FM_HIP(hipGetLastError());
  return 0;
}

}  // namespace fmidx
