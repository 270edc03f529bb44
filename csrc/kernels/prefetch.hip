// Infinity-Cache warming for the lone engine's decode (host: llmc_prefetch). A decode layer's fused
// attention + o_proj launch is a latency chain that keeps HBM at ~3.3 TB/s (profiles/r5_dec9k_kernel_stats.md:
// 71 MB in 21.5 us at 9k keys); the gate_up GEMV right after it is a pure ~6.6 TB/s weight stream.
// This kernel runs on a side stream BESIDE the attention launch (a fork/join inside the decode graph)
// and reads the first bytes of the NEXT projection's weights with default-policy loads, so they
// are in the 256 MiB Infinity Cache when the GEMV arrives (the layer's ~70 MB of K/V + o_proj
// weights + the prefetched bytes stay well inside it: MI355X_MICROARCH.md "Infinity Cache").
// Nothing is written except an impossible-value sink, so the loads cannot be dropped.
#include "common.h"

namespace llmc {

constexpr int kPfThreads = 256, kPfUnroll = 8;

__global__ __launch_bounds__(kPfThreads) void prefetch_kernel(const u32x4* __restrict__ p, int64_t n16,
                                                              uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kPfThreads;
  for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * kPfThreads + threadIdx.x; i0 < n16; i0 += stride * kPfUnroll) {
    u32x4 v[kPfUnroll];
#pragma unroll
    for (int u = 0; u < kPfUnroll; ++u) {
      const int64_t i = i0 + u * stride;
      v[u] = i < n16 ? p[i] : u32x4{0u, 0u, 0u, 0u};  // all kPfUnroll loads in flight at once
    }
#pragma unroll
    for (int u = 0; u < kPfUnroll; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x9e3779b9u && sink != nullptr) *sink = acc;
}

}  // namespace llmc

using namespace llmc;

// Read `bytes` (a multiple of 16) at `p` on `blocks` workgroups of 256 threads.
extern "C" int llmc_prefetch(const void* p, int64_t bytes, int blocks, void* sink, hipStream_t s) {
  if (bytes <= 0 || bytes % 16 != 0 || blocks < 1) return -1;
  prefetch_kernel<<<blocks, kPfThreads, 0, s>>>((const u32x4*)p, bytes / 16, (uint32_t*)sink);
  return static_cast<int>(hipGetLastError());
}
