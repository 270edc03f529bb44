// Streaming rate of the o_proj weight tile access patterns (attn_oproj.hip design study):
// 256 blocks x 512 threads, 83 KB of LDS (one block per CU), each block reads 128 KB of a
// [4096 x 4096] bf16 matrix, cycling over 16 copies (> the 256 MB Infinity Cache).
//   v1: tile [128 rows x 1 KB] (rows c*128.., cols g*1 KB), 4 waves x 32 rows, nt loads (attn_oproj)
//   v2: same tile, 8 waves x 16 rows
//   v3: 16 whole rows (8 KB each) per block, 4 waves x 4 rows x 8 loads
//   v4: v1 with default-policy loads
//   v5: v1, loads issued in 4 rounds of 8 (wait between rounds)
// build: hipcc -O3 --offload-arch=gfx950 scripts/bench_tile_stream.hip -o /tmp/bts
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
constexpr int K = 4096, N = 4096;

template <int V>
__global__ __launch_bounds__(512) void stream_kernel(const uint16_t* __restrict__ W, float* __restrict__ out) {
  extern __shared__ char smem[];
  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  const int c = blockIdx.x, g = blockIdx.y;  // grid (32, 8)
  u32x4 acc = {0, 0, 0, 0};
  if constexpr (V == 1 || V == 4 || V == 5) {
    if (wave < 4) {
      const uint16_t* p = W + static_cast<int64_t>(c * 128 + wave * 32) * K + g * 512 + 8 * lane;
      u32x4 w[32];
      if constexpr (V == 5) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            w[8 * r + j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + static_cast<int64_t>(8 * r + j) * K));
#pragma unroll
          for (int j = 0; j < 8; ++j) acc ^= w[8 * r + j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const u32x4* a = reinterpret_cast<const u32x4*>(p + static_cast<int64_t>(j) * K);
          w[j] = V == 1 ? __builtin_nontemporal_load(a) : *a;
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) acc ^= w[j];
      }
    }
  } else if constexpr (V == 2) {
    const uint16_t* p = W + static_cast<int64_t>(c * 128 + wave * 16) * K + g * 512 + 8 * lane;
    u32x4 w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + static_cast<int64_t>(j) * K));
#pragma unroll
    for (int j = 0; j < 16; ++j) acc ^= w[j];
  } else {  // V == 3
    if (wave < 4) {
      const uint16_t* p = W + static_cast<int64_t>(blk * 16 + wave * 4) * K + 8 * lane;
      u32x4 w[32];
#pragma unroll
      for (int j = 0; j < 32; ++j)
        w[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + static_cast<int64_t>(j / 8) * K + (j % 8) * 512));
#pragma unroll
      for (int j = 0; j < 32; ++j) acc ^= w[j];
    }
  }
  smem[tid] = static_cast<char>(acc[0] ^ acc[1] ^ acc[2] ^ acc[3]);
  __syncthreads();
  if (tid == 0) out[blk] = smem[1] + smem[300];
}

template <int V>
static float run(const uint16_t* W, float* out, int copies, int iters) {
  const size_t lds = 83 * 1024;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(stream_kernel<V>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  for (int i = 0; i < copies; ++i) stream_kernel<V><<<dim3(32, 8), 512, lds>>>(W + static_cast<size_t>(i) * N * K, out);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) stream_kernel<V><<<dim3(32, 8), 512, lds>>>(W + static_cast<size_t>(i % copies) * N * K, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000 / iters;
}

int main() {
  const int copies = 16, iters = 64;
  uint16_t* W;
  float* out;
  if (hipMalloc(&W, static_cast<size_t>(copies) * N * K * 2) != hipSuccess) return 1;
  hipMalloc(&out, 4096 * 4);
  hipMemset(W, 0x3c, static_cast<size_t>(copies) * N * K * 2);
  const double mb = N * K * 2 / 1e6;
  float t;
  t = run<1>(W, out, copies, iters); printf("v1 tile 4 waves x 32 rows nt : %7.2f us  %5.2f TB/s\n", t, mb / t);
  t = run<2>(W, out, copies, iters); printf("v2 tile 8 waves x 16 rows nt : %7.2f us  %5.2f TB/s\n", t, mb / t);
  t = run<3>(W, out, copies, iters); printf("v3 whole rows 4 waves nt     : %7.2f us  %5.2f TB/s\n", t, mb / t);
  t = run<4>(W, out, copies, iters); printf("v4 tile 4 waves plain        : %7.2f us  %5.2f TB/s\n", t, mb / t);
  t = run<5>(W, out, copies, iters); printf("v5 tile 4 waves 4 rounds     : %7.2f us  %5.2f TB/s\n", t, mb / t);
  return 0;
}
