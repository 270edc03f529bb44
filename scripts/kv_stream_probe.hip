// Streaming rate of the decode attention's K/V reads (attn_core.h SubTile::issue) by access shape
// and key split, Llama-3-8B at L keys of one layer: paged cache [pages][8 kv heads][64][128] bf16,
// grid (32 blocks, 8 kv heads) x 512 threads, each wave 64 keys (two 32-key sub-tiles), K and V.
//   kshape 0: K as the MFMA A operand (lane = key row & 15, 16 B at dim 8 * (lane >> 4) + 32 ks):
//             one instruction = 16 rows x 64 B
//   kshape 1: K like V: one instruction = 4 whole 256-B rows
//   split 0: 512-key blocks (the 16k bucket: only ceil(L / 512) blocks per head hold keys)
//   split 1: keys spread evenly over the 32 blocks (64-key units)
// Cold: NL layers' caches cycled (> the 256 MB Infinity Cache). Prints us per layer.
// build: hipcc -O3 --offload-arch=gfx950 scripts/kv_stream_probe.hip -o /tmp/kvp ; run: /tmp/kvp [L]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
constexpr int NKV = 8, BS = 64, D = 128, NC = 32, NL = 40;

template <int KSHAPE, int SPLIT>
__global__ __launch_bounds__(512) void kv_kernel(const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc, int L,
                                                 uint32_t* __restrict__ out) {
  const int c = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  int k0, k1;
  if (SPLIT == 0) {
    k0 = c * 512;
    k1 = min(L, k0 + 512);
  } else {
    const int units = (L + 63) / 64;
    k0 = 64 * (c * units / NC);
    k1 = min(L, 64 * ((c + 1) * units / NC));
  }
  const int wk = k0 + wave * 64;  // split 0: 8 waves x 64 = 512; split 1: waves beyond the range idle
  u32x4 acc = {0, 0, 0, 0};
  if (wk < k1) {
    const int page = wk / BS;  // identity block table, 64-key units never straddle a page
    const uint16_t* kb = kc + (static_cast<int64_t>(page) * NKV + g) * BS * D;
    const uint16_t* vb = vc + (static_cast<int64_t>(page) * NKV + g) * BS * D;
    const int r0 = wk % BS;
    u32x4 kr[16], vr[16];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int rb = r0 + 32 * st;
      if constexpr (KSHAPE == 0) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            kr[st * 8 + kt * 4 + ks] = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(kb + (rb + kt * 16 + (lane & 15)) * D + ks * 32 + 8 * (lane >> 4)));
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int flat = u * 64 + lane, r = flat / 16, ch = flat % 16;
          kr[st * 8 + u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(kb + (rb + r) * D + ch * 8));
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int flat = u * 64 + lane, r = flat / 16, ch = flat % 16;
        vr[st * 8 + u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(vb + (rb + r) * D + ch * 8));
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) acc ^= kr[i] ^ vr[i];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) out[blockIdx.y * NC + blockIdx.x] = acc[0];
}

template <int KS, int SP>
static float run(const uint16_t* kc, const uint16_t* vc, size_t layer_elems, int L, uint32_t* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int l = 0; l < NL; ++l) kv_kernel<KS, SP><<<dim3(NC, NKV), 512>>>(kc + l * layer_elems, vc + l * layer_elems, L, out);
  hipEventRecord(a);
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    for (int l = 0; l < NL; ++l)
      kv_kernel<KS, SP><<<dim3(NC, NKV), 512>>>(kc + l * layer_elems, vc + l * layer_elems, L, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / (reps * NL);
}

int main(int argc, char** argv) {
  const int L = argc > 1 ? atoi(argv[1]) : 9000;
  const int pages = (16384 + BS - 1) / BS;
  const size_t layer_elems = static_cast<size_t>(pages) * NKV * BS * D;
  uint16_t *kc, *vc;
  uint32_t* out;
  hipMalloc(&kc, layer_elems * NL * 2);
  hipMalloc(&vc, layer_elems * NL * 2);
  hipMalloc(&out, 4096);
  hipMemset(kc, 1, layer_elems * NL * 2);
  hipMemset(vc, 2, layer_elems * NL * 2);
  hipDeviceSynchronize();
  const double mb = 2.0 * L * NKV * D * 2 / 1e6;
  float t;
  t = run<0, 0>(kc, vc, layer_elems, L, out);
  printf("L=%d  K as MFMA operand, 512-key blocks : %7.2f us  %.2f TB/s\n", L, t, mb / t);
  t = run<1, 0>(kc, vc, layer_elems, L, out);
  printf("L=%d  K whole rows,      512-key blocks : %7.2f us  %.2f TB/s\n", L, t, mb / t);
  t = run<0, 1>(kc, vc, layer_elems, L, out);
  printf("L=%d  K as MFMA operand, even split     : %7.2f us  %.2f TB/s\n", L, t, mb / t);
  t = run<1, 1>(kc, vc, layer_elems, L, out);
  printf("L=%d  K whole rows,      even split     : %7.2f us  %.2f TB/s\n", L, t, mb / t);
  return 0;
}
