// K6 (prefill class): C[M, N] = A[M, K] . W[N, K]^T  bf16 in, f32 accumulate, MFMA 32x32x16.
//
// Both operands K-contiguous (weights stored [out][in]) -> both MFMA operands are 16-B row
// reads. Structure (cdna_hip_programming.md §5, "Minimum 2-phase" + T1 + T2):
//  * 128x128 output tile per 256-thread block (2x2 waves, 64x64 per wave = 2x2 MFMA tiles),
//    BK = 64, two LDS buffers (64 KB) -> 2 blocks/CU.
//  * global -> LDS with global_load_lds_dwordx4 (16 B/lane, no VGPR round trip); the LDS image
//    is lane-linear, so the XOR swizzle (chunk ^ ((row >> 1) & 7), 128-B rows) is applied on the
//    per-lane SOURCE address and again on the ds_read_b128 address (rule 21) -> conflict-free.
//  * one STAGE(next) / compute(cur) / barrier per K-step.
//  * bijective XCD-aware block remap (T1): consecutive tiles (same W panel, M fastest) land on
//    one XCD so the weight panel is fetched from HBM once per XCD L2.
//  * fused epilogues: bf16 store | f32 store | in-place residual add (C += A.W^T).
#include "common.h"

namespace llmc {

constexpr int kBM = 128, kBN = 128, kBK = 64;
constexpr int kGemmTileBytes = 128 * kBK * 2;  // 16 KB per operand tile

__device__ __forceinline__ int gswz(int row, int ch) { return row * (kBK * 2) + ((ch ^ ((row >> 1) & 7)) << 4); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return base + bid / 8;
}

// GATHER = MoE grouped GEMM (K11): the M axis is a list of expert-sorted rows padded to 128-row
// tiles (moe_align); tile t multiplies by expert tile_expert[t]'s weights, gathers A rows
// sorted_rows[i] / a_row_div and scatters C rows sorted_rows[i] (-1 = padding).
template <int EPI, bool GATHER>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const bf16_t* __restrict__ A, int lda,
                                                      const bf16_t* __restrict__ W, int ldw, void* __restrict__ C,
                                                      int ldc, int M, int N, int K,
                                                      const int32_t* __restrict__ sorted_rows = nullptr,
                                                      const int32_t* __restrict__ tile_expert = nullptr,
                                                      const int32_t* __restrict__ tile_count = nullptr,
                                                      int a_row_div = 1) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * kGemmTileBytes];
  const int num_n = (N + kBN - 1) / kBN;
  int m0, n0;
  if constexpr (GATHER) {
    const int max_tiles = M / kBM;  // M = padded row capacity
    const int tile = blockIdx.x % max_tiles;
    if (tile >= tile_count[0]) return;
    m0 = tile * kBM;
    n0 = (blockIdx.x / max_tiles) * kBN;
    W += static_cast<int64_t>(tile_expert[tile]) * N * ldw;
  } else {
    const int num_m = (M + kBM - 1) / kBM;
    const int id = xcd_remap(blockIdx.x, num_m * num_n);
    m0 = (id % num_m) * kBM;
    n0 = (id / num_m) * kBN;
  }
  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  const int r = lane & 31, hh = lane >> 5;
  const int wr = wave >> 1, wc = wave & 1;

  // per-lane global source offsets for the 4 staging instructions (fixed across K)
  const bf16_t* asrc[4];
  const bf16_t* bsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s = i * 256 + tid;
    const int row = s >> 3, cp = s & 7;
    const int ch = cp ^ ((row >> 1) & 7);
    int arow;
    if constexpr (GATHER) {
      const int sr = sorted_rows[m0 + row];
      arow = sr < 0 ? 0 : sr / a_row_div;
    } else {
      arow = min(m0 + row, M - 1);
    }
    asrc[i] = A + static_cast<int64_t>(arow) * lda + ch * 8;
    bsrc[i] = W + static_cast<int64_t>(min(n0 + row, N - 1)) * ldw + ch * 8;
  }
  auto stage = [&](int buf, int k0) {
    char* ab = smem + buf * 2 * kGemmTileBytes;
    char* bb = ab + kGemmTileBytes;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int wbase = (i * 256 + wave * 64) * 16;  // wave-uniform LDS byte offset
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + k0), (__attribute__((address_space(3))) void*)(ab + wbase), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + k0), (__attribute__((address_space(3))) void*)(bb + wbase), 16, 0, 0);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  const int nk = K / kBK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * kBK);
    const char* ab = smem + cur * 2 * kGemmTileBytes;
    const char* bb = ab + kGemmTileBytes;
#pragma unroll
    for (int kk = 0; kk < kBK / 16; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        af[t] = *reinterpret_cast<const bf16x8*>(ab + gswz(wr * 64 + t * 32 + r, kk * 2 + hh));
        bfr[t] = *reinterpret_cast<const bf16x8*>(bb + gswz(wc * 64 + t * 32 + r, kk * 2 + hh));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a], bfr[b], acc[a][b], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: C layout col = lane & 31 (n), row = (i&3) + 8(i>>2) + 4hh (m)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wc * 64 + b * 32 + r;
      if (n >= N) continue;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        int m = m0 + wr * 64 + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
        if constexpr (GATHER) {
          m = sorted_rows[m];
          if (m < 0) continue;
        } else {
          if (m >= M) continue;
        }
        const float v = acc[a][b][i];
        if constexpr (EPI == 0) {
          reinterpret_cast<bf16_t*>(C)[static_cast<int64_t>(m) * ldc + n] = f32_to_bf16(v);
        } else if constexpr (EPI == 1) {
          reinterpret_cast<float*>(C)[static_cast<int64_t>(m) * ldc + n] = v;
        } else {
          bf16_t* p = reinterpret_cast<bf16_t*>(C) + static_cast<int64_t>(m) * ldc + n;
          *p = f32_to_bf16(bf16_to_f32(*p) + v);
        }
      }
    }
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_gemm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                         int epi, hipStream_t s) {
  if (K % kBK != 0 || M <= 0 || N <= 0) return -1;
  const int nwg = ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
  switch (epi) {
    case 0: gemm_kernel<0, false><<<nwg, 256, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, M, N, K); break;
    case 1: gemm_kernel<1, false><<<nwg, 256, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, M, N, K); break;
    case 2: gemm_kernel<2, false><<<nwg, 256, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, M, N, K); break;
    default: return -2;
  }
  return static_cast<int>(hipGetLastError());
}

// Grouped expert GEMM over moe_align's padded row list (max_tiles * 128 rows of capacity).
extern "C" int llmc_moe_gemm(const void* A, int lda, const void* W, const void* sorted_rows, const void* tile_expert,
                             const void* tile_count, void* C, int ldc, int N, int K, int max_tiles, int a_row_div,
                             int epi, hipStream_t s) {
  if (K % kBK != 0) return -1;
  const int nwg = max_tiles * ((N + kBN - 1) / kBN);
  const int M = max_tiles * kBM;
  const int32_t* sr = (const int32_t*)sorted_rows;
  const int32_t* te = (const int32_t*)tile_expert;
  const int32_t* tc = (const int32_t*)tile_count;
  switch (epi) {
    case 0: gemm_kernel<0, true><<<nwg, 256, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, K, C, ldc, M, N, K, sr, te, tc, a_row_div); break;
    case 1: gemm_kernel<1, true><<<nwg, 256, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, K, C, ldc, M, N, K, sr, te, tc, a_row_div); break;
    default: return -2;
  }
  return static_cast<int>(hipGetLastError());
}
