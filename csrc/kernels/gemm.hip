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

// GATHER = MoE grouped GEMM (K11) for small expert groups (< 256 rows per expert on average;
// larger ones take gemm256_kernel<EPI, true>): the M axis is a list of expert-sorted rows padded to
// 128-row tiles (moe_align); tile t multiplies by expert tile_expert[t]'s weights, gathers A rows
// sorted_rows[i] / a_row_div and scatters C rows sorted_rows[i] (-1 = padding). EPI 3 = SiLU-mul of
// interleaved gate/up columns, as the dense kernel's.
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
    // bijective XCD remap: consecutive tiles of one expert share an N panel on one XCD's L2
    const int max_tiles = M / kBM;  // M = padded row capacity
    const int id = xcd_remap(blockIdx.x, max_tiles * num_n);
    const int tile = id % max_tiles;
    if (tile >= tile_count[0]) return;
    m0 = tile * kBM;
    n0 = (id / max_tiles) * kBN;
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
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float v = acc[a][b][i];
        // EPI 3: interleaved (gate, up) columns n, n + 1 sit in lanes r, r ^ 1 (N even: both or
        // neither in range), exchanged before any lane leaves the loop body
        const float pv = EPI == 3 ? __shfl_xor(v, 1, 64) : 0.f;
        if (n >= N) continue;
        int m = m0 + wr * 64 + a * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
        if constexpr (GATHER) {
          m = sorted_rows[m];
          if (m < 0) continue;
        } else {
          if (m >= M) continue;
        }
        if constexpr (EPI == 0) {
          reinterpret_cast<bf16_t*>(C)[static_cast<int64_t>(m) * ldc + n] = f32_to_bf16(v);
        } else if constexpr (EPI == 3) {
          if ((n & 1) == 0) reinterpret_cast<bf16_t*>(C)[static_cast<int64_t>(m) * ldc + n / 2] = f32_to_bf16(silu(v) * pv);
        } else if constexpr (EPI == 1) {
          reinterpret_cast<float*>(C)[static_cast<int64_t>(m) * ldc + n] = v;
        } else {
          bf16_t* p = reinterpret_cast<bf16_t*>(C) + static_cast<int64_t>(m) * ldc + n;
          *p = f32_to_bf16(bf16_to_f32(*p) + v);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Dense prefill GEMM (K6, M >= 5): C = A . W^T, both operands K-contiguous, 256 x 256 tiles,
// 512 threads = 8 waves (2 M x 4 N), one block per CU (160 KiB of LDS).
//  * wave block 128 x 64 = 8 x 4 tiles of mfma_f32_16x16x32_bf16 with the operands SWAPPED (W
//    fragment as A, activation as B: D[n][m]) so a lane ends with 4 consecutive output columns of
//    one row -> 8-/16-byte epilogue stores.
//  * a K-step (64) is consumed in 2 phases: P1 reads A rows 0-63 of the wave + its 64 W columns
//    (16 ds_read_b128) -> output rows 0-63; P2 reads A rows 64-127 (8) -> rows 64-127. The step's
//    operands are 4 "quarters" (A0 / W0 / W1 / A1: 128 rows x 64 K = 16 KiB each), every byte read
//    from LDS exactly once.
//  * LDS = a RING of 10 quarter slots. Quarter n (= 4 kstep + j) lives in slot n % 10 and is
//    fetched by LDS-DMA (buffer_load_dwordx4 ... lds: per-lane 32-bit offsets fixed for the whole
//    K loop, the K position in the scalar offset, so a fetch costs no vector instruction) one phase
//    after its slot's previous quarter was last read — each phase retires its LDS reads before its
//    first barrier — so the ring runs TWO K-steps ahead: every fetch has two phases (~2k cycles)
//    to land before the counted `s_waitcnt vmcnt(8)` that precedes its first read; no barrier ever
//    drains the load queue (cdna_hip_programming.md §5 "Pipelining across barriers").
//  * ping-pong: the two wave rows run one barrier apart (waves 4-7 take an extra barrier up
//    front), so one row's LDS reads + fetch issue overlap the other row's MFMA cluster on the same
//    SIMD; s_setprio(1) around each cluster keeps hipcc from scattering it (T5).
//  * LDS XOR swizzle chunk ^ ((row >> 1) & 7) (128-B rows): on the per-lane SOURCE offset of the
//    lane-linear LDS-DMA and on the ds_read_b128 address (rule 21): conflict-free
//    (SQ_LDS_BANK_CONFLICT 0).
//  * grid: bijective XCD remap (T1) then grouped tile order (8 M-tiles x all N per group).
//  * fused epilogues: bf16 | f32 | residual add (C += A.W^T) | SiLU-mul of interleaved gate/up
//    columns (C[m][n/2] = silu(g) * u).
// Measured (MI355X, random bf16; profiles/r3_gemm_4wave_ab.md): 1.33-1.41 PF/s on the Llama-3-8B
// prefill shapes with the LDS-staged dwordx4 epilogue (r2: 1.26-1.40), 86-88 % of hipBLASLt (PMC: hipBLASLt runs 4 waves x 128 x 128
// with 512 registers each and 1.5x fewer LDS reads; this 8-wave layout parks waves at barriers).
// 4-wave 128 x 128-per-wave forms (AGPR accumulators, one barrier per 32- or 64-K step) measured
// 1.09-1.19 PF/s on the same shapes and were dropped (profiles/r3_gemm_4wave_ab.md).
constexpr int kT = 256, kTK = 64;
constexpr int kQuarter = 128 * kTK * 2;  // bytes
constexpr int kSlots = 10;
constexpr int kGroupM = 8;

// Epilogue store of 4 consecutive output columns C[m][n .. n + 3] (f32 accumulators) with the
// fused epilogue; m < M checked by the caller.
template <int EPI>
__device__ __forceinline__ void store4(void* __restrict__ C, int ldc, int N, int m, int n, const f32x4& v, bool vec_ok) {
  if constexpr (EPI == 3) {  // SiLU(gate) * up over interleaved (gate, up) column pairs
    float o[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const float g = v[2 * p], u = v[2 * p + 1];
      o[p] = g / (1.f + __expf(-g)) * u;
    }
    bf16_t* crow = reinterpret_cast<bf16_t*>(C) + static_cast<int64_t>(m) * ldc;
    if (vec_ok && n + 3 < N) {
      *reinterpret_cast<uint32_t*>(crow + n / 2) = pack_bf16x2(o[0], o[1]);
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p)
        if (n + 2 * p + 1 < N) crow[n / 2 + p] = f32_to_bf16(o[p]);
    }
  } else if constexpr (EPI == 1) {
    float* crow = reinterpret_cast<float*>(C) + static_cast<int64_t>(m) * ldc;
    if (vec_ok && n + 3 < N) {
      *reinterpret_cast<f32x4*>(crow + n) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (n + e < N) crow[n + e] = v[e];
    }
  } else {
    bf16_t* crow = reinterpret_cast<bf16_t*>(C) + static_cast<int64_t>(m) * ldc;
    if (vec_ok && n + 3 < N) {
      float o[4] = {v[0], v[1], v[2], v[3]};
      if constexpr (EPI == 2) {
        const u32x2 old = *reinterpret_cast<const u32x2*>(crow + n);
        o[0] += bf16_lo(old[0]);
        o[1] += bf16_hi(old[0]);
        o[2] += bf16_lo(old[1]);
        o[3] += bf16_hi(old[1]);
      }
      *reinterpret_cast<u32x2*>(crow + n) = u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (n + e >= N) continue;
        const float x = EPI == 2 ? bf16_to_f32(crow[n + e]) + v[e] : v[e];
        crow[n + e] = f32_to_bf16(x);
      }
    }
  }
}

// Epilogue of the 16x16x32 kernels: acc[mi][ni] holds D[n][m] of 16 x 16 tile (mi, ni) of the wave's
// 128 x 64 block (operands swapped), i.e. lane (l16, lg) has C[m][n .. n + 3].
template <int EPI>
__device__ __forceinline__ void gemm256_epilogue(const f32x4 (&acc)[8][4], void* __restrict__ C, int ldc, int M, int N,
                                                 int m0, int n0, int wr, int wc, int l16, int lg) {
  const bool vec_ok = (N % 4 == 0) && (ldc % 4 == 0);
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int m = m0 + wr * 128 + mi * 16 + l16;
    if (m >= M) continue;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) store4<EPI>(C, ldc, N, m, n0 + wc * 64 + ni * 16 + 4 * lg, acc[mi][ni], vec_ok);
  }
}

// bf16 epilogue through LDS (EPI 0 with N % 8 == 0, EPI 3 with N % 16 == 0; the residual add keeps the direct form, which
// rounds acc + old once): each wave's 128 x 64 output block (128 x 32
// for the SiLU-mul) is written to its own 16 KiB of the (drained) staging ring as 8-byte pieces
// (4-byte for SiLU) and read back as 16-byte row chunks, so the global stores are dwordx4 covering
// whole 128-byte (64-byte) row segments: half (a quarter of) the store instructions of the direct
// 8-byte form. LDS image [128][OW] bf16 with the 16-byte chunk index XORed by row bits (conflict-
// free writes and reads); only the wave's own region is touched, so one wave-local wait suffices
// between the two passes.
template <int EPI>
__device__ __forceinline__ void gemm256_epilogue_lds(const f32x4 (&acc)[8][4], char* smem, void* __restrict__ C, int ldc,
                                                     int M, int N, int m0, int n0, int wave, int wr, int wc, int lane,
                                                     int l16, int lg) {
  constexpr int OW = EPI == 3 ? 32 : 64;  // output columns per wave
  constexpr int RB = OW * 2;              // bytes per LDS row
  constexpr int CPR = RB / 16;            // 16-byte chunks per row (8 or 4)
  char* img = smem + wave * 128 * RB;
  auto sw = [&](int r, int chunk) { return r * RB + ((chunk ^ ((r >> 1) & (CPR - 1))) << 4); };
  // all waves are past their last ring read (the caller's final barrier) and every LDS-DMA landed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#pragma unroll
  for (int mi = 0; mi < 8; ++mi) {
    const int r = mi * 16 + l16;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const f32x4& v = acc[mi][ni];
      if constexpr (EPI == 3) {  // columns ni * 16 + 4 lg .. + 3 -> outputs ni * 8 + 2 lg, + 1 (4 bytes)
        const float o0 = v[0] / (1.f + __expf(-v[0])) * v[1], o1 = v[2] / (1.f + __expf(-v[2])) * v[3];
        const int ob = (ni * 8 + 2 * lg) * 2;
        *reinterpret_cast<uint32_t*>(img + sw(r, ob >> 4) + (ob & 15)) = pack_bf16x2(o0, o1);
      } else {  // columns ni * 16 + 4 lg .. + 3 (8 bytes)
        const int ob = (ni * 16 + 4 * lg) * 2;
        *reinterpret_cast<u32x2*>(img + sw(r, ob >> 4) + (ob & 15)) =
            u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's writes done (wave-local image)
  constexpr int RPI = 64 / CPR;  // rows per wave instruction
  const int rr = lane / CPR, ch = lane % CPR;
  const int n_out = EPI == 3 ? N / 2 : N;
  const int col = (EPI == 3 ? n0 / 2 : n0) + wc * OW + ch * 8;
  if (col >= n_out) return;  // n_out % 8 == 0: a chunk is all in or all out
#pragma unroll
  for (int it = 0; it < 128 / RPI; ++it) {
    const int r = it * RPI + rr;
    const int m = m0 + wr * 128 + r;
    if (m >= M) break;
    const uint4 d = *reinterpret_cast<const uint4*>(img + sw(r, ch));
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(C) + static_cast<int64_t>(m) * ldc + col) = d;
  }
}

// GATHER = the MoE grouped GEMM (K11) on this pipeline: M = max_tiles x 256 rows of moe_align's
// expert-sorted, 256-row-padded pair list; tile t multiplies by expert tile_expert[t]'s [N, K]
// weights, its A rows are gathered (sorted_rows[i] / a_row_div of the a_rows-row matrix A: the
// per-lane LDS-DMA offsets simply point at the gathered rows) and its C rows scattered to
// sorted_rows[i] (-1 = padding, not stored). Tiles beyond tile_count[0] exit at once.
template <int EPI, bool GATHER = false>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(const bf16_t* __restrict__ A, int lda,
                                                          const bf16_t* __restrict__ W, int ldw, void* __restrict__ C,
                                                          int ldc, int M, int N, int K,
                                                          const int32_t* __restrict__ sorted_rows = nullptr,
                                                          const int32_t* __restrict__ tile_expert = nullptr,
                                                          const int32_t* __restrict__ tile_count = nullptr,
                                                          int a_row_div = 1, int a_rows = 0) {
  __shared__ __attribute__((aligned(16))) char smem[kSlots * kQuarter];
  const int num_m = (M + kT - 1) / kT, num_n = (N + kT - 1) / kT;
  const int id = xcd_remap(blockIdx.x, num_m * num_n);
  const int group = id / (kGroupM * num_n);
  const int first_m = group * kGroupM;
  const int gsz = min(num_m - first_m, kGroupM);
  const int in_group = id - group * kGroupM * num_n;
  const int m0 = (first_m + in_group % gsz) * kT, n0 = (in_group / gsz) * kT;
  if constexpr (GATHER) {
    const int tile = m0 / kT;
    if (tile >= tile_count[0]) return;  // block-uniform, before any barrier
    W += static_cast<int64_t>(tile_expert[tile]) * N * ldw;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int l16 = lane & 15, lg = lane >> 4;
  // buffer descriptors on this tile's rows (offsets stay < 2 GiB: 256 rows x ld; GATHER: the whole
  // A, host-checked); per-lane byte offsets of the 4 quarter types x 2 pieces (rows clamped)
  const int rowsA = min(kT, M - m0), rowsW = min(kT, N - n0);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(GATHER ? A : A + static_cast<int64_t>(m0) * lda), 0, (GATHER ? a_rows : rowsA) * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W + static_cast<int64_t>(n0) * ldw), 0, rowsW * ldw * 2, 0x00020000);
  uint32_t voff[4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int s = i * 512 + tid;
    const int r = s >> 3, c = (s & 7) ^ ((r >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int ar = min((r >> 6) * 128 + h * 64 + (r & 63), rowsA - 1);
      if constexpr (GATHER) {
        const int sr = sorted_rows[m0 + ar];
        ar = sr < 0 ? 0 : sr / a_row_div;
      }
      const int wrow = min((r >> 5) * 64 + h * 32 + (r & 31), rowsW - 1);
      voff[h == 0 ? 0 : 3][i] = static_cast<uint32_t>((ar * lda + c * 8) * 2);
      voff[1 + h][i] = static_cast<uint32_t>((wrow * ldw + c * 8) * 2);
    }
  }
  const int nk = K / kTK, nq = 4 * nk;
  auto stage = [&](int n) {
    const int j = n & 3, kbytes = (n >> 2) * kTK * 2;
    char* q = smem + (n % kSlots) * kQuarter + wave * 64 * 16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds((j == 0 || j == 3) ? rsA : rsW,
                                               (__attribute__((address_space(3))) void*)(q + i * 512 * 16), 16,
                                               voff[j][i], kbytes, 0, 0);
  };
  auto lds_off = [&](int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); };
  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bw0[2][2], bw1[2][2];
  for (int n = 0; n < 8 && n < nq; ++n) stage(n);
  if (nq >= 8) {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // k-step 0 landed, k-step 1 in flight
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if (wr == 1) asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  auto sync_wait = [&](int n_issue) {
    if (n_issue + 1 < nq) {
      stage(n_issue);
      stage(n_issue + 1);
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
    } else {
      if (n_issue < nq) stage(n_issue);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto end_phase = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int t = 0; t < nk; ++t) {
    const char* qa0 = smem + ((4 * t + 0) % kSlots) * kQuarter;
    const char* qw0 = smem + ((4 * t + 1) % kSlots) * kQuarter;
    const char* qw1 = smem + ((4 * t + 2) % kSlots) * kQuarter;
    const char* qa1 = smem + ((4 * t + 3) % kSlots) * kQuarter;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bw0[ni][kk] = *reinterpret_cast<const bf16x8*>(qw0 + lds_off(wc * 32 + ni * 16 + l16, kk * 4 + lg));
        bw1[ni][kk] = *reinterpret_cast<const bf16x8*>(qw1 + lds_off(wc * 32 + ni * 16 + l16, kk * 4 + lg));
      }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        af[mi][kk] = *reinterpret_cast<const bf16x8*>(qa0 + lds_off(wr * 64 + mi * 16 + l16, kk * 4 + lg));
    sync_wait(4 * t + 8);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw0[ni][kk], af[mi][kk], acc[mi][ni], 0, 0, 0);
          acc[mi][2 + ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw1[ni][kk], af[mi][kk], acc[mi][2 + ni], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
    end_phase();
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        af[mi][kk] = *reinterpret_cast<const bf16x8*>(qa1 + lds_off(wr * 64 + mi * 16 + l16, kk * 4 + lg));
    sync_wait(4 * t + 10);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          acc[4 + mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw0[ni][kk], af[mi][kk], acc[4 + mi][ni], 0, 0, 0);
          acc[4 + mi][2 + ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw1[ni][kk], af[mi][kk], acc[4 + mi][2 + ni], 0, 0, 0);
        }
    __builtin_amdgcn_s_setprio(0);
    end_phase();
  }
  if (wr == 0) asm volatile("s_barrier" ::: "memory");
  if constexpr (GATHER) {
    const bool vec_ok = (N % 4 == 0) && (ldc % 4 == 0);
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = sorted_rows[m0 + wr * 128 + mi * 16 + l16];
      if (m < 0) continue;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) store4<EPI>(C, ldc, N, m, n0 + wc * 64 + ni * 16 + 4 * lg, acc[mi][ni], vec_ok);
    }
  } else if ((EPI == 0 || EPI == 3) && N % (EPI == 3 ? 16 : 8) == 0 && ldc % 8 == 0) {
    gemm256_epilogue_lds<EPI>(acc, smem, C, ldc, M, N, m0, n0, wave, wr, wc, lane, l16, lg);
  } else {
    gemm256_epilogue<EPI>(acc, C, ldc, M, N, m0, n0, wr, wc, l16, lg);
  }
}

// ---------------------------------------------------------------------------------------------
// Narrow-N prefill GEMM: 128 x (32 NI) tiles (NI = 6: 128 x 192) for the outputs whose 256 x 256
// grid cannot fill the chip — a Llama-3-8B TP=8 rank's qkv (N = 768) has 96 such tiles for 256 CUs
// (0.62 PF/s) but 256 tiles of 128 x 192 at M = 8192, one per CU.
//  * 256 threads = 4 waves (2 M x 2 N), one per SIMD, one block per CU; a wave owns 64 x (16 NI) of
//    the tile = 4 x NI tiles of mfma_f32_16x16x32_bf16 with the operands swapped (W fragment as A:
//    D[n][m], so the epilogue stores 4 consecutive columns per lane, as gemm256_kernel's).
//  * LDS = 4 slots of one K-step (64) each (160 KiB): A 128 rows + W 32 NI rows, 128-B rows with
//    the chunk ^ ((row >> 1) & 7) swizzle on the LDS-DMA source offset and on the ds_read_b128
//    address (conflict-free, as gemm256_kernel's). Stage t + 4 is fetched into the slot of step t
//    right after the barrier that retires step t's reads: three K-steps to land (3 slots measured
//    the same: 53.6 vs 53.5 us at M = 8192, N = 768, so the fetch latency is covered).
//  * each K-step is two halves of 32 K; the second half's fragments are read while the first
//    half's 4 NI MFMAs run, the next step's first half while the second half's run, so the one
//    barrier per K-step sits between two MFMA clusters and no LDS read latency is exposed
//    (one wave per SIMD: MI355X_MICROARCH.md §LDS, keep reads in flight across MFMAs).
//  * LDS reads per K-step: 4 waves x (64 + 16 NI) rows x 128 B = 80 KiB (NI = 6) = 320 cycles at
//    256 B/clk against 768 MFMA cycles per SIMD.
template <int EPI, int NI>
__global__ __launch_bounds__(256, 1) void gemm_narrow_kernel(const bf16_t* __restrict__ A, int lda,
                                                             const bf16_t* __restrict__ W, int ldw,
                                                             void* __restrict__ C, int ldc, int M, int N, int K) {
  constexpr int TM = 128, TN = 32 * NI, WN = 16 * NI, NS = 4;
  constexpr int kAB = TM * kTK * 2, kWB = TN * kTK * 2, kSlot = kAB + kWB;
  constexpr int LA = kAB / 4096, LI = LA + kWB / 4096;  // LDS-DMA instructions per lane per K-step
  static_assert(kWB % 4096 == 0 && NS * kSlot <= 160 * 1024 && LI <= 10, "narrow GEMM tile");
  __shared__ __attribute__((aligned(16))) char smem[NS * kSlot];
  const int num_m = (M + TM - 1) / TM, num_n = (N + TN - 1) / TN;
  // XCD remap (T1) with N fastest: the N tiles of one A row panel are consecutive ids on one XCD
  const int id = xcd_remap(blockIdx.x, num_m * num_n);
  const int m0 = (id / num_n) * TM, n0 = (id % num_n) * TN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int l16 = lane & 15, lg = lane >> 4;
  const int rowsA = min(TM, M - m0), rowsW = min(TN, N - n0);
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + static_cast<int64_t>(m0) * lda), 0, rowsA * lda * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW =
      __builtin_amdgcn_make_buffer_rsrc((void*)(W + static_cast<int64_t>(n0) * ldw), 0, rowsW * ldw * 2, 0x00020000);
  uint32_t voff[10];  // fixed size: a template-dependent operand type on the buffer builtin drops the host stub
#pragma unroll
  for (int i = 0; i < LI; ++i) {
    const int s = (i < LA ? i : i - LA) * 256 + tid;
    const int r = s >> 3, c = (s & 7) ^ ((r >> 1) & 7);
    voff[i] = i < LA ? static_cast<uint32_t>((min(r, rowsA - 1) * lda + c * 8) * 2)
                     : static_cast<uint32_t>((min(r, rowsW - 1) * ldw + c * 8) * 2);
  }
  // stage(n, slot): K-step n into the slot at byte offset `slot`
  auto stage = [&](int n, int slot) {
    char* q = smem + slot + wave * 1024;
    const int kbytes = n * kTK * 2;
#pragma unroll
    for (int i = 0; i < LI; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i < LA ? rsA : rsW, (__attribute__((address_space(3))) void*)(q + i * 4096),
                                               16, voff[i], kbytes, 0, 0);
  };
  // per-lane read offsets: rows 16 apart share the swizzle, so one base per half (kk) and operand
  const int offA[2] = {(wr * 64 + l16) * 128 + (((0 + lg) ^ ((l16 >> 1) & 7)) << 4),
                       (wr * 64 + l16) * 128 + (((4 + lg) ^ ((l16 >> 1) & 7)) << 4)};
  const int offW[2] = {kAB + (wc * WN + l16) * 128 + (((0 + lg) ^ ((l16 >> 1) & 7)) << 4),
                       kAB + (wc * WN + l16) * 128 + (((4 + lg) ^ ((l16 >> 1) & 7)) << 4)};
  auto read_half = [&](int slot, int kk, bf16x8(&af)[4], bf16x8(&bw)[NI]) {
    const char* qa = smem + slot + offA[kk];
    const char* qw = smem + slot + offW[kk];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) af[mi] = *reinterpret_cast<const bf16x8*>(qa + mi * 2048);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) bw[ni] = *reinterpret_cast<const bf16x8*>(qw + ni * 2048);
  };
  f32x4 acc[4][NI];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NI; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const bf16x8(&af)[4], const bf16x8(&bw)[NI]) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[ni], af[mi], acc[mi][ni], 0, 0, 0);
  };
  // one MFMA, one ds_read, ... : the next half's 4 + NI fragment reads ride between this half's
  // first MFMAs (the fragments they replace were consumed at issue of the cluster's first MFMAs)
  auto interleave = [&]() {
#pragma unroll
    for (int i = 0; i < 4 + NI; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4 * NI - (4 + NI), 0);
  };
  static_assert(LI == 10, "the counted waits below are written for 10 LDS-DMA loads per K-step");
  const int nk = K / kTK;
  bf16x8 af0[4], bw0[NI], af1[4], bw1[NI];
  for (int n = 0; n < NS && n < nk; ++n) stage(n, n * kSlot);
  if (nk >= 4) {
    asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
  } else if (nk == 3) {
    asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  } else if (nk == 2) {
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  asm volatile("s_barrier" ::: "memory");
  int slot = 0;  // byte offset of step t's slot
  read_half(0, 0, af0, bw0);
  for (int t = 0; t + 1 < nk; ++t) {
    const int nslot = slot + kSlot == NS * kSlot ? 0 : slot + kSlot;
    __builtin_amdgcn_sched_barrier(0);
    read_half(slot, 1, af1, bw1);
    mma(af0, bw0);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    // step t + 1 landed (steps t + 2, t + 3 may still be in flight); this wave's reads of step t retired
    if (t + 3 < nk) {
      asm volatile("s_waitcnt vmcnt(20) lgkmcnt(0)" ::: "memory");
    } else if (t + 2 < nk) {
      asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t + NS < nk) stage(t + NS, slot);  // the slot step t just retired
    __builtin_amdgcn_sched_barrier(0);
    read_half(nslot, 0, af0, bw0);
    mma(af1, bw1);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    slot = nslot;
  }
  read_half(slot, 1, af1, bw1);
  mma(af0, bw0);
  mma(af1, bw1);
  const bool vec_ok = (N % 4 == 0) && (ldc % 4 == 0);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int m = m0 + wr * 64 + mi * 16 + l16;
    if (m >= M) continue;
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) store4<EPI>(C, ldc, N, m, n0 + wc * WN + ni * 16 + 4 * lg, acc[mi][ni], vec_ok);
  }
}

}  // namespace llmc

using namespace llmc;

// Kernel choice for a dense C[M, N]: 0 = 256 x 256 (gemm256_kernel), 1 = 128 x 192 (gemm_narrow_kernel).
// Makespan model: rounds of 256 blocks (one per CU for both kernels) x the tile's area over its
// full-chip rate; the narrow kernel's rate per unit area is 0.69 of the 256 x 256 kernel's (MI355X,
// M = 8192: 870 vs 1268 TF/s at N = 6144), its tile 0.375 of the area. It wins where the 256 x 256
// grid leaves CUs idle: a TP=8 rank's qkv (N = 768) at M = 8192 runs 53.5 us against 81.5
// (hipBLASLt 50.5), at M = 2048 45.8 against 75.9; at M = 33000 (2 rounds against 5) the 256 x 256
// kernel stays (188 vs 259 us). profiles/r5_gemm_narrow.md.
extern "C" int llmc_gemm_plan(int M, int N) {
  const int64_t t256 = static_cast<int64_t>((M + kT - 1) / kT) * ((N + kT - 1) / kT);
  const int64_t tn = static_cast<int64_t>((M + 127) / 128) * ((N + 191) / 192);
  const double r256 = static_cast<double>((t256 + 255) / 256), rn = static_cast<double>((tn + 255) / 256);
  return rn * (0.375 / 0.69) < r256 ? 1 : 0;
}

extern "C" int llmc_gemm_narrow(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                                int epi, hipStream_t s);

// C[M, N] (+)= A[M, K] . W[N, K]^T. epi: 0 bf16, 1 f32, 2 C += (bf16), 3 SiLU-mul of interleaved
// gate/up columns into C[M, N / 2] (bf16). K must be a multiple of 64, lda/ldw multiples of 8.
// kind: -1 = llmc_gemm_plan's choice, 0 = 256 x 256, 1 = 128 x 192.
extern "C" int llmc_gemm_kind(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                              int epi, int kind, hipStream_t s) {
  if (kind < 0) kind = M > 0 && N > 0 ? llmc_gemm_plan(M, N) : 0;
  if (kind == 1) return llmc_gemm_narrow(A, lda, W, ldw, C, ldc, M, N, K, epi, s);
  if (kind != 0) return -1;
  if (K % kTK != 0 || M <= 0 || N <= 0 || K <= 0 || (epi == 3 && N % 2 != 0)) return -1;
  if (lda % 8 != 0 || ldw % 8 != 0) return -1;  // 16-B aligned rows for the LDS-DMA
  // buffer offsets inside one 256-row tile must stay below 2^31 bytes
  if (static_cast<int64_t>(kT) * lda * 2 >= (1ll << 31) || static_cast<int64_t>(kT) * ldw * 2 >= (1ll << 31)) return -1;
  const int nwg = ((M + kT - 1) / kT) * ((N + kT - 1) / kT);
  switch (epi) {
    case 0: gemm256_kernel<0><<<nwg, 512, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, M, N, K); break;
    case 1: gemm256_kernel<1><<<nwg, 512, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, M, N, K); break;
    case 2: gemm256_kernel<2><<<nwg, 512, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, M, N, K); break;
    case 3: gemm256_kernel<3><<<nwg, 512, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)W, ldw, C, ldc, M, N, K); break;
    default: return -2;
  }
  return static_cast<int>(hipGetLastError());
}

extern "C" int llmc_gemm(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                         int epi, hipStream_t s) {
  return llmc_gemm_kind(A, lda, W, ldw, C, ldc, M, N, K, epi, -1, s);
}

// The narrow-N kernel (128 x 192 tiles) on a dense problem: same operands / epilogues as llmc_gemm
// (microbenchmarks, tests and llmc_gemm's narrow-N dispatch).
extern "C" int llmc_gemm_narrow(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                                int epi, hipStream_t s) {
  if (K % kTK != 0 || M <= 0 || N <= 0 || K <= 0 || (epi == 3 && N % 2 != 0) || lda % 8 != 0 || ldw % 8 != 0) return -1;
  if (static_cast<int64_t>(192) * ldw * 2 >= (1ll << 31) || static_cast<int64_t>(128) * lda * 2 >= (1ll << 31)) return -1;
  const int nwg = ((M + 127) / 128) * ((N + 191) / 192);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  switch (epi) {
    case 0: gemm_narrow_kernel<0, 6><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    case 1: gemm_narrow_kernel<1, 6><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    case 2: gemm_narrow_kernel<2, 6><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    case 3: gemm_narrow_kernel<3, 6><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    default: return -2;
  }
  return static_cast<int>(hipGetLastError());
}

// The 128 x 128 two-buffer kernel on a dense problem (microbenchmarks and the narrow-N dispatch
// of llmc_gemm): same operands / epilogues as llmc_gemm.
extern "C" int llmc_gemm_t128(const void* A, int lda, const void* W, int ldw, void* C, int ldc, int M, int N, int K,
                              int epi, hipStream_t s) {
  if (K % kBK != 0 || M <= 0 || N <= 0 || K <= 0 || (epi == 3 && N % 2 != 0) || lda % 8 != 0 || ldw % 8 != 0) return -1;
  const int nwg = ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  switch (epi) {
    case 0: gemm_kernel<0, false><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    case 1: gemm_kernel<1, false><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    case 2: gemm_kernel<2, false><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    case 3: gemm_kernel<3, false><<<nwg, 256, 0, s>>>(a, lda, w, ldw, C, ldc, M, N, K); break;
    default: return -2;
  }
  return static_cast<int>(hipGetLastError());
}

// Grouped expert GEMM over moe_align's padded row list (max_tiles * tile rows of capacity; tile =
// 256: the 256 x 256 LDS-DMA pipeline, 128: the two-buffer 128 x 128 kernel for small groups).
// A: a_rows rows (gathered by sorted_rows / a_row_div); epi 0 bf16, 1 f32, 3 SiLU-mul of
// interleaved gate/up columns into C[., N / 2].
extern "C" int llmc_moe_gemm(const void* A, int lda, int a_rows, const void* W, const void* sorted_rows,
                             const void* tile_expert, const void* tile_count, void* C, int ldc, int N, int K,
                             int max_tiles, int a_row_div, int epi, int tile, hipStream_t s) {
  if (K <= 0 || N <= 0 || K % kTK != 0 || lda % 8 != 0 || K % 8 != 0 || a_rows < 1 || (epi == 3 && N % 2 != 0)) return -1;
  if (epi != 0 && epi != 1 && epi != 3) return -2;
  const int32_t* sr = (const int32_t*)sorted_rows;
  const int32_t* te = (const int32_t*)tile_expert;
  const int32_t* tc = (const int32_t*)tile_count;
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* w = (const bf16_t*)W;
  if (tile == kT) {
    // gathered-row offsets are 32-bit byte offsets into the whole A
    if (static_cast<int64_t>(a_rows) * lda * 2 >= (1ll << 31) || static_cast<int64_t>(kT) * K * 2 >= (1ll << 31))
      return -1;
    const int M = max_tiles * kT, nwg = max_tiles * ((N + kT - 1) / kT);
    switch (epi) {
      case 0: gemm256_kernel<0, true><<<nwg, 512, 0, s>>>(a, lda, w, K, C, ldc, M, N, K, sr, te, tc, a_row_div, a_rows); break;
      case 1: gemm256_kernel<1, true><<<nwg, 512, 0, s>>>(a, lda, w, K, C, ldc, M, N, K, sr, te, tc, a_row_div, a_rows); break;
      default: gemm256_kernel<3, true><<<nwg, 512, 0, s>>>(a, lda, w, K, C, ldc, M, N, K, sr, te, tc, a_row_div, a_rows); break;
    }
    return static_cast<int>(hipGetLastError());
  }
  if (tile != kBM) return -1;
  const int nwg = max_tiles * ((N + kBN - 1) / kBN);
  const int M = max_tiles * kBM;
  switch (epi) {
    case 0: gemm_kernel<0, true><<<nwg, 256, 0, s>>>(a, lda, w, K, C, ldc, M, N, K, sr, te, tc, a_row_div); break;
    case 1: gemm_kernel<1, true><<<nwg, 256, 0, s>>>(a, lda, w, K, C, ldc, M, N, K, sr, te, tc, a_row_div); break;
    default: gemm_kernel<3, true><<<nwg, 256, 0, s>>>(a, lda, w, K, C, ldc, M, N, K, sr, te, tc, a_row_div); break;
  }
  return static_cast<int>(hipGetLastError());
}
