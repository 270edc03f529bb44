// K6 (decode class): skinny GEMM  y[m, n] = sum_k x[m, k] * W[n, k]   for M = 1..4 rows.
//
// Batch-1 decode is HBM-bound weight streaming (8B = 15 GB/token), so this is
// THE hot kernel. Design (cdna_hip_programming.md §5 row "GEMV / M <= 16"; MI355X_MICROARCH
// rows nt-weights, launches-baseline):
//  * W [N, K] bf16, K contiguous. A wave owns RPW output rows; lane l streams chunks
//    c = l + 64 i (16 B = 8 bf16 each) of all RPW rows -> RPW*UNROLL independent 16 B loads in
//    flight per lane, straight to VGPRs (no LDS round trip for W), non-temporal (read once).
//  * x is staged ONCE per block in LDS (M*K bf16); every lane reads the same chunk index it
//    loads from W, so ds_read_b128 addresses are lane-consecutive (conflict-free).
//  * v_dot2_f32_bf16 does convert+multiply+accumulate of 2 elements per VALU op.
//  * Fused prologue  PRO_NORM: x <- bf16(rmsnorm(x) * w_norm)  (the layer's input norm), so the
//    decode layer needs no separate norm launch.
//  * Fused epilogues: bf16 store | f32 store (logits) | in-place residual add h += W.x |
//    SiLU-mul over interleaved gate/up rows (row 2i = gate_i, 2i+1 = up_i).
#include "common.h"

#include "gemv_core.h"

namespace llmc {

template <int M, int PRO, int EPI>
static int launch_gemv(const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                       int out_stride, int N, int K, hipStream_t s) {
  constexpr int RPW = 4;
  constexpr int UNROLL = (M <= 2) ? 4 : 2;
  auto kern = gemv_kernel<M, RPW, UNROLL, PRO, EPI>;
  const size_t lds = static_cast<size_t>(M) * K * sizeof(bf16_t) + M * kGemvWaves * sizeof(float);
  if (lds > 160 * 1024) return -2;
  static bool attr_set = false;
  if (lds > 64 * 1024 && !attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    attr_set = true;
  }
  const int rows_per_block = kGemvWaves * RPW;
  const int grid = (N + rows_per_block - 1) / rows_per_block;
  kern<<<grid, kGemvThreads, lds, s>>>((const bf16_t*)x, x_stride, (const bf16_t*)nw, eps, (const bf16_t*)W, out,
                                       out_stride, N, K, nullptr, 1);
  return static_cast<int>(hipGetLastError());
}

template <int PRO, int EPI>
static int dispatch_m(int M, const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                      int out_stride, int N, int K, hipStream_t s) {
  switch (M) {
    case 1: return launch_gemv<1, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, s);
    case 2: return launch_gemv<2, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, s);
    case 3: return launch_gemv<3, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, s);
    case 4: return launch_gemv<4, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, s);
    default: return -3;
  }
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_gemv(int M, const void* x, int x_stride, const void* norm_w, float eps, const void* W, void* out,
                         int out_stride, int N, int K, int epi, hipStream_t s) {
  if (K % 8 != 0) return -1;
  if (epi == EPI_SILU && (N % 2 != 0)) return -1;
  const bool norm = norm_w != nullptr;
#define LLMC_GEMV_CASE(E)                                                                             \
  case E:                                                                                             \
    return norm ? dispatch_m<PRO_NORM, E>(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, s)   \
                : dispatch_m<PRO_NONE, E>(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, s);
  switch (epi) {
    LLMC_GEMV_CASE(EPI_BF16)
    LLMC_GEMV_CASE(EPI_F32)
    LLMC_GEMV_CASE(EPI_RESADD)
    LLMC_GEMV_CASE(EPI_SILU)
    default: return -4;
  }
#undef LLMC_GEMV_CASE
}

// MoE decode (K11 at batch 1): one GEMV per (token, top-k slot) pair against the selected
// expert's weights; expert ids are read on device, so the launch is graph-replayable.
extern "C" int llmc_moe_gemv(int npairs, const void* x, int x_stride, const void* norm_w, float eps, const void* W,
                             const void* ids, int x_div, void* out, int out_stride, int N, int K, int epi,
                             hipStream_t s) {
  if (K % 8 != 0 || norm_w != nullptr) return -1;
  constexpr int RPW = 4, UNROLL = 4;
  const size_t lds = static_cast<size_t>(K) * sizeof(bf16_t) + kGemvWaves * sizeof(float);
  if (lds > 64 * 1024) return -2;
  dim3 grid((N + kGemvWaves * RPW - 1) / (kGemvWaves * RPW), npairs);
#define LLMC_MOEGV(E)                                                                                              \
  gemv_kernel<1, RPW, UNROLL, PRO_NONE, E, true><<<grid, kGemvThreads, lds, s>>>(                                 \
      (const bf16_t*)x, x_stride, nullptr, eps, (const bf16_t*)W, out, out_stride, N, K, (const int32_t*)ids, x_div)
  switch (epi) {
    case EPI_BF16: LLMC_MOEGV(EPI_BF16); break;
    case EPI_SILU: LLMC_MOEGV(EPI_SILU); break;
    default: return -4;
  }
#undef LLMC_MOEGV
  return static_cast<int>(hipGetLastError());
}
