// Launchers for the decode GEMV (kernel body: gemv_core.h).
//
// Geometry (cold-weight sweep on MI355X, scripts/microbench_kernels.py sweep,
// profiles/r1_gemv_geometry_sweep.md): fat blocks (8-16 waves), one row per wave, 4 x 16 B loads
// per lane in flight (+ the next batch prefetched) were fastest on every Llama-3-8B shape: x is
// staged/normalised once per 8-16 rows, and 12-16 waves per CU keep streaming. The waves per
// block are picked so the grid fills whole rounds of the 256 CUs (pick_waves). Paired epilogues
// (SiLU gate/up, RoPE) meet their partner row of the next wave through LDS (PAIR_LDS); shapes
// that do not tile keep 256 threads x 2 rows/wave.
#include <cstdlib>

#include "gemv_core.h"

namespace llmc {

template <int M, int NT, int RPW, int PRO, int EPI, int UNROLL_OVERRIDE = 0>
static int launch_gemv_g(const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                         int out_stride, int N, int K, const RopeEpi& rope, hipStream_t s) {
  constexpr int UNROLL = UNROLL_OVERRIDE ? UNROLL_OVERRIDE : (RPW == 1 ? 4 : (RPW == 2 ? 4 : (M <= 2 ? 4 : 2)));
  constexpr int WAVES = NT / kWave;
  auto kern = gemv_kernel<M, NT, RPW, UNROLL, PRO, EPI, false>;
  // x [M][K] bf16 | norm partials [M][WAVES] f32 | pair exchange [WAVES/2][M] f32
  const size_t lds = static_cast<size_t>(M) * K * sizeof(bf16_t) + 2 * M * WAVES * sizeof(float);
  if (lds > 160 * 1024) return -2;
  static bool attr_set = false;
  if (lds > 64 * 1024 && !attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  const int rows_per_block = WAVES * RPW;
  const int grid = (N + rows_per_block - 1) / rows_per_block;
  kern<<<grid, NT, lds, s>>>((const bf16_t*)x, x_stride, (const bf16_t*)nw, eps, (const bf16_t*)W, out, out_stride, N,
                             K, nullptr, 1, rope, CarArgs{});
  return static_cast<int>(hipGetLastError());
}

// Waves per block so that the grid fills whole rounds of the 256 CUs (a 6144-row qkv at 16
// rows/block = 384 blocks leaves half the CUs with twice the work; 12 rows/block = 512 blocks
// is exact): the smallest idle fraction of the last round, ties to the larger block.
static int pick_waves(int N, bool paired) {
  // short outputs (a TP rank's qkv: 768 / 1536 rows) cannot fill the chip with fat blocks: 4-wave
  // blocks with 8 loads per lane spread them over 3-6x the CUs (768x4096: 4.04 vs 5.68 us,
  // profiles/r1_attn_decode_tp_shapes.md)
  if (N < 2048 && (!paired || N % 8 == 0)) return 4;
  // 10-wave blocks: a 70B TP=4 rank's qkv (2560 rows) is 256 blocks of 10 rows instead of 160 of 16
  // (96 CUs idle)
  // 14-wave blocks (paired outputs): a TP=8 / TP=4 rank's gate_up (3584 / 7168 rows) is 256 / 512
  // blocks instead of 224 / 448
  static const bool no10 = std::getenv("LLMC_GEMV_NO_W10") != nullptr;  // A/B runs only
  static const bool no14 = std::getenv("LLMC_GEMV_NO_W14") != nullptr;
  int best = 16;
  double best_idle = 2.0;
  for (int w : {16, 14, 12, 10, 8}) {
    if ((w == 10 && no10) || (w == 14 && (no14 || !paired))) continue;
    if (paired && N % (2 * w) != 0) continue;
    const long blocks = (N + w - 1) / w;
    const long slots = (blocks + 255) / 256 * 256;
    const double idle = static_cast<double>(slots - blocks) / static_cast<double>(slots);
    if (idle < best_idle - 1e-9) {
      best_idle = idle;
      best = w;
    }
  }
  return best_idle > 1.0 ? 0 : best;
}

template <int M, int PRO, int EPI>
static int launch_gemv(const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                       int out_stride, int N, int K, const RopeEpi& rope, hipStream_t s) {
  constexpr bool paired = EPI == EPI_SILU || EPI == EPI_ROPE;
  const int w = pick_waves(N, paired);
  // long rows on few blocks (a 70B TP=4 rank's qkv: 2560 x 8192 = 160 fat blocks): 8 loads per
  // lane in flight instead of 4 (9.67 vs 10.99 us, profiles/r1_attn_decode_tp_shapes.md). One or
  // two rows only: with 3-4 rows (the VALU form runs them only when K is off the MFMA form's 128-k
  // tiles) that geometry kept 20-48 B per lane in scratch (tests/test_kernel_plan_cpu.py)
  if constexpr (M <= 2) {
    // the RoPE epilogue with both rows of a pair in one wave (no LDS pair exchange behind a block
    // barrier) where that still fills whole rounds: Llama-3-8B / Mixtral qkv (6144 rows) as 256
    // blocks of 12 waves x 2 rows
    static const bool rope_rpw1 = std::getenv("LLMC_GEMV_ROPE_RPW1") != nullptr;  // A/B runs only
    if (EPI == EPI_ROPE && w == 12 && N % (2 * 12 * 256) == 0 && !rope_rpw1)
      return launch_gemv_g<M, 768, 2, PRO, EPI, 4>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    // ... and the SiLU gate/up pairs, at the widest block that still fills whole rounds with two rows
    // per wave (8B gate_up 28672 rows: 14 waves, 1024 blocks; Phi-3 16384: 16 waves, 512)
    static const bool silu_rpw1 = std::getenv("LLMC_GEMV_SILU_RPW1") != nullptr;  // A/B runs only
    if (EPI == EPI_SILU && !silu_rpw1 && K < 8192) {
      if (N % (2 * 16 * 256) == 0)
        return launch_gemv_g<M, 1024, 2, PRO, EPI, 4>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
      if (N % (2 * 14 * 256) == 0)
        return launch_gemv_g<M, 896, 2, PRO, EPI, 4>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    }
    if (w == 16 && K >= 8192 && N <= 4096)
      return launch_gemv_g<M, 1024, 1, PRO, EPI, 8>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    if (w == 10 && K >= 8192)
      return launch_gemv_g<M, 640, 1, PRO, EPI, 8>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
  }
  switch (w) {
    case 16: return launch_gemv_g<M, 1024, 1, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 14: return launch_gemv_g<M, 896, 1, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 12: return launch_gemv_g<M, 768, 1, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 10: return launch_gemv_g<M, 640, 1, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 8: return launch_gemv_g<M, 512, 1, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 4: return launch_gemv_g<M, 256, 1, PRO, EPI, 8>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    default:  // paired rows that do not tile by 16-32 rows: pairs inside one wave
      return launch_gemv_g<M, 256, 2, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
  }
}

template <int PRO, int EPI>
static int dispatch_m(int M, const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                      int out_stride, int N, int K, const RopeEpi& rope, hipStream_t s) {
  switch (M) {
    case 1: return launch_gemv<1, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 2: return launch_gemv<2, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 3: return launch_gemv<3, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    case 4: return launch_gemv<4, PRO, EPI>(x, x_stride, nw, eps, W, out, out_stride, N, K, rope, s);
    default: return -3;
  }
}

static int gemv_dispatch(int M, const void* x, int x_stride, const void* norm_w, float eps, const void* W, void* out,
                         int out_stride, int N, int K, int epi, const RopeEpi& rope, bool mfma, hipStream_t s) {
  if (K % 8 != 0) return -1;
  if ((epi == EPI_SILU || epi == EPI_ROPE) && (N % 2 != 0)) return -1;
  // 3-16 rows: the MFMA form (profiles/r2_batched_decode.md: from 3 rows on the VALU dot products,
  // not the weight stream, set this kernel's time); 1-2 rows, or K off the 128-k tiles: VALU GEMV.
  // `mfma` pins the MFMA form at every row count: an engine that batches >= 3 rows decodes all its
  // steps on one form, so a request's tokens do not depend on how many rows shared its steps.
  if ((M > kGemvMaxM || mfma) && K % 128 == 0 && x_stride % 8 == 0)
    return gemvm_dispatch(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, epi, rope, s);
  const bool norm = norm_w != nullptr;
#define LLMC_GEMV_CASE(E)                                                                                   \
  case E:                                                                                                   \
    return norm ? dispatch_m<PRO_NORM, E>(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, rope, s)   \
                : dispatch_m<PRO_NONE, E>(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, rope, s);
  switch (epi) {
    LLMC_GEMV_CASE(EPI_BF16)
    LLMC_GEMV_CASE(EPI_F32)
    LLMC_GEMV_CASE(EPI_RESADD)
    LLMC_GEMV_CASE(EPI_SILU)
    case EPI_ROPE:
      if (!norm) return -5;
      return dispatch_m<PRO_NORM, EPI_ROPE>(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, rope, s);
    default: return -4;
  }
#undef LLMC_GEMV_CASE
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_gemv(int M, const void* x, int x_stride, const void* norm_w, float eps, const void* W, void* out,
                         int out_stride, int N, int K, int epi, int mfma, hipStream_t s) {
  if (epi == EPI_ROPE) return -5;
  RopeEpi rope{};
  return gemv_dispatch(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, epi, rope, mfma != 0, s);
}

// qkv projection for decode with fused RMSNorm prologue and RoPE + paged-KV-write epilogue.
extern "C" int llmc_gemv_qkv_rope(int M, const void* x, int x_stride, const void* norm_w, float eps, const void* W,
                                  int N, int K, void* q_out, int q_stride, void* k_cache, void* v_cache,
                                  const void* positions, const void* slots, const void* cos_t, const void* sin_t,
                                  int nh, int nkv, int D, int bs, int mfma, hipStream_t s) {
  if (N != (nh + 2 * nkv) * D || D % 2 != 0) return -1;
  RopeEpi rope{(bf16_t*)q_out, q_stride, (bf16_t*)k_cache, (bf16_t*)v_cache, (const int32_t*)positions,
               (const int32_t*)slots, (const float*)cos_t, (const float*)sin_t, nh, nkv, D, bs};
  return gemv_dispatch(M, x, x_stride, norm_w, eps, W, nullptr, 0, N, K, EPI_ROPE, rope, mfma != 0, s);
}

// Row-parallel decode projection with the all-reduce fused into the epilogue (EPI_AR, gemv_core.h):
// h = sum over ranks of W_r . x_r (+ h on rank 0), for M <= 2 tokens. `bases`: every rank's fused-AR
// buffer (car_proto.h layout), `cap` its bytes per data parity.
namespace llmc {
template <int M, int NT, int UNROLL>
static int launch_gemv_ar(const void* x, int x_stride, const void* W, void* h, int h_stride, int N, int K,
                          const CarArgs& ar, hipStream_t s) {
  constexpr int WAVES = NT / kWave;
  auto kern = gemv_kernel<M, NT, 1, UNROLL, PRO_NONE, EPI_AR, false>;
  const size_t lds = static_cast<size_t>(M) * K * sizeof(bf16_t) + 2 * M * WAVES * sizeof(float);
  if (lds > 160 * 1024) return -2;
  static bool attr_set = false;
  if (lds > 64 * 1024 && !attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  const int grid = (N + WAVES - 1) / WAVES;
  if (grid > kMaxBlocks || static_cast<size_t>(grid) * kArGranulesPerBlock * 8 > static_cast<size_t>(ar.cap) / kMaxRanks)
    return -6;
  kern<<<grid, NT, lds, s>>>((const bf16_t*)x, x_stride, nullptr, 0.f, (const bf16_t*)W, h, h_stride, N, K, nullptr, 1,
                             RopeEpi{}, ar);
  return static_cast<int>(hipGetLastError());
}

template <int M>
static int gemv_ar_geom(const void* x, int x_stride, const void* W, void* h, int h_stride, int N, int K,
                        const CarArgs& ar, hipStream_t s) {
  // the dense GEMV's geometry rule (pick_waves): same blocks, same accumulation order, same bits
  const int w = pick_waves(N, false);
  if (w == 16 && K >= 8192 && N <= 4096) return launch_gemv_ar<M, 1024, 8>(x, x_stride, W, h, h_stride, N, K, ar, s);
  if (w == 10 && K >= 8192) return launch_gemv_ar<M, 640, 8>(x, x_stride, W, h, h_stride, N, K, ar, s);
  switch (w) {
    case 16: return launch_gemv_ar<M, 1024, 4>(x, x_stride, W, h, h_stride, N, K, ar, s);
    case 12: return launch_gemv_ar<M, 768, 4>(x, x_stride, W, h, h_stride, N, K, ar, s);
    case 10: return launch_gemv_ar<M, 640, 4>(x, x_stride, W, h, h_stride, N, K, ar, s);
    case 8: return launch_gemv_ar<M, 512, 4>(x, x_stride, W, h, h_stride, N, K, ar, s);
    case 4: return launch_gemv_ar<M, 256, 8>(x, x_stride, W, h, h_stride, N, K, ar, s);
    default: return -7;
  }
}
}  // namespace llmc

extern "C" int llmc_gemv_ar(int M, const void* x, int x_stride, const void* W, void* h, int h_stride, int N, int K,
                            const void* const* bases, void* host, int rank, int world, size_t cap, hipStream_t s) {
  if (K % 8 != 0 || N % 2 != 0 || world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return -1;
  CarArgs ar{};
  for (int r = 0; r < kMaxRanks; ++r)
    ar.P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
  ar.P.host = static_cast<uint32_t*>(host);
  ar.rank = rank;
  ar.world = world;
  ar.cap = static_cast<long>(cap);
  switch (M) {
    case 1: return gemv_ar_geom<1>(x, x_stride, W, h, h_stride, N, K, ar, s);
    case 2: return gemv_ar_geom<2>(x, x_stride, W, h, h_stride, N, K, ar, s);
    default: return -3;
  }
}

// MoE decode (K11 at batch 1): one GEMV per (token, top-k slot) pair against the selected
// expert's weights; expert ids are read on device, so the launch is graph-replayable.
namespace llmc {
template <int NT, int RPW, int EPI, int PRO>
static int launch_moe_gemv(int npairs, const void* x, int x_stride, const void* nw, float eps, const void* W,
                           const void* ids, int x_div, void* out, int out_stride, int N, int K, hipStream_t s) {
  constexpr int WAVES = NT / kWave;
  const size_t lds = static_cast<size_t>(K) * sizeof(bf16_t) + 2 * WAVES * sizeof(float);
  if (lds > 64 * 1024) return -2;
  dim3 grid((N + WAVES * RPW - 1) / (WAVES * RPW), npairs);
  gemv_kernel<1, NT, RPW, 4, PRO, EPI, true><<<grid, NT, lds, s>>>(
      (const bf16_t*)x, x_stride, (const bf16_t*)nw, eps, (const bf16_t*)W, out, out_stride, N, K,
      (const int32_t*)ids, x_div, RopeEpi{}, CarArgs{});
  return static_cast<int>(hipGetLastError());
}

template <int EPI, int PRO>
static int moe_gemv_geom(int npairs, const void* x, int x_stride, const void* nw, float eps, const void* W,
                         const void* ids, int x_div, void* out, int out_stride, int N, int K, hipStream_t s) {
  // same geometry rule as the dense GEMV; the grid's y dimension (token, expert) pairs multiplies
  // the rounds, so whole rounds per pair are whole rounds overall. SiLU pairs in one wave where
  // that fills whole rounds (Mixtral's expert gate_up, 28672 rows: 14 waves x 2 rows), as the
  // dense launcher does
  static const bool silu_rpw1 = std::getenv("LLMC_GEMV_SILU_RPW1") != nullptr;  // A/B runs only
  if (EPI == EPI_SILU && !silu_rpw1 && K < 8192) {
    if (N % (2 * 16 * 256) == 0)
      return launch_moe_gemv<1024, 2, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    if (N % (2 * 14 * 256) == 0)
      return launch_moe_gemv<896, 2, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
  }
  switch (pick_waves(N, EPI == EPI_SILU)) {
    case 16: return launch_moe_gemv<1024, 1, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    case 14: return launch_moe_gemv<896, 1, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    case 12: return launch_moe_gemv<768, 1, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    case 10: return launch_moe_gemv<640, 1, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    case 8: return launch_moe_gemv<512, 1, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    case 4: return launch_moe_gemv<256, 1, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    default: return launch_moe_gemv<256, 2, EPI, PRO>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
  }
}
}  // namespace llmc

// MoE decode down projection fused with the combine: h[t] += sum_j w[t, j] * (W_down[ids[t, j]] . act[t*k + j])
// for top-2 routing (k == 2), one block per 16 output rows per token, each wave streaming its row
// of both experts. Expert-parallel ranks (ids -1) keep the separate GEMV + combine.
// MoE decode down projection fused with the combine: h[t] += sum_j w[t, j] * (W_down[ids[t, j]] . act[t*k + j])
// for top-2 routing (k == 2), one block per 16 output rows per token, each wave streaming its row
// of both experts. Expert-parallel ranks (ids -1) keep the separate GEMV + combine.
// (Measured against 512 threads x 4 / 1024 x 2 / 512 x 8 loads per lane: none faster,
// profiles/r6_decode_experiments.md.)
extern "C" int llmc_moe_down_combine(int T, const void* act, int act_stride, const void* W, const void* ids,
                                     const void* w, void* h, int h_stride, int N, int K, int k, hipStream_t s) {
  if (k != 2 || K % 8 != 0) return -1;
  constexpr int NT = 1024, WAVES = NT / kWave;
  auto kern = gemv_kernel<2, NT, 2, 4, PRO_NONE, EPI_COMBINE, true>;
  const size_t lds = static_cast<size_t>(2) * K * sizeof(bf16_t) + 2 * 2 * WAVES * sizeof(float);
  if (lds > 160 * 1024) return -2;
  static bool attr_set = false;
  if (lds > 64 * 1024 && !attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  RopeEpi wts{};
  wts.cos_t = static_cast<const float*>(w);
  dim3 grid((N + WAVES - 1) / WAVES, T);
  kern<<<grid, NT, lds, s>>>((const bf16_t*)act, act_stride, nullptr, 0.f, (const bf16_t*)W, h, h_stride, N, K,
                             (const int32_t*)ids, 1, wts, CarArgs{});
  return static_cast<int>(hipGetLastError());
}

extern "C" int llmc_moe_gemv(int npairs, const void* x, int x_stride, const void* norm_w, float eps, const void* W,
                             const void* ids, int x_div, void* out, int out_stride, int N, int K, int epi,
                             hipStream_t s) {
  // norm_w: x is the raw hidden row, RMS-normalised in the prologue (the decode gate_up after the
  // fused router); nullptr: x is used as is (down projection)
  if (K % 8 != 0) return -1;
  const void* nw = norm_w;
  switch (epi) {
    case EPI_BF16:
      return nw ? moe_gemv_geom<EPI_BF16, PRO_NORM>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s)
                : moe_gemv_geom<EPI_BF16, PRO_NONE>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    case EPI_SILU:
      return nw ? moe_gemv_geom<EPI_SILU, PRO_NORM>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s)
                : moe_gemv_geom<EPI_SILU, PRO_NONE>(npairs, x, x_stride, nw, eps, W, ids, x_div, out, out_stride, N, K, s);
    default: return -4;
  }
}

// ---- geometry sweep entry (microbenchmarks only: M = 1, fused norm, bf16 out) ----
namespace llmc {
template <int NT, int RPW, int UNROLL>
static int launch_sweep(const void* x, const void* nw, const void* W, void* out, int N, int K, hipStream_t s) {
  constexpr int WAVES = NT / kWave;
  const size_t lds = static_cast<size_t>(K) * sizeof(bf16_t) + WAVES * sizeof(float);
  const int grid = (N + WAVES * RPW - 1) / (WAVES * RPW);
  gemv_kernel<1, NT, RPW, UNROLL, PRO_NORM, EPI_BF16, false><<<grid, NT, lds, s>>>(
      (const bf16_t*)x, K, (const bf16_t*)nw, 1e-5f, (const bf16_t*)W, out, N, N, K, nullptr, 1, RopeEpi{}, CarArgs{});
  return static_cast<int>(hipGetLastError());
}
}  // namespace llmc

extern "C" int llmc_gemv_sweep(int variant, const void* x, const void* nw, const void* W, void* out, int N, int K,
                               hipStream_t s) {
  if (K % 8 != 0 || K * 2 > 64 * 1024) return -1;
  switch (variant) {
    case 0: return launch_sweep<256, 1, 8>(x, nw, W, out, N, K, s);
    case 1: return launch_sweep<256, 2, 4>(x, nw, W, out, N, K, s);
    case 2: return launch_sweep<256, 4, 4>(x, nw, W, out, N, K, s);
    case 3: return launch_sweep<512, 1, 8>(x, nw, W, out, N, K, s);
    case 4: return launch_sweep<512, 2, 4>(x, nw, W, out, N, K, s);
    case 5: return launch_sweep<128, 1, 8>(x, nw, W, out, N, K, s);
    case 6: return launch_sweep<64, 1, 8>(x, nw, W, out, N, K, s);
    case 7: return launch_sweep<1024, 1, 4>(x, nw, W, out, N, K, s);
    case 8: return launch_sweep<256, 1, 4>(x, nw, W, out, N, K, s);
    case 9: return launch_sweep<256, 2, 8>(x, nw, W, out, N, K, s);
    case 10: return launch_sweep<512, 4, 2>(x, nw, W, out, N, K, s);
    case 11: return launch_sweep<128, 2, 4>(x, nw, W, out, N, K, s);
    case 12: return launch_sweep<1024, 1, 8>(x, nw, W, out, N, K, s);
    case 13: return launch_sweep<1024, 2, 4>(x, nw, W, out, N, K, s);
    case 14: return launch_sweep<1024, 2, 2>(x, nw, W, out, N, K, s);
    case 15: return launch_sweep<1024, 1, 2>(x, nw, W, out, N, K, s);
    case 16: return launch_sweep<768, 1, 4>(x, nw, W, out, N, K, s);
    case 17: return launch_sweep<1024, 4, 2>(x, nw, W, out, N, K, s);
    case 18: return launch_sweep<1024, 1, 6>(x, nw, W, out, N, K, s);
    case 19: return launch_sweep<768, 2, 4>(x, nw, W, out, N, K, s);
    case 20: return launch_sweep<640, 1, 8>(x, nw, W, out, N, K, s);
    case 21: return launch_sweep<896, 1, 4>(x, nw, W, out, N, K, s);
    case 22: return launch_sweep<768, 2, 2>(x, nw, W, out, N, K, s);
    case 23: return launch_sweep<1024, 2, 2>(x, nw, W, out, N, K, s);
    default: return -2;
  }
}
