// K6 (batched-decode class): y[m, n] = sum_k x[m, k] * W[n, k] for M = 3..32 rows on the matrix
// cores — the decode step of a continuous batch of up to 32 sequences per engine.
//
// Why a third GEMM shape: the VALU GEMV (gemv_core.h) does 8 v_dot2 per 16-B weight chunk per row,
// so past ~4 rows it turns VALU- and LDS-bound, and the 256 x 256 prefill GEMM launches only
// N / 256 blocks (16 for a 4096-row projection). Here the weight stream stays the whole cost:
//  * one block = 16 weight rows x all of K; its S waves split K (S = 4-8 on model shapes, so the
//    grid holds ~8 waves per CU), wave w owns tiles [w*ntile, (w+1)*ntile) of 128 k.
//  * a tile = 16 rows x 256 B, loaded as four whole 256-B row segments per instruction (lane
//    -> row 4i + lane/16, chunk lane%16; non-temporal), one tile in flight behind the one being
//    computed. The MFMA A fragment wants 16 rows x 64 B per instruction instead (lane -> row
//    lane%16, k 8*(lane/16)): loaded that way the same bytes streamed 1.35x slower, so the tile
//    goes through the wave's own 4 KiB of LDS (chunk c of row q at 16-B slot c ^ q: conflict-free
//    for the 8-lane b128 write groups and the 4 fragment-read groups) — no barrier, one wave.
//  * B fragment = x[lane%16][32j + 8*(lane/16) ..] (x is tiny and L2-resident), 4 per tile.
//  * D[n][m] lands as 4 consecutive rows n (= 4*(lane/16) + t) of one token m (= lane%16) per lane:
//    the (2i, 2i+1) row pairs of the SiLU gate/up and RoPE epilogues meet inside one lane.
//  * PRO_NORM: rmsnorm(x)*w factorises as inv_rms[m] * (x * w): the MFMA takes bf16(x * w) and the
//    epilogue scales by inv_rms[m], whose sum of squares every wave gathers from the x chunks it
//    already loaded (no extra pass over x).
//  * split-K partials meet in LDS (S x 1 KiB); wave 0 runs the fused epilogue: bf16 | f32 |
//    residual add | SiLU-mul | RoPE + paged-KV write (same semantics as the GEMV's).
//  * 17-32 rows (TG = 2 token groups): every A fragment feeds two MFMAs, one per 16-token column
//    group, so the weights still stream once for all rows; each group has its own B fragments,
//    accumulators and norm sums.
// K % 128 == 0 (every model shape); other K take the GEMM path (ops.linear / ops.qkv_rope).
#include "gemv_core.h"

namespace llmc {

// MoE decode (EXP): the (token, slot) pairs of `ids` [P] (local expert ids, -1 = another rank's)
// grouped by expert: block (n, e) streams expert e's rows n once for every pair routed to e (at
// most one per token, so <= 16 for <= 16 tokens); x row of pair p = p / x_div, output row p.
struct ExpertMap {
  const int32_t* ids = nullptr;
  int P = 0, x_div = 1, E = 1;
};

// Fused epilogue of one lane: rows nb .. nb + 3 (f32 accumulators v) of token m.
template <int EPI>
__device__ __forceinline__ void gemvm_epilogue(const f32x4& v, int nb, int m, int N, void* __restrict__ out,
                                               int out_stride, const RopeEpi& rope) {
  if (nb >= N) return;
  const bool full = nb + 3 < N;
  if constexpr (EPI == EPI_F32) {
    float* o = reinterpret_cast<float*>(out) + static_cast<int64_t>(m) * out_stride + nb;
    if (full && (out_stride % 4 == 0)) {
      *reinterpret_cast<f32x4*>(o) = v;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (nb + t < N) o[t] = v[t];
    }
  } else if constexpr (EPI == EPI_BF16 || EPI == EPI_RESADD) {
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + static_cast<int64_t>(m) * out_stride + nb;
    if (full && (out_stride % 4 == 0)) {
      float f[4] = {v[0], v[1], v[2], v[3]};
      if constexpr (EPI == EPI_RESADD) {
        const u32x2 old = *reinterpret_cast<const u32x2*>(o);
        f[0] += bf16_lo(old[0]);
        f[1] += bf16_hi(old[0]);
        f[2] += bf16_lo(old[1]);
        f[3] += bf16_hi(old[1]);
      }
      *reinterpret_cast<u32x2*>(o) = u32x2{pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3])};
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (nb + t >= N) continue;
        o[t] = f32_to_bf16(EPI == EPI_RESADD ? bf16_to_f32(o[t]) + v[t] : v[t]);
      }
    }
  } else if constexpr (EPI == EPI_SILU) {  // rows (2j, 2j + 1) = (gate_j, up_j) -> column j
    bf16_t* o = reinterpret_cast<bf16_t*>(out) + static_cast<int64_t>(m) * out_stride + nb / 2;
    if (full && out_stride % 2 == 0) {  // 4-B aligned pair
      *reinterpret_cast<uint32_t*>(o) = pack_bf16x2(silu(v[0]) * v[1], silu(v[2]) * v[3]);
    } else {
      if (nb + 1 < N) o[0] = f32_to_bf16(silu(v[0]) * v[1]);
      if (nb + 3 < N) o[1] = f32_to_bf16(silu(v[2]) * v[3]);
    }
  } else if constexpr (EPI == EPI_ROPE) {
    // rows (2i, 2i + 1) of a Q/K head = dims (i, i + D/2) (pair-interleaved on the host); V rows
    // keep canonical order. The token's position and KV slot are per lane (token m).
    const int D = rope.D, half = D / 2;
    const int slot = rope.slots[m];
    const int pos = rope.positions[m];
    const int64_t page = slot >= 0 ? slot / rope.bs : 0;
    const int off = slot >= 0 ? slot % rope.bs : 0;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int n = nb + 2 * p;
      if (n + 1 >= N) continue;
      const float a = v[2 * p], b = v[2 * p + 1];
      const int head = n / D;
      if (head < rope.nh + rope.nkv) {
        const int i = (n % D) / 2;
        const int64_t t = static_cast<int64_t>(pos) * half + i;
        const float c = rope.cos_t[t], sn = rope.sin_t[t];
        const float o1 = a * c - b * sn, o2 = b * c + a * sn;
        if (head < rope.nh) {
          bf16_t* qo = rope.q_out + static_cast<int64_t>(m) * rope.q_stride + head * D;
          qo[i] = f32_to_bf16(o1);
          qo[i + half] = f32_to_bf16(o2);
        } else if (slot >= 0) {
          bf16_t* ko = rope.k_cache + ((page * rope.nkv + (head - rope.nh)) * rope.bs + off) * D;
          ko[i] = f32_to_bf16(o1);
          ko[i + half] = f32_to_bf16(o2);
        }
      } else if (slot >= 0) {
        const int vh = head - rope.nh - rope.nkv, d = n % D;
        bf16_t* vv = rope.v_cache + ((page * rope.nkv + vh) * rope.bs + off) * D;
        *reinterpret_cast<uint32_t*>(vv + d) = pack_bf16x2(a, b);
      }
    }
  }
}


template <int S, int RB, int XL, int PRO, int EPI, bool EXP, int TG>
__global__ __launch_bounds__(S * 64) void gemvm_kernel(const bf16_t* __restrict__ x, int x_stride,
                                                       const bf16_t* __restrict__ norm_w, float eps,
                                                       const bf16_t* __restrict__ W, void* __restrict__ out,
                                                       int out_stride, int M, int N, int K, RopeEpi rope,
                                                       ExpertMap ex) {
  static_assert(TG == 1 || (TG == 2 && !EXP), "MoE pairs fit one token group");
  constexpr int TK = 128;       // k per tile: one 256-B LDS bank row per matrix row
  constexpr int WR = 16 * RB;   // weight rows per block (RB 16-row groups share every x fragment)
  constexpr int TB = 16 * TK * 2;
  // per-wave transposition tiles: RB weight row groups (+ the 16 * TG token rows of x when XL)
  __shared__ __attribute__((aligned(16))) char lds_t[S][(RB + XL * TG) * TB];
  __shared__ f32x4 red[S][RB * TG][64];
  __shared__ float ssr[S][16 * TG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * WR;
  // token column m -> x row / output row (identity; MoE: the pairs routed to this block's expert)
  __shared__ int pmap[16];
  if constexpr (EXP) {
    __shared__ int pcnt;
    const int e = blockIdx.y;
    if (wave == 0) {
      const bool hit = lane < ex.P && ex.ids[lane] == e;
      const uint64_t mask = __ballot(hit);
      const int j = __popcll(mask & ((1ull << lane) - 1));
      if (hit && j < 16) pmap[j] = lane;
      if (lane == 0) pcnt = min(__popcll(mask), 16);
    }
    __syncthreads();
    M = pcnt;
    if (M == 0) return;  // no pair routed here: this expert's rows are not streamed
    W += static_cast<int64_t>(e) * N * K;
  }
  auto xrow = [&](int m) { return EXP ? pmap[min(m, M - 1)] / ex.x_div : min(m, M - 1); };
  const int ntile = K / TK / S;  // tiles of this wave (host: K % (TK * S) == 0)
  const int kw = wave * ntile * TK;
  // tile loads: instruction i covers rows 4i + lane/16, 16-B chunk lane%16 — four whole 256-B
  // row segments per instruction (the MFMA fragment order, 16 rows x 64 B per instruction, streamed
  // the same weight bytes 1.35x slower; x, L2-resident, the same way)
  const u32x4* wsrc[4 * RB];
#pragma unroll
  for (int i = 0; i < 4 * RB; ++i)
    wsrc[i] = reinterpret_cast<const u32x4*>(W + static_cast<int64_t>(min(n0 + 4 * i + g, N - 1)) * K + kw + r * 8);
  // x: XL = 1 -> row-contiguous loads transposed through LDS like the weights; XL = 0 -> the B
  // fragments straight from L2 (lane (r, g) loads x[r][32j + 8g ..]; few distinct token rows are
  // mostly broadcasts, cheaper than the LDS round trip)
  const u32x4* xsrc[TG][4];
#pragma unroll
  for (int t = 0; t < TG; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xsrc[t][i] = XL ? reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(xrow(16 * t + 4 * i + g)) * x_stride + kw + r * 8)
                      : reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(xrow(16 * t + r)) * x_stride + kw + g * 8) + 4 * i;
  const u32x4* gp = reinterpret_cast<const u32x4*>(norm_w + kw + g * 8);  // PRO_NORM only
  char* tw = lds_t[wave];
  char* tx = tw + RB * TB;

  auto issue = [&](u32x4 (&wv)[4 * RB], u32x4 (&xv)[TG][4], u32x4 (&gv)[4], int t) {
    const int tu = min(t, ntile - 1) * (TK / 8);  // 16-B units
#pragma unroll
    for (int i = 0; i < 4 * RB; ++i) wv[i] = load16<true>(wsrc[i] + tu);
#pragma unroll
    for (int q = 0; q < TG; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) xv[q][i] = XL ? xsrc[q][i][tu] : xsrc[q][0][tu + 4 * i];
    if constexpr (PRO == PRO_NORM) {
#pragma unroll
      for (int j = 0; j < 4; ++j) gv[j] = gp[tu + 4 * j];
    }
  };
  f32x4 acc[RB][TG];
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int q = 0; q < TG; ++q) acc[b][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[TG];
#pragma unroll
  for (int q = 0; q < TG; ++q) ss[q] = 0.f;
  // row-major tiles -> this wave's LDS (chunk c of row q at 16-B slot c ^ q: conflict-free for the
  // 8-lane b128 write groups and the four 16-lane fragment-read groups) -> fragments (row r,
  // chunk 4j + g): A = weights of each row group, B = x (normalised on the way when PRO_NORM)
  auto consume = [&](const u32x4 (&wv)[4 * RB], const u32x4 (&xv)[TG][4], const u32x4 (&gv)[4]) {
#pragma unroll
    for (int i = 0; i < 4 * RB; ++i) {
      const int q = 4 * i + g;  // weight row within the block
      *reinterpret_cast<u32x4*>(tw + (q >> 4) * TB + (q & 15) * 256 + ((r ^ (q & 15)) << 4)) = wv[i];
    }
    if constexpr (XL) {
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = 4 * i + g;
          *reinterpret_cast<u32x4*>(tx + t * TB + q * 256 + ((r ^ q) << 4)) = xv[t][i];
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int slot = ((4 * j + g) ^ r) << 4;
      u32x4 xb[TG];
#pragma unroll
      for (int t = 0; t < TG; ++t) {
        xb[t] = XL ? *reinterpret_cast<const u32x4*>(tx + t * TB + r * 256 + slot) : xv[t][j];
        if constexpr (PRO == PRO_NORM) {
          float f[8], w8[8];
          unpack8(xb[t], f);
          unpack8(gv[j], w8);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            ss[t] += f[e] * f[e];
            f[e] *= w8[e];
          }
          xb[t] = pack8(f);
        }
      }
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        const u32x4 a = *reinterpret_cast<const u32x4*>(tw + b * TB + r * 256 + slot);
#pragma unroll
        for (int t = 0; t < TG; ++t)
          acc[b][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                              __builtin_bit_cast(bf16x8, xb[t]), acc[b][t], 0, 0, 0);
      }
    }
  };
  u32x4 wc[4 * RB], xc[TG][4], gc[4];
  issue(wc, xc, gc, 0);
  for (int t = 0; t + 1 < ntile; ++t) {
    u32x4 wn[4 * RB], xn[TG][4], gn[4];
    issue(wn, xn, gn, t + 1);
    consume(wc, xc, gc);
#pragma unroll
    for (int i = 0; i < 4 * RB; ++i) wc[i] = wn[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int q = 0; q < TG; ++q) xc[q][i] = xn[q][i];
      if constexpr (PRO == PRO_NORM) gc[i] = gn[i];
    }
  }
  consume(wc, xc, gc);

  // ---- split-K reduction over the block's waves ----
#pragma unroll
  for (int b = 0; b < RB; ++b)
#pragma unroll
    for (int t = 0; t < TG; ++t) red[wave][b * TG + t][lane] = acc[b][t];
  if constexpr (PRO == PRO_NORM) {
#pragma unroll
    for (int t = 0; t < TG; ++t) {
      float v = ss[t];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) ssr[wave][16 * t + r] = v;
    }
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int t = 0; t < TG; ++t) {
    const int m = 16 * t + r;
    if (m >= M) continue;
    float inv = 1.f;
    if constexpr (PRO == PRO_NORM) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < S; ++w) sum += ssr[w][m];
      inv = rsqrtf(sum / K + eps);
    }
#pragma unroll
    for (int b = 0; b < RB; ++b) {
      f32x4 v = red[0][b * TG + t][lane];
#pragma unroll
      for (int w = 1; w < S; ++w) v += red[w][b * TG + t][lane];
      if constexpr (PRO == PRO_NORM) v *= inv;
      gemvm_epilogue<EPI>(v, n0 + 16 * b + 4 * g, EXP ? pmap[m] : m, N, out, out_stride, rope);
    }
  }
}

// Form per shape (profiles/r2_batched_decode.md, `microbench_kernels.py gemvm-forms`): two 16-row
// weight groups per wave from 6144 output rows (8B qkv / gate_up / lm_head: 3-8 % faster; the
// 4096-row o_proj / down lose 25-45 % with half the blocks), x through LDS once the distinct token
// rows make its fragment loads cost (12+ rows; 8+ with one group per wave).
// Two token groups (17-32 rows): x from L2 with two row groups per wave (the LDS x tiles of both
// token groups beside two weight groups would not fit 160 KiB at 8 waves), x through LDS with one.
static int gemvm_form(int M, int N, int K) {
  (void)K;
  const bool rb2 = N >= 6144;
  if (M > 16) return rb2 ? 3 : 2;
  const bool xl = rb2 ? M >= 12 : M >= 8;
  return 1 + (xl ? 1 : 0) + (rb2 ? 2 : 0);
}

template <int S, int RB, int XL, int PRO, int EPI, bool EXP>
static int launch_gemvm_s(const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                          int out_stride, int M, int N, int K, const RopeEpi& rope, const ExpertMap& ex,
                          hipStream_t st) {
  const dim3 grid((N + 16 * RB - 1) / (16 * RB), EXP ? ex.E : 1);
  if constexpr (!EXP && !(RB == 2 && XL == 1)) {
    if (M > 16) {
      gemvm_kernel<S, RB, XL, PRO, EPI, EXP, 2><<<grid, S * 64, 0, st>>>(
          (const bf16_t*)x, x_stride, (const bf16_t*)nw, eps, (const bf16_t*)W, out, out_stride, M, N, K, rope, ex);
      return static_cast<int>(hipGetLastError());
    }
  }
  if (M > 16) return -6;  // two token groups: not with two LDS x tiles beside two weight groups
  gemvm_kernel<S, RB, XL, PRO, EPI, EXP, 1><<<grid, S * 64, 0, st>>>(
      (const bf16_t*)x, x_stride, (const bf16_t*)nw, eps, (const bf16_t*)W, out, out_stride, M, N, K, rope, ex);
  return static_cast<int>(hipGetLastError());
}

// Waves per block: enough split-K that the grid holds ~8 waves per CU (2048), while every wave
// keeps >= 2 tiles of 128 k (one in flight behind the one it computes) and the tiles divide
// evenly (at least 4 waves when K allows it; at most 8: 16 x 64 threads would cap a lane at 128
// VGPRs and spill).
static int pick_split(int blocks, int K) {
  const int tiles = K / 128;
  int S = 1;
  while (S < 8 && tiles % (2 * S) == 0 &&
         (S < 4 || (static_cast<long>(blocks) * S < 2048 && tiles / (2 * S) >= 2)))
    S *= 2;
  return S;
}

template <int RB, int XL, int PRO, int EPI, bool EXP>
static int launch_gemvm_rb(const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                           int out_stride, int M, int N, int K, const RopeEpi& rope, const ExpertMap& ex,
                           hipStream_t st) {
#define LLMC_S(SS) \
  return launch_gemvm_s<SS, RB, XL, PRO, EPI, EXP>(x, x_stride, nw, eps, W, out, out_stride, M, N, K, rope, ex, st)
  switch (pick_split((N + 16 * RB - 1) / (16 * RB), K)) {
    case 1: LLMC_S(1);
    case 2: LLMC_S(2);
    case 4: LLMC_S(4);
    case 8: LLMC_S(8);
    default: return -1;
  }
#undef LLMC_S
}

// form: 0 = by shape (gemvm_form); 1-4 pin (row groups, x path) = (1, L2), (1, LDS), (2, L2),
// (2, LDS) (microbenchmarks / tests)
template <int PRO, int EPI, bool EXP = false>
static int launch_gemvm(const void* x, int x_stride, const void* nw, float eps, const void* W, void* out,
                        int out_stride, int M, int N, int K, const RopeEpi& rope, int form, hipStream_t st,
                        const ExpertMap& ex = ExpertMap{}) {
  if (form == 0) form = gemvm_form(M, N, K);
#define LLMC_F(RB, XL) \
  return launch_gemvm_rb<RB, XL, PRO, EPI, EXP>(x, x_stride, nw, eps, W, out, out_stride, M, N, K, rope, ex, st)
  switch (form) {
    case 1: LLMC_F(1, 0);
    case 2: LLMC_F(1, 1);
    case 3: LLMC_F(2, 0);
    case 4: LLMC_F(2, 1);
    default: return -1;
  }
#undef LLMC_F
}

int gemvm_dispatch(int M, const void* x, int x_stride, const void* norm_w, float eps, const void* W, void* out,
                   int out_stride, int N, int K, int epi, const RopeEpi& rope, hipStream_t st, int form) {
  if (M < 1 || M > kGemvmMaxM || K % 128 != 0 || x_stride % 8 != 0) return -1;
  if ((epi == EPI_SILU || epi == EPI_ROPE) && N % 4 != 0) return -1;
  const bool norm = norm_w != nullptr;
#define LLMC_GEMVM_CASE(E)                                                                                    \
  case E:                                                                                                     \
    return norm ? launch_gemvm<PRO_NORM, E>(x, x_stride, norm_w, eps, W, out, out_stride, M, N, K, rope, form, st) \
                : launch_gemvm<PRO_NONE, E>(x, x_stride, norm_w, eps, W, out, out_stride, M, N, K, rope, form, st);
  switch (epi) {
    LLMC_GEMVM_CASE(EPI_BF16)
    LLMC_GEMVM_CASE(EPI_F32)
    LLMC_GEMVM_CASE(EPI_RESADD)
    LLMC_GEMVM_CASE(EPI_SILU)
    case EPI_ROPE:
      if (!norm) return -5;
      return launch_gemvm<PRO_NORM, EPI_ROPE>(x, x_stride, norm_w, eps, W, out, out_stride, M, N, K, rope, form, st);
    default: return -4;
  }
#undef LLMC_GEMVM_CASE
}

}  // namespace llmc

// Direct entry (tests / microbenchmarks: the MFMA form at any M <= 32).
extern "C" int llmc_gemvm(int M, const void* x, int x_stride, const void* norm_w, float eps, const void* W, void* out,
                          int out_stride, int N, int K, int epi, int form, hipStream_t s) {
  if (epi == llmc::EPI_ROPE) return -5;
  llmc::RopeEpi rope{};
  return llmc::gemvm_dispatch(M, x, x_stride, norm_w, eps, W, out, out_stride, N, K, epi, rope, s, form);
}

// MoE decode, pairs grouped by expert (see ExpertMap): out[p] = W[ids[p]] . x[p / x_div] (+ fused
// norm on x / SiLU), for P <= 64 pairs of <= 16 tokens. Rows of other ranks' pairs (id -1) are
// not written.
extern "C" int llmc_moe_gemvm(int P, const void* x, int x_stride, const void* norm_w, float eps, const void* W,
                              const void* ids, int x_div, int E, void* out, int out_stride, int N, int K, int epi,
                              hipStream_t s) {
  using namespace llmc;
  // P <= 64: one wave's ballot maps the pairs; <= 16 pairs per expert holds for <= 16 tokens with
  // distinct experts per token (the caller's contract: ops.moe_gemvm checks the token count)
  if (P < 1 || P > 64 || x_div < 1 || E < 1 || K % 128 != 0 || x_stride % 8 != 0) return -1;
  if (epi == EPI_SILU && N % 4 != 0) return -1;
  ExpertMap ex{static_cast<const int32_t*>(ids), P, x_div, E};
  const int form = 1 + (N >= 6144 ? 2 : 0);  // few pairs per expert: x fragments from L2
  RopeEpi rope{};
  const bool norm = norm_w != nullptr;
  switch (epi) {
    case EPI_BF16:
      return norm ? launch_gemvm<PRO_NORM, EPI_BF16, true>(x, x_stride, norm_w, eps, W, out, out_stride, kMoeGemvmMaxTokens, N, K,
                                                           rope, form, s, ex)
                  : launch_gemvm<PRO_NONE, EPI_BF16, true>(x, x_stride, norm_w, eps, W, out, out_stride, kMoeGemvmMaxTokens, N, K,
                                                           rope, form, s, ex);
    case EPI_SILU:
      return norm ? launch_gemvm<PRO_NORM, EPI_SILU, true>(x, x_stride, norm_w, eps, W, out, out_stride, kMoeGemvmMaxTokens, N, K,
                                                           rope, form, s, ex)
                  : launch_gemvm<PRO_NONE, EPI_SILU, true>(x, x_stride, norm_w, eps, W, out, out_stride, kMoeGemvmMaxTokens, N, K,
                                                           rope, form, s, ex);
    default: return -4;
  }
}
