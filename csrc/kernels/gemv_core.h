// K6 (decode class): skinny GEMM  y[m, n] = sum_k x[m, k] * W[n, k]   for M = 1..4 rows.
//
// Batch-1 decode is HBM-bound weight streaming (8B = 15 GB/token), so this is
// THE hot kernel. Design (cdna_hip_programming.md §5 row "GEMV / M <= 16"; MI355X_MICROARCH
// rows nt-weights, launches-baseline):
//  * W [N, K] bf16, K contiguous. A wave owns RPW output rows; lane l streams chunks
//    c = l + 64 i (16 B = 8 bf16 each) of all RPW rows -> RPW*UNROLL independent 16 B loads in
//    flight per lane, straight to VGPRs (no LDS round trip for W), non-temporal (read once).
//  * Geometry (NT threads, RPW rows/wave) is chosen per shape on the host so the grid is a
//    balanced multiple of the 256 CUs with >= 16 waves/CU in flight (launch_gemv in gemv.hip).
//  * x is staged ONCE per block in LDS (M*K bf16); every lane reads the same chunk index it
//    loads from W, so ds_read_b128 addresses are lane-consecutive (conflict-free).
//  * v_dot2_f32_bf16 does convert+multiply+accumulate of 2 elements per VALU op.
//  * Fused prologue  PRO_NORM: x <- bf16(rmsnorm(x) * w_norm)  (the layer's input norm).
//  * Fused epilogues: bf16 store | f32 store (logits) | in-place residual add h += W.x |
//    SiLU-mul over interleaved gate/up rows (row 2i = gate_i, 2i+1 = up_i) |
//    ROPE: qkv projection with pair-interleaved Q/K head rows -> rotate-half RoPE from the f32
//    accumulators, q to the q buffer, k/v straight into the paged KV cache at the device slot
//    (replaces the separate RoPE + KV-write launch of the decode step).
#pragma once
#include <type_traits>

#include "car_proto.h"
#include "common.h"

namespace llmc {

enum { PRO_NONE = 0, PRO_NORM = 1 };
enum { EPI_BF16 = 0, EPI_F32 = 1, EPI_RESADD = 2, EPI_SILU = 3, EPI_ROPE = 4, EPI_COMBINE = 5, EPI_AR = 6 };

// EPI_AR: a tensor-parallel rank's row-parallel projection (decode o_proj / down_proj) with the
// all-reduce in its own epilogue: h = sum over ranks of (W_r . x_r), rank 0's term carrying the
// residual h. Block b of every rank owns the same rows, so block b only exchanges with block b
// of its peers, over car_proto.h's push protocol (its own buffer, granules [16 b, 16 b + NG) of
// every slot): the block's bf16 partials go straight into every peer's buffer as data-tagged
// granules, and it sums its peers' granules in rank order as they land — the numerics of a
// separate EPI_RESADD / EPI_BF16 GEMV followed by the one-shot all-reduce, bit for bit, without
// that kernel's launch, its boundary and its re-read of h. What holds: every wait is bounded (1 s,
// car_proto.h car_spin; a give-up fails the request on every rank). Forward progress within that
// bound is guaranteed only when each rank owns its GPU and no other engine's blocks can take the
// CUs a peer's blocks need: blocks are dispatched in index order, so on a GPU of its own the lowest
// unfinished block of every rank is resident. Ranks sharing a GPU, or a TP engine beside engines
// that decode at the same time, keep the separate all-reduce launch (comm.py enable_custom,
// placement.fused_ar_allowed). Granules per block: car_proto.h kArGranulesPerBlock.

struct RopeEpi {
  bf16_t* q_out;            // [M, q_stride], canonical head-major layout
  int q_stride;
  bf16_t* k_cache;          // [nb][nkv][bs][D]
  bf16_t* v_cache;
  const int32_t* positions; // [M]
  const int32_t* slots;     // [M]
  const float* cos_t;       // [max_pos][D/2]
  const float* sin_t;
  int nh, nkv, D, bs;
  // optional (qkv_attn.hip): every rotated q / k pair and v pair also published as an 8-B
  // {bf16x2, gtag} granule for the attention blocks of the same launch: q head h pair i at
  // [h][i] = dims (i, i + D/2); k head j at [nh + j][i], same dims; v head j at [nh + nkv + j][d/2]
  // = dims (d, d + 1); D/2 granules per head
  uint64_t* granules;
  uint32_t gtag;
};

// Batched decode (3 <= M <= 32 rows): the MFMA form in gemv_mfma.hip, same prologue/epilogues
// (one 16-token MFMA column group up to 16 rows, two above). This kernel serves M <= kGemvMaxM
// (and M <= 4 when K is not a multiple of 128). MoE pairs stay within one token group.
constexpr int kGemvMaxM = 2, kGemvmMaxM = 32, kMoeGemvmMaxTokens = 16;
int gemvm_dispatch(int M, const void* x, int x_stride, const void* norm_w, float eps, const void* W, void* out,
                   int out_stride, int N, int K, int epi, const RopeEpi& rope, hipStream_t st, int form = 0);

// One block of the GEMV (block (bx, by) of its grid; smem = the block's dynamic LDS): the body of
// gemv_kernel, also the projection role of fused launches (qkv_attn.hip).
template <int M, int NT, int RPW, int UNROLL, int PRO, int EPI, bool EXPERT = false>
__device__ __forceinline__ void gemv_block(const int bx, const int by, char* smem, const bf16_t* __restrict__ x,
                                           int x_stride, const bf16_t* __restrict__ norm_w, float eps,
                                           const bf16_t* __restrict__ W, void* __restrict__ out, int out_stride, int N,
                                           int K, const int32_t* __restrict__ expert_ids, int x_div, const RopeEpi& rope,
                                           const CarArgs& ar) {
  constexpr int WAVES = NT / kWave;
  constexpr bool PAIR_LDS = (EPI == EPI_SILU || EPI == EPI_ROPE) && RPW == 1;  // host: N % (2 * WAVES) == 0
  // RoPE operands through the scalar cache, early (below): one pair per wave (PAIR_LDS: the even
  // wave's row and its partner; RPW == 2: the wave's own two rows)
  constexpr bool ROPE_PRE = EPI == EPI_ROPE && (PAIR_LDS || RPW == 2);
  // EXPERT (MoE decode): by = (token, slot) pair; weights of expert expert_ids[pair],
  // input row pair / x_div, output row pair (M must be 1).
  // EPI_COMBINE (MoE decode down projection fused with the combine; EXPERT, M == RPW == top-k):
  // by = token t; wave row n streams row n of each of the token's k experts ("rows" r =
  // slots), x row r = the slot's activation; acc[r][r] is that expert's output and the epilogue
  // does h[t][n] += sum_r w[t][r] * acc[r][r] in a fixed order (replaces moe_combine's launch and
  // the y round trip). x_div carries nothing here; the router weights come in through `rope.cos_t`.
  constexpr bool COMBINE = EPI == EPI_COMBINE;
  static_assert(!COMBINE || (EXPERT && M == RPW), "combine: one x row per expert slot");
  if constexpr (EXPERT && !COMBINE) {
    const int pair = by;
    if (expert_ids[pair] < 0) return;  // another rank's expert (expert parallel): whole block exits
    W += static_cast<int64_t>(expert_ids[pair]) * N * K;
    x += static_cast<int64_t>(pair / x_div) * x_stride;
    out = reinterpret_cast<char*>(out) + static_cast<int64_t>(pair) * out_stride * (EPI == EPI_F32 ? 4 : 2);
  }
  if constexpr (COMBINE) {
    const int t = by;
    x += static_cast<int64_t>(t) * RPW * x_stride;
    out = reinterpret_cast<char*>(out) + static_cast<int64_t>(t) * out_stride * 2;
  }
  bf16_t* xs = reinterpret_cast<bf16_t*>(smem);  // [M][K]
  const int tid = threadIdx.x;
  const int nchunk = K / 8;
  const int wave = tid / kWave, lane = tid % kWave;
  const int row0 = COMBINE ? bx * WAVES + wave : (bx * WAVES + wave) * RPW;

  // Weight rows (clamped: waves past N still load a valid row and discard it, so no lane
  // diverges before the block barrier). The first UNROLL-batch of W is issued BEFORE the x
  // prologue: W does not depend on x, so the HBM latency of the first batch overlaps the
  // x staging / RMS norm, and the loop keeps the next batch in flight while it computes.
  const u32x4* wrow[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    if constexpr (COMBINE) {
      const int e = expert_ids[by * RPW + r];
      wrow[r] = reinterpret_cast<const u32x4*>(W + (static_cast<int64_t>(e) * N + min(row0, N - 1)) * K);
    } else {
      const int n = min(row0 + r, N - 1);
      wrow[r] = reinterpret_cast<const u32x4*>(W + static_cast<int64_t>(n) * K);
    }
  }
  constexpr int STEP = kWave * UNROLL;
  const int iters = (nchunk + STEP - 1) / STEP;
  u32x4 cur[RPW][UNROLL];
  auto issue = [&](u32x4 (&dst)[RPW][UNROLL], int cbase) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int c = min(cbase + u * kWave, nchunk - 1);  // clamped tail: loads stay batched
#pragma unroll
      for (int r = 0; r < RPW; ++r) dst[r][u] = load16<true>(wrow[r] + c);
    }
  };
  // x (and the norm weights) are loaded BEFORE the first weight batch: vmcnt retires loads in
  // issue order, so the prologue's wait for x then leaves the weight batch in flight, and the main
  // loop issues the second batch while the first is still landing (x last would make the
  // prologue wait for the whole first batch and open a bubble in every wave's stream).
  constexpr bool kXRegs = (PRO == PRO_NORM || PRO == PRO_NONE);
  const bool x_fast = nchunk <= 2 * NT;  // x fits in two 16-B chunks per thread
  u32x4 xr[2][M], gr[2];
  if constexpr (kXRegs) {
    if (x_fast) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = tid + j * NT;
        if (c < nchunk) {
          if constexpr (PRO == PRO_NORM) gr[j] = reinterpret_cast<const u32x4*>(norm_w)[c];
#pragma unroll
          for (int m = 0; m < M; ++m) xr[j][m] = reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(m) * x_stride)[c];
        }
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  issue(cur, lane);
  __builtin_amdgcn_sched_barrier(0);


  // EPI_AR: this block's epoch and (rank 0) the residual of this wave's row, both issued behind the
  // first weight batch (in-order retirement: waiting for them later waits for nothing else)
  uint32_t ar_epoch = 0;
  float ar_resid[M];
  if constexpr (EPI == EPI_AR) {
    static_assert(RPW == 1 && M <= 2 && M * WAVES / 2 <= kArGranulesPerBlock, "EPI_AR geometry");
    if (tid == 0)
      ar_epoch = __hip_atomic_load(car_ctr(ar.P.base[ar.rank]) + bx, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM) + 1;
#pragma unroll
    for (int m = 0; m < M; ++m)
      ar_resid[m] = ar.rank == 0 && row0 < N
                        ? bf16_to_f32(reinterpret_cast<const bf16_t*>(out)[static_cast<int64_t>(m) * out_stride + row0])
                        : 0.f;
  }

  // RoPE epilogue operands (PAIR_LDS: one row per even wave) are wave-uniform, so they come
  // through the SCALAR cache (s_load, counted by lgkmcnt): as vector loads they queued behind the
  // weight stream in the in-order vmcnt counter, and the position -> cos/sin dependency held the
  // second weight batch back by a memory round trip (qkv 11.2 -> ~10.3 us for Llama-3-8B
  // without them). Position and slot are issued here, behind the first weight batch; the
  // dependent cos/sin loads after the prologue, when the position has landed.
  int pre_pos[M], pre_slot[M];
  float pre_c[M], pre_s[M];
  if constexpr (ROPE_PRE) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      pre_slot[m] = ld_scalar(rope.slots + m);
      pre_pos[m] = ld_scalar(rope.positions + m);
    }
  }

  // ---- prologue: x -> LDS (optionally RMS-normalised) ----
  if constexpr (PRO == PRO_NORM) {
    float(*red)[WAVES] = reinterpret_cast<float(*)[WAVES]>(smem + static_cast<size_t>(M) * K * sizeof(bf16_t));
    float ss[M];
#pragma unroll
    for (int m = 0; m < M; ++m) ss[m] = 0.f;
    if (x_fast) {
      // ONE global round trip (issued above): x and the norm weights stay in registers between
      // the sum of squares and the normalisation (K <= 16 Ki at 1024 threads)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (tid + j * NT < nchunk) {
#pragma unroll
          for (int m = 0; m < M; ++m) {
            float f[8];
            unpack8(xr[j][m], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) ss[m] += f[e] * f[e];
          }
        }
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const float sm = wave_sum(ss[m]);
        if ((tid & 63) == 0) red[m][tid / 64] = sm;
      }
      __syncthreads();
      float inv[M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) t += red[m][w];
        inv[m] = rsqrtf(t / K + eps);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = tid + j * NT;
        if (c < nchunk) {
          float g[8];
          unpack8(gr[j], g);
#pragma unroll
          for (int m = 0; m < M; ++m) {
            float f[8];
            unpack8(xr[j][m], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] = f[e] * inv[m] * g[e];
            reinterpret_cast<u32x4*>(xs + m * K)[c] = pack8(f);
          }
        }
      }
    } else {  // long rows: two passes over x (L2-resident)
      for (int c = tid; c < nchunk; c += NT) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          float f[8];
          unpack8(reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(m) * x_stride)[c], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) ss[m] += f[j] * f[j];
        }
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const float sm = wave_sum(ss[m]);
        if ((tid & 63) == 0) red[m][tid / 64] = sm;
      }
      __syncthreads();
      float inv[M];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) t += red[m][w];
        inv[m] = rsqrtf(t / K + eps);
      }
      for (int c = tid; c < nchunk; c += NT) {
        float g[8];
        unpack8(reinterpret_cast<const u32x4*>(norm_w)[c], g);
#pragma unroll
        for (int m = 0; m < M; ++m) {
          float f[8];
          unpack8(reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(m) * x_stride)[c], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] * inv[m] * g[j];
          reinterpret_cast<u32x4*>(xs + m * K)[c] = pack8(f);
        }
      }
    }
  } else if (x_fast) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = tid + j * NT;
      if (c < nchunk) {
#pragma unroll
        for (int m = 0; m < M; ++m) reinterpret_cast<u32x4*>(xs + m * K)[c] = xr[j][m];
      }
    }
  } else {
    for (int c = tid; c < nchunk; c += NT) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        reinterpret_cast<u32x4*>(xs + m * K)[c] =
            reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(m) * x_stride)[c];
    }
  }
  __syncthreads();
  if (!PAIR_LDS && EPI != EPI_AR && row0 >= N) return;  // PAIR_LDS / EPI_AR: every wave reaches the barriers
  if constexpr (ROPE_PRE) {
    const int w_u = __builtin_amdgcn_readfirstlane(wave);
    const int r_u = (bx * WAVES + w_u) * RPW;
    const int D = rope.D, half = D / 2;
    const bool qk = r_u / D < rope.nh + rope.nkv;
    const int i = (r_u % D) / 2;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      pre_c[m] = 1.f;
      pre_s[m] = 0.f;
      if (qk) {
        const int64_t t = static_cast<int64_t>(pre_pos[m]) * half + i;
        pre_c[m] = ld_scalar(rope.cos_t + t);
        pre_s[m] = ld_scalar(rope.sin_t + t);
      }
    }
  }

  // ---- main loop: RPW weight rows per wave, one UNROLL-batch ahead ----
  float acc[RPW][M];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;

  const u32x4* xv = reinterpret_cast<const u32x4*>(xs);
  // MASKED only for the last batch when K is not a multiple of 64 * 8 * UNROLL elements: the
  // full batches run branch-free (no per-chunk exec-mask juggling between the waits)
  auto consume = [&](const u32x4 (&wv)[RPW][UNROLL], int cbase, auto masked) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int c = cbase + u * kWave;
      if (!decltype(masked)::value || c < nchunk) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const u32x4 xx = xv[m * nchunk + c];
#pragma unroll
          for (int r = 0; r < RPW; ++r)
            if (!COMBINE || r == m) acc[r][m] = dot8_bf16(wv[r][u], xx, acc[r][m]);
        }
      }
    }
  };
  using Full = std::integral_constant<bool, false>;
  using Masked = std::integral_constant<bool, true>;
  const int full = nchunk / STEP;  // batches in which every lane's chunks are all in range
  int c0 = lane;
  for (int it = 0; it + 1 < iters; ++it, c0 += STEP) {  // it < iters - 1 <= full
    u32x4 nxt[RPW][UNROLL];
    issue(nxt, c0 + STEP);
    consume(cur, c0, Full{});
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int r = 0; r < RPW; ++r) cur[r][u] = nxt[r][u];
  }
  if (full == iters) {
    consume(cur, c0, Full{});
  } else {
    consume(cur, c0, Masked{});
  }

#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (!COMBINE || r == m) acc[r][m] = wave_sum(acc[r][m]);

  // ---- epilogue ----
  // paired epilogues (SiLU, RoPE) combine rows (2j, 2j + 1): the same wave holds both when
  // RPW >= 2; with RPW == 1 they sit in waves (w, w + 1) and meet through LDS (PAIR_LDS).
  // RoPE operands of (row n, token m): cos/sin of the pair's frequency and the KV slot
  auto rope_ops = [&](int n, int m, float& c, float& sn, int& slot) {
    const int D = rope.D, half = D / 2;
    slot = rope.slots[m];
    c = 1.f;
    sn = 0.f;
    if (n / D < rope.nh + rope.nkv) {
      const int i = (n % D) / 2;
      const int pos = rope.positions[m];
      c = rope.cos_t[static_cast<int64_t>(pos) * half + i];
      sn = rope.sin_t[static_cast<int64_t>(pos) * half + i];
    }
  };
  auto pair_epi = [&](int n, int m, float v, float x2, float c, float sn, int slot) {
    if constexpr (EPI == EPI_SILU) {  // rows (2j, 2j+1) = (gate, up) -> output column n/2
      reinterpret_cast<bf16_t*>(out)[static_cast<int64_t>(m) * out_stride + n / 2] = f32_to_bf16(silu(v) * x2);
    } else if constexpr (EPI == EPI_ROPE) {  // rows (2j, 2j+1) of a Q/K head = dims (i, i + D/2)
      const int D = rope.D, half = D / 2;
      const int head = n / D;
      const int64_t page = slot >= 0 ? slot / rope.bs : 0;
      const int off = slot >= 0 ? slot % rope.bs : 0;
      if (head < rope.nh + rope.nkv) {
        const int i = (n % D) / 2;
        const float o1 = v * c - x2 * sn, o2 = x2 * c + v * sn;
        if (head < rope.nh) {
          bf16_t* qo = rope.q_out + static_cast<int64_t>(m) * rope.q_stride + head * D;
          qo[i] = f32_to_bf16(o1);
          qo[i + half] = f32_to_bf16(o2);
        } else if (slot >= 0) {
          bf16_t* ko = rope.k_cache + ((page * rope.nkv + (head - rope.nh)) * rope.bs + off) * D;
          ko[i] = f32_to_bf16(o1);
          ko[i + half] = f32_to_bf16(o2);
        }
        if (rope.granules != nullptr)  // one row (M == 1): rows are heads x D
          __hip_atomic_store(rope.granules + head * half + i,
                             static_cast<uint64_t>(pack_bf16x2(o1, o2)) | (static_cast<uint64_t>(rope.gtag) << 32),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {  // V rows keep canonical order
        const int vh = head - rope.nh - rope.nkv, d = n % D;
        if (slot >= 0) {
          bf16_t* vv = rope.v_cache + ((page * rope.nkv + vh) * rope.bs + off) * D;
          vv[d] = f32_to_bf16(v);
          vv[d + 1] = f32_to_bf16(x2);
        }
        if (rope.granules != nullptr)
          __hip_atomic_store(rope.granules + head * half + d / 2,
                             static_cast<uint64_t>(pack_bf16x2(v, x2)) | (static_cast<uint64_t>(rope.gtag) << 32),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  };
  if constexpr (PAIR_LDS) {
    float* pairx = reinterpret_cast<float*>(smem + static_cast<size_t>(M) * K * sizeof(bf16_t)) + M * WAVES;
    if ((wave & 1) && lane < M) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (lane == m) pairx[(wave >> 1) * M + m] = acc[0][m];
    }
    __syncthreads();
    if (!(wave & 1)) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (lane == m && row0 < N) {
          if constexpr (EPI == EPI_ROPE) {
            pair_epi(row0, m, acc[0][m], pairx[(wave >> 1) * M + m], pre_c[m], pre_s[m], pre_slot[m]);
          } else {
            pair_epi(row0, m, acc[0][m], pairx[(wave >> 1) * M + m], 1.f, 0.f, -1);
          }
        }
    }
    return;
  }
  if constexpr (EPI == EPI_AR) {
    constexpr int HP = WAVES / 2, NG = M * HP;  // row pairs per block; granules per rank
    // the block's values (rank 0: + residual), [M][WAVES] f32 after the norm-partials area
    float* rowv = reinterpret_cast<float*>(smem + static_cast<size_t>(M) * K * sizeof(bf16_t)) + M * WAVES;
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (lane == m) rowv[m * WAVES + wave] = acc[0][m] + ar_resid[m];
    __syncthreads();
    if (wave != 0) return;
    const uint32_t epoch = __shfl(ar_epoch, 0, 64);
    const int rb = bx * WAVES;
    const int pairs = max(0, min(WAVES, N - rb)) / 2;  // N even: a pair is whole or absent
    const long gbase = static_cast<long>(bx) * kArGranulesPerBlock;
    auto payload = [&](int gi) {  // my bf16 pair of granule gi (rows 2j, 2j + 1 of token m)
      const int m = gi / HP, j = gi % HP;
      return pack_bf16x2(rowv[m * WAVES + 2 * j], rowv[m * WAVES + 2 * j + 1]);
    };
    for (int idx = lane; idx < ar.world * NG; idx += kWave) {  // push: (peer, granule)
      const int p = idx / NG, gi = idx % NG;
      if (p != ar.rank && gi % HP < pairs)
        car_put(ar.P.base[p] + car_granule_off(epoch, ar.cap, ar.rank, gbase + gi), payload(gi), epoch);
    }
    if (lane < NG && lane % HP < pairs) {  // collect my granule of every peer, sum in rank order
      const long g[1] = {gbase + lane};
      uint32_t in[kMaxRanks][1];
      car_collect<1>(ar.P, ar.rank, ar.world, ar.cap, epoch, g, in);
      in[ar.rank][0] = payload(lane);
      float lo = 0.f, hi = 0.f;
#pragma unroll
      for (int r = 0; r < kMaxRanks; ++r) {
        if (r < ar.world) {
          lo += bf16_lo(in[r][0]);
          hi += bf16_hi(in[r][0]);
        }
      }
      const int m = lane / HP, j = lane % HP;
      *reinterpret_cast<uint32_t*>(reinterpret_cast<bf16_t*>(out) + static_cast<int64_t>(m) * out_stride + rb + 2 * j) =
          pack_bf16x2(lo, hi);
    }
    if (lane == 0)
      __hip_atomic_store(car_ctr(ar.P.base[ar.rank]) + bx, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if constexpr (COMBINE) {
    if (lane == 0 && row0 < N) {
      const float* wt = rope.cos_t + by * RPW;  // router weights [T, k]
      bf16_t* h = reinterpret_cast<bf16_t*>(out) + row0;
      float v = bf16_to_f32(*h);
#pragma unroll
      for (int r = 0; r < RPW; ++r) v += wt[r] * acc[r][r];
      *h = f32_to_bf16(v);
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int n = row0 + r;
      if (lane != r * M + m || n >= N) continue;
      const float v = acc[r][m];
      if constexpr (EPI == EPI_BF16) {
        reinterpret_cast<bf16_t*>(out)[static_cast<int64_t>(m) * out_stride + n] = f32_to_bf16(v);
      } else if constexpr (EPI == EPI_F32) {
        reinterpret_cast<float*>(out)[static_cast<int64_t>(m) * out_stride + n] = v;
      } else if constexpr (EPI == EPI_RESADD) {
        bf16_t* h = reinterpret_cast<bf16_t*>(out) + static_cast<int64_t>(m) * out_stride + n;
        *h = f32_to_bf16(bf16_to_f32(*h) + v);
      } else {
        if constexpr (RPW >= 2) {
          if ((r & 1) == 0) {
            float c = 1.f, sn = 0.f;
            int slot = -1;
            if constexpr (EPI == EPI_ROPE && RPW == 2) {  // r == 0: the wave's pair, preloaded
              c = pre_c[m];
              sn = pre_s[m];
              slot = pre_slot[m];
            } else if constexpr (EPI == EPI_ROPE) {
              rope_ops(n, m, c, sn, slot);
            }
            pair_epi(n, m, v, acc[r + 1][m], c, sn, slot);
          }
        }
      }
    }
  }
}

template <int M, int NT, int RPW, int UNROLL, int PRO, int EPI, bool EXPERT = false>
__global__ __launch_bounds__(NT) void gemv_kernel(const bf16_t* __restrict__ x, int x_stride,
                                                  const bf16_t* __restrict__ norm_w, float eps,
                                                  const bf16_t* __restrict__ W, void* __restrict__ out,
                                                  int out_stride, int N, int K, const int32_t* __restrict__ expert_ids,
                                                  int x_div, RopeEpi rope, CarArgs ar) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  gemv_block<M, NT, RPW, UNROLL, PRO, EPI, EXPERT>(blockIdx.x, blockIdx.y, smem, x, x_stride, norm_w, eps, W, out,
                                                   out_stride, N, K, expert_ids, x_div, rope, ar);
}

}  // namespace llmc
