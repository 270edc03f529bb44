// K4: paged flash-attention PREFILL (chunked, causal, GQA) on MFMA 32x32x16 bf16.
//
// One workgroup = 4 waves = 4 "row tiles" of 32 query rows that share a kv head (with GQA
// group G = 4 the 4 waves are the 4 query heads of one kv head at the same 32 positions, so
// every K/V tile staged in LDS feeds 4 heads). Per 64-key tile (= one 64-token KV page):
//
//   S^T[key][q] = K . Q^T      A = K rows from LDS (ds_read_b128, XOR-swizzled chunks:
//                              chunk ^ (row & 15) -> conflict-free, cdna_hip_programming T2)
//                              B = Q^T fragments held in VGPRs for the whole kernel
//   online softmax             the accumulator puts ONE query per lane (col = lane & 31) with 32
//                              of the 64 keys in registers; the other 32 are in lane ^ 32
//                              -> row max/sum = in-register reduce + one xor-32 exchange
//   O^T[d][q] += V^T . P^T     B = P straight from the S^T accumulator (cvt to bf16, the
//                              permuted-k trick of guide §3 "accumulator tile as the next
//                              MFMA's operand"); A = V^T via ds_read_b64_tr_b16 (T10) from a
//                              row-major V tile swizzled chunk ^ ((row & 3) << 2): conflict-free.
//                              O^T keeps query on the lane, so the online-softmax rescale uses
//                              the lane's own alpha (no cross-lane broadcast).
//
// K/V tiles are register-staged one tile ahead (issue global loads for t+1 before computing t,
// write LDS after: T14 async-STAGE split) into a 2-deep LDS ring. Keys are looked up through
// the block table per row, so any page size works (64 is the engine default).
// Numerics: S in f32, exp2 with log2(e) folded into the scale, P rounded to bf16 for PV, O in f32.
#include <stdlib.h>

#include "common.h"

namespace llmc {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kKT = 64;        // keys per tile
constexpr int kRowBytes = 256; // LDS row pitch (128 bf16), D <= 128
constexpr int kTileBytes = kKT * kRowBytes;  // 16 KB
constexpr int kPrefillLookahead = 2;          // K/V tiles requested ahead of the one computing

__device__ __forceinline__ int k_swz(int row, int ch) { return row * kRowBytes + ((ch ^ (row & 15)) << 4); }
__device__ __forceinline__ int v_swz(int row, int ch) { return row * kRowBytes + ((ch ^ ((row & 3) << 2)) << 4); }

template <int D, int WPB, int LA>
__global__ __launch_bounds__(WPB * 64) void attn_prefill_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int32_t* __restrict__ block_tables, int bt_stride, const int32_t* __restrict__ q_start,
    const int32_t* __restrict__ q_lens, const int32_t* __restrict__ ctx_lens, bf16_t* __restrict__ out,
    int out_stride, int nh, int nkv, int bs, float scale_log2) {
  constexpr int CH = D / 8;            // 16-B chunks per row
  constexpr int NT = WPB * 64;
  constexpr int NL = (kKT * CH + NT - 1) / NT;  // staging chunks per thread per tensor
  constexpr bool NL_EXACT = (kKT * CH) % NT == 0;
  constexpr int KS = D / 16;           // k-steps for Q.K
  constexpr int DT = D / 32;           // 32-wide d tiles of O

  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * kTileBytes];  // [buf][K|V]

  const int G = nh / nkv;
  // grid.x = row-tile groups x kv heads, kv head fastest: the dispatch order is longest-first over
  // the whole grid (latest query rows = most causal key tiles), not per kv head, so the last
  // rounds of a multi-round grid hold the shortest blocks of every head (no long-job tail)
  const int b = blockIdx.z, kvh = blockIdx.x % nkv, grp = blockIdx.x / nkv;
  const int ngrp = gridDim.x / nkv;
  const int qlen = q_lens[b];
  if (qlen <= 0) return;
  const int ctx = ctx_lens[b];
  const int q0 = q_start[b];
  const int npb = (qlen + 31) / 32;
  const int nrt = G * npb;
  const int rt_base = (ngrp - 1 - grp) * WPB;
  if (rt_base >= nrt) return;  // block-uniform

  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  const int r = lane & 31, hh = lane >> 5;
  const int rt = rt_base + wave;
  const bool wvalid = rt < nrt;
  const int g = wvalid ? rt % G : 0;
  const int pb = wvalid ? rt / G : 0;
  const int h = kvh * G + g;
  const int first_pos = ctx - qlen;
  const int row_i = pb * 32 + r;                  // query row within the sequence chunk
  const int qi = min(row_i, qlen - 1);
  const int qpos = first_pos + qi;                 // absolute position (causal limit)
  const int last_rt = min(rt_base + WPB - 1, nrt - 1);
  const int pb_last = last_rt / G;
  const int kend = min(ctx, first_pos + min(pb_last * 32 + 31, qlen - 1) + 1);
  const int ntiles = (kend + kKT - 1) / kKT;
  const int wave_kend = wvalid ? first_pos + min(pb * 32 + 31, qlen - 1) + 1 : 0;
  const int wave_qpos0 = first_pos + pb * 32;  // smallest query position of this wave

  // Q^T fragments (B operand): lane (r, hh) holds Q[qi][h*D + ks*16 + 8hh .. +8]
  bf16x8 qf[KS];
  {
    const bf16_t* qrow = q + static_cast<int64_t>(q0 + qi) * q_stride + h * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + ks * 16 + 8 * hh);
  }

  f32x16 acc_o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc_o[dt][i] = 0.f;
  float m_run = -1e30f, l_run = 0.f;

  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int64_t head_stride = static_cast<int64_t>(bs) * D;

  // LA register staging sets: tile t + LA is requested while tile t computes, so a tile's global
  // loads have LA - 1 whole compute steps (plus one) to land before its commit to LDS (one tile
  // of lookahead left every tile waiting on HBM latency at 2k tokens: ~3 us per 64-key tile)
  u32x4 stk[LA][NL], stv[LA][NL];
  auto issue = [&](int t, int set) {
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int idx = tid + u * NT;
      if (!NL_EXACT && idx >= kKT * CH) continue;
      const int row = idx / CH, ch = idx % CH;
      int key = t * kKT + row;
      key = min(key, ctx - 1);
      const int64_t page = bt[key / bs];
      const int64_t off = (page * nkv + kvh) * head_stride + static_cast<int64_t>(key % bs) * D + ch * 8;
      stk[set][u] = *reinterpret_cast<const u32x4*>(k_cache + off);
      stv[set][u] = *reinterpret_cast<const u32x4*>(v_cache + off);
    }
  };
  auto commit = [&](int buf, int set) {
    char* kb = smem + buf * 2 * kTileBytes;
    char* vb = kb + kTileBytes;
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int idx = tid + u * NT;
      if (!NL_EXACT && idx >= kKT * CH) continue;
      const int row = idx / CH, ch = idx % CH;
      *reinterpret_cast<u32x4*>(kb + k_swz(row, ch)) = stk[set][u];
      *reinterpret_cast<u32x4*>(vb + v_swz(row, ch)) = stv[set][u];
    }
  };

  issue(0, 0);
#pragma unroll
  for (int j = 1; j < LA; ++j)
    if (j < ntiles) issue(j, j);
  commit(0, 0);
  __syncthreads();

  // unrolled by LA so that every staging-set index is a compile-time constant (a runtime index into
  // a register array would go through scratch)
  for (int t0 = 0; t0 < ntiles; t0 += LA) {
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    const int t = t0 + j;
    if (t >= ntiles) break;
    const int buf = t & 1;
    // the set tile t was staged in (j) is free again (committed): tile t + LA goes into it
    if (t + LA < ntiles) issue(t + LA, j);
    const int kt = t * kKT;
    if (wvalid && kt < wave_kend) {
      const char* kb = smem + buf * 2 * kTileBytes;
      const char* vb = kb + kTileBytes;
      // ---- S^T = K . Q^T for two 32-key halves ----
      f32x16 s[2];
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kb2][i] = 0.f;
        const int row = kb2 * 32 + r;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(kb + k_swz(row, 2 * ks + hh));
          s[kb2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[ks], s[kb2], 0, 0, 0);
        }
      }
      // ---- online softmax (lane owns query qpos; keys in registers) ----
      // Causal masking only on tiles that reach past the wave's first query position (the
      // diagonal band); the others are plain scale + max. Raw v_exp_f32 (inputs are <= 0 after
      // the max subtraction, so no range reduction is needed).
      const bool diag = kt + kKT - 1 > wave_qpos0;  // wave-uniform
      float mx = -1e30f;
      if (diag) {
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = kt + kb2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
            s[kb2][i] = key <= qpos ? s[kb2][i] * scale_log2 : -1e30f;
            mx = fmaxf(mx, s[kb2][i]);
          }
      } else {
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            s[kb2][i] *= scale_log2;
            mx = fmaxf(mx, s[kb2][i]);
          }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run, mx);
      const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
      float rs = 0.f;
      if (diag) {
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float sv = s[kb2][i];
            const float p = sv <= -1e29f ? 0.f : __builtin_amdgcn_exp2f(sv - m_new);
            s[kb2][i] = p;
            rs += p;
          }
      } else {
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float p = __builtin_amdgcn_exp2f(s[kb2][i] - m_new);
            s[kb2][i] = p;
            rs += p;
          }
      }
      rs += __shfl_xor(rs, 32, 64);
      l_run = l_run * alpha + rs;
      m_run = m_new;
      if (__any(alpha != 1.f)) {  // the running max moved for some query of the wave
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc_o[dt][i] *= alpha;
      }
      // ---- P fragments: k-step k4 = kb2*2 + sidx uses registers 8*sidx .. +7 of s[kb2] ----
      bf16x8 pf[4];
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
        for (int sidx = 0; sidx < 2; ++sidx) {
          u32x4 pk;
#pragma unroll
          for (int j = 0; j < 4; ++j) pk[j] = pack_bf16x2(s[kb2][8 * sidx + 2 * j], s[kb2][8 * sidx + 2 * j + 1]);
          pf[kb2 * 2 + sidx] = __builtin_bit_cast(bf16x8, pk);
        }
      // ---- O^T += V^T . P^T ----
      const int g1 = (lane >> 4) & 1, qq = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int ch = 4 * dt + 2 * g1 + (p4 >> 1);
        const int sub = (p4 & 1) * 8;
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const int row0 = k4 * 16 + 4 * hh + qq;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + v_swz(row0, ch) + sub));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(vb + v_swz(row0 + 8, ch) + sub));
          bf16x8 a;
          a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
          a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
          acc_o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pf[k4], acc_o[dt], 0, 0, 0);
        }
      }
    }
    if (t + 1 < ntiles) commit(buf ^ 1, (j + 1) % LA);
    __syncthreads();
  }
  }

  if (!wvalid || row_i >= qlen) return;
  const float inv_l = l_run > 0.f ? 1.f / l_run : 0.f;
  bf16_t* orow = out + static_cast<int64_t>(q0 + row_i) * out_stride + h * D;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      const int d = dt * 32 + 8 * i4 + 4 * hh;
      u32x2 v;
      v[0] = pack_bf16x2(acc_o[dt][4 * i4 + 0] * inv_l, acc_o[dt][4 * i4 + 1] * inv_l);
      v[1] = pack_bf16x2(acc_o[dt][4 * i4 + 2] * inv_l, acc_o[dt][4 * i4 + 3] * inv_l);
      *reinterpret_cast<u32x2*>(orow + d) = v;
    }
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_attn_prefill(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                 const void* block_tables, int bt_stride, const void* q_start, const void* q_lens,
                                 const void* ctx_lens, void* out, int out_stride, int B, int max_qlen, int nh, int nkv,
                                 int D, int bs, float scale, hipStream_t s) {
  if (nh % nkv != 0) return -1;
  const int G = nh / nkv;
  const int npb = (max_qlen + 31) / 32;
  constexpr int WPB = 8;  // 8 waves = 2 row tiles x 4 heads share every staged K/V tile
  dim3 grid((G * npb + WPB - 1) / WPB * nkv, 1, B);
  const float sl2 = scale * 1.4426950408889634f;
  static const int la = [] {
    const char* e = getenv("LLMC_PREFILL_LOOKAHEAD");  // A/B runs: K/V tiles requested ahead
    return e ? atoi(e) : kPrefillLookahead;
  }();
#define LLMC_PF(DD, L)                                                                                           \
  attn_prefill_kernel<DD, WPB, L><<<grid, WPB * 64, 0, s>>>((const bf16_t*)q, q_stride, (const bf16_t*)k_cache, \
                                               (const bf16_t*)v_cache, (const int32_t*)block_tables, bt_stride,   \
                                               (const int32_t*)q_start, (const int32_t*)q_lens,                  \
                                               (const int32_t*)ctx_lens, (bf16_t*)out, out_stride, nh, nkv, bs, sl2)
#define LLMC_PF_D(DD)                \
  do {                               \
    if (la >= 3) LLMC_PF(DD, 3);     \
    else if (la == 2) LLMC_PF(DD, 2); \
    else LLMC_PF(DD, 1);             \
  } while (0)
  switch (D) {
    case 64: LLMC_PF_D(64); break;
    case 96: LLMC_PF_D(96); break;
    case 128: LLMC_PF_D(128); break;
    default: return -2;
  }
#undef LLMC_PF_D
#undef LLMC_PF
  return static_cast<int>(hipGetLastError());
}
