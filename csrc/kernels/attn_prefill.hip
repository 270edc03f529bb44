// K4: paged flash-attention PREFILL (chunked, causal, GQA) on MFMA 32x32x16 bf16.
//
// A wave owns a "row tile" of 32 query rows of one head; the waves of a workgroup share a kv head,
// so every K/V tile staged in LDS feeds all of them (with G = 4 query heads per kv head, an 8-wave
// block = 2 row positions x 4 heads). Per 64-key tile (= one 64-token KV page):
//
//   S^T[key][q] = K . Q^T      A = K rows from LDS (ds_read_b128, XOR-swizzled chunks:
//                              chunk ^ (row & 15) -> conflict-free, cdna_hip_programming T2)
//                              B = Q^T fragments held in VGPRs for the whole kernel
//   online softmax             the accumulator puts ONE query per lane (col = lane & 31) with 32
//                              of the 64 keys in registers; the other 32 are in lane ^ 32
//                              -> row max/sum = in-register reduce + one xor-32 exchange; one fma +
//                              exp per score, the running max moved only past a slack (kSlack)
//   O^T[d][q] += V^T . P^T     B = P straight from the S^T accumulator (v_cvt_pk_bf16_f32, the
//                              permuted-k trick of guide §3 "accumulator tile as the next
//                              MFMA's operand"); A = V^T via ds_read_b64_tr_b16 (T10) from a
//                              row-major V tile swizzled chunk ^ ((row & 3) << 2): conflict-free.
//                              O^T keeps query on the lane, so the online-softmax rescale uses
//                              the lane's own alpha (no cross-lane broadcast).
//
// K/V staging: LDS-DMA (buffer_load ... lds, the swizzle inverted on the source side) into a 4-slot
// ring for D = 128 on 64-key pages; otherwise register-staged one or two tiles ahead into a 2-deep
// LDS ring. Numerics: S in f32, exp2 with log2(e) folded into the scale, P rounded to bf16 for PV,
// O in f32.
//
// Block forms (llmc_attn_prefill_form): 8 waves; 8 waves with paired late / early row tiles; 4 waves
// (two blocks per CU); key halves (two wave halves over the two halves of the key tiles, merged
// through LDS). The grid is ordered longest-first over all kv heads.
//
// KV split (llmc_attn_prefill_plan): when the grid cannot keep the chip busy to the end (a TP=8
// rank's single kv head = 32-128 blocks), the long row-tile groups' key ranges are cut into 2-4
// ranges on their own blocks; each writes (unnormalised O, m, l) in f32 and the last to finish merges
// them in split order (deterministic).
#include <stdlib.h>

#include <algorithm>
#include <queue>
#include <vector>

#include "common.h"

namespace llmc {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;

constexpr int kKT = 64;        // keys per tile
constexpr int kRowBytes = 256; // LDS row pitch (128 bf16), D <= 128
constexpr int kTileBytes = kKT * kRowBytes;  // 16 KB
constexpr int kPrefillLookahead = 2;          // K/V tiles requested ahead of the one computing
constexpr int kDmaSlots = 4;                   // LDS-DMA staging: tiles resident (3 in flight)
constexpr int kMaxSplit = 4;                   // KV-split ways (llmc_attn_prefill_plan)
constexpr float kSlack = 8.f;                  // deferred running-max update threshold (log2 units)

// two floats -> packed bf16x2 (RNE) in one instruction (no builtin for the two-operand form)
__device__ __forceinline__ uint32_t cvt_pk_bf16(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

__device__ __forceinline__ int k_swz(int row, int ch) { return row * kRowBytes + ((ch ^ (row & 15)) << 4); }
__device__ __forceinline__ int v_swz(int row, int ch) { return row * kRowBytes + ((ch ^ ((row & 3) << 2)) << 4); }

template <int D, int WPB, int LA, bool P64, bool DMA = false>
__global__ __launch_bounds__(WPB * 64, 8 / WPB) void attn_prefill_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int32_t* __restrict__ block_tables, int bt_stride, const int32_t* __restrict__ q_start,
    const int32_t* __restrict__ q_lens, const int32_t* __restrict__ ctx_lens, bf16_t* __restrict__ out,
    int out_stride, int nh, int nkv, int bs, float scale_log2, int ksplit, int kmin, float* __restrict__ part,
    int* __restrict__ counters, int T_all, int mode) {
  constexpr int CH = D / 8;            // 16-B chunks per row
  constexpr int NT = WPB * 64;
  constexpr int NL = (kKT * CH + NT - 1) / NT;  // staging chunks per thread per tensor
  constexpr bool NL_EXACT = (kKT * CH) % NT == 0;
  constexpr int KS = D / 16;           // k-steps for Q.K
  constexpr int DT = D / 32;           // 32-wide d tiles of O

  static_assert(!DMA || (P64 && D == 128 && WPB == 8), "LDS-DMA staging: 64-key pages, D = 128, 8 waves");
  // [slot][K|V], then the split hand-off's is_last word. ONE LDS object: with a second __shared__
  // variable the LDS lowering tags every access with alias scopes, and hipcc's waitcnt pass then
  // makes each tile's first LDS read wait for every LDS-DMA in flight (vmcnt(0): no lookahead)
  constexpr int kSmemMain = (DMA ? kDmaSlots : 2) * 2 * kTileBytes;
  __shared__ __attribute__((aligned(16))) char smem[kSmemMain + 16];

  const int G = nh / nkv;
  // grid.x = row-tile groups x kv heads, kv head fastest: the dispatch order is longest-first over
  // the whole grid (latest query rows = most causal key tiles), not per kv head, so the last
  // rounds of a multi-round grid hold the shortest blocks of every head (no long-job tail)
  // with a KV split (ksplit > 1: few blocks for the chip) grid.x = groups x splits x kv heads, the
  // split index between the two: every split of a group keeps the group's longest-first position
  const int b = blockIdx.z, kvh = blockIdx.x % nkv, sp = (blockIdx.x / nkv) % ksplit, grp = blockIdx.x / nkv / ksplit;
  const int ngrp = gridDim.x / nkv / ksplit;
  const int qlen = q_lens[b];
  if (qlen <= 0) return;
  const int ctx = ctx_lens[b];
  const int q0 = q_start[b];
  const int npb = (qlen + 31) / 32;
  const int nrt = G * npb;
  // mode: 0 = WPB row tiles per block, 1 = paired late / early row tiles, 2 = key halves (DMA
  // staging only): WPB / 2 row tiles, waves [0, WPB / 2) on the first half of their key tiles and
  // waves [WPB / 2, WPB) on the second half, merged through LDS at the end
  const bool pair = mode == 1, halves = DMA && mode == 2;
  const int rt_base = (ngrp - 1 - grp) * (halves ? WPB / 2 : WPB);
  if (!pair && rt_base >= nrt) return;  // block-uniform

  // wave index through readfirstlane: everything derived from it (row tile, head, descriptors)
  // is then known wave-uniform (a divergent-looking descriptor costs a waterfall loop per access)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  const int r = lane & 31, hh = lane >> 5;
  // pair (unsplit grids, WPB / G = R >= 2 even): block grp (0 = dispatched first) takes the R / 2
  // LATEST 32-row tiles still free (npb - 1 - grp R/2 - j) for waves [0, WPB / 2) and the R / 2
  // EARLIEST (grp R/2 + j) for the others. An early tile's causal key range is a prefix of the late
  // one's, so the block stages the late tiles' keys once for both, and every SIMD holds one late
  // and one early wave: ~npb + 1 tile steps per SIMD in every block instead of 2 x the block's
  // latest tile, whose longest block set the critical path of one-round grids.
  const int khalf = halves ? wave / (WPB / 2) : 0;  // halves: which half of the key tiles
  int rt = rt_base + (halves ? wave % (WPB / 2) : wave);
  bool wvalid = rt < nrt;
  if (pair) {
    const int R = WPB / G, half = R / 2, slot = wave / G, top = ngrp * half;
    const int pbp = slot < half ? npb - 1 - (grp * half + slot) : grp * half + (slot - half);
    wvalid = pbp >= 0 && (slot < half || pbp < npb - top);
    rt = pbp * G + wave % G;
  }
  const int g = wvalid ? rt % G : 0;
  const int pb = wvalid ? rt / G : 0;
  const int h = kvh * G + g;
  const int first_pos = ctx - qlen;
  const int row_i = pb * 32 + r;                  // query row within the sequence chunk
  const int qi = min(row_i, qlen - 1);
  const int qpos = first_pos + qi;                 // absolute position (causal limit)
  const int last_rt = min(rt_base + (halves ? WPB / 2 : WPB) - 1, nrt - 1);
  const int pb_last = pair ? max(npb - 1 - grp * (WPB / G / 2), 0) : last_rt / G;
  const int kend = min(ctx, first_pos + min(pb_last * 32 + 31, qlen - 1) + 1);
  const int ntiles_all = (kend + kKT - 1) / kKT;
  // only groups with >= 2 kmin key tiles split (a causal grid's short groups run whole); the
  // surplus split blocks of the others exit here (block-uniform, before any barrier)
  const int nsplit = ksplit > 1 ? min(ksplit, max(1, ntiles_all / kmin)) : 1;
  if (sp >= nsplit) return;
  // this block's key tiles: split sp of the group's [0, ntiles_all) (all of it without a split)
  const int t_lo = sp * ntiles_all / nsplit, ntiles = (sp + 1) * ntiles_all / nsplit;
  const int wave_kend = wvalid ? first_pos + min(pb * 32 + 31, qlen - 1) + 1 : 0;
  const int wave_qpos0 = first_pos + pb * 32;  // smallest query position of this wave

  // Q^T fragments (B operand): lane (r, hh) holds Q[qi][h*D + ks*16 + 8hh .. +8]
  bf16x8 qf[KS];
  {
    const bf16_t* qrow = q + static_cast<int64_t>(q0 + qi) * q_stride + h * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + ks * 16 + 8 * hh);
    // Consume the Q loads here, before the tile loop: left pending at the loop entry, hipcc's
    // waitcnt pass charged them to every iteration - a vmcnt(7..0) ladder across the QK^T MFMAs
    // that waited for the K/V tiles just requested, i.e. no lookahead at all.
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(qf[ks]));
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
  int voff[NL];  // P64: byte offset of this lane's 16-B chunk u within a page's [64][D] image
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    const int idx = tid + u * NT;
    voff[u] = (idx / CH) * D * 2 + (idx % CH) * 16;
  }
  auto issue = [&](int t, int set) {
    if constexpr (P64) {
      // 64-token pages = one page per key tile: the page number is ONE wave-uniform scalar load
      // (lgkm-counted: no vmcnt drain of the K/V loads in flight, as a per-lane lookup forced) and
      // K/V come by buffer loads off a per-tile descriptor with lane-constant offsets (no per-tile
      // address VALU; a reused address register also made hipcc wait for the loads it fed). Rows
      // past ctx - 1 of the last page lie beyond the descriptor's range and read as zeros.
      const int tu = __builtin_amdgcn_readfirstlane(t);
      const int64_t base = (static_cast<int64_t>(ld_scalar(bt + tu)) * nkv + kvh) * head_stride;
      const int bytes = min(kKT, ctx - tu * kKT) * D * 2;
      const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)(k_cache + base), 0, bytes, 0x00020000);
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)(v_cache + base), 0, bytes, 0x00020000);
#pragma unroll
      for (int u = 0; u < NL; ++u) {
        if (!NL_EXACT && tid + u * NT >= kKT * CH) continue;
        stk[set][u] = __builtin_amdgcn_raw_buffer_load_b128(rk, voff[u], 0, 0);
        stv[set][u] = __builtin_amdgcn_raw_buffer_load_b128(rv, voff[u], 0, 0);
      }
      return;
    }
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

  // one 64-key tile of every wave (kb / vb: the tile's K and V images in LDS)
  auto tile_compute = [&](int t, const char* kb, const char* vb) {
      const int kt = t * kKT;
      if (wvalid && kt < wave_kend) {
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
        // VALU diet (the loop is VALU-bound at 2 waves/SIMD, ~2x the MFMA cycles before it): the
        // max on raw scores (scale > 0), then ONE fma + exp per score; causal masking only on the
        // tiles that reach past the wave's first query position; the running max moves only when a
        // new score exceeds it by > kSlack (log2 units, so P <= 2^kSlack: exact in f32, same bf16
        // relative rounding), which leaves the O rescale out of almost every tile; P packed by
        // v_cvt_pk_bf16_f32 (two floats per instruction, RNE).
        const bool diag = kt + kKT - 1 > wave_qpos0;  // wave-uniform
        float mx = -1e30f;
        // diag: score (kb2, i) is key kt + 4 hh + kb2*32 + (i & 3) + 8 (i >> 2): visible iff that
        // compile-time offset <= lim (an inline-constant compare, no per-score add)
        const int lim = qpos - kt - 4 * hh;
        if (diag) {
  #pragma unroll
          for (int kb2 = 0; kb2 < 2; ++kb2)
  #pragma unroll
            for (int i = 0; i < 16; ++i)
              mx = fmaxf(mx, kb2 * 32 + (i & 3) + 8 * (i >> 2) <= lim ? s[kb2][i] : -1e30f);
        } else {
  #pragma unroll
          for (int kb2 = 0; kb2 < 2; ++kb2)
  #pragma unroll
            for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[kb2][i]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mx_s = mx * scale_log2;
        const float m_new = mx_s > m_run + kSlack ? mx_s : m_run;
        const float neg_m = -m_new;
        float rs2[4] = {0.f, 0.f, 0.f, 0.f};
        if (diag) {
  #pragma unroll
          for (int kb2 = 0; kb2 < 2; ++kb2)
  #pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float p = kb2 * 32 + (i & 3) + 8 * (i >> 2) <= lim
                                  ? __builtin_amdgcn_exp2f(fmaf(s[kb2][i], scale_log2, neg_m))
                                  : 0.f;
              s[kb2][i] = p;
              rs2[i & 3] += p;
            }
        } else {
  #pragma unroll
          for (int kb2 = 0; kb2 < 2; ++kb2)
  #pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float p = __builtin_amdgcn_exp2f(fmaf(s[kb2][i], scale_log2, neg_m));
              s[kb2][i] = p;
              rs2[i & 3] += p;
            }
        }
        float rs = (rs2[0] + rs2[1]) + (rs2[2] + rs2[3]);
        rs += __shfl_xor(rs, 32, 64);
        if (__any(m_new != m_run)) {  // the running max moved for some query of the wave
          const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
          l_run *= alpha;
  #pragma unroll
          for (int dt = 0; dt < DT; ++dt)
  #pragma unroll
            for (int i = 0; i < 16; ++i) acc_o[dt][i] *= alpha;
        }
        l_run += rs;
        m_run = m_new;
        // ---- P fragments: k-step k4 = kb2*2 + sidx uses registers 8*sidx .. +7 of s[kb2] ----
        bf16x8 pf[4];
  #pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
  #pragma unroll
          for (int sidx = 0; sidx < 2; ++sidx) {
            u32x4 pk;
  #pragma unroll
            for (int j = 0; j < 4; ++j) pk[j] = cvt_pk_bf16(s[kb2][8 * sidx + 2 * j], s[kb2][8 * sidx + 2 * j + 1]);
            pf[kb2 * 2 + sidx] = __builtin_bit_cast(bf16x8, pk);
          }
        // ---- O^T += V^T . P^T ----
        const int g1 = (lane >> 4) & 1, qq = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int ch = 4 * dt + 2 * g1 + (p4 >> 1);
          const int sub = (p4 & 1) * 8;
          if constexpr (DMA) {
            // the transposing reads as inline asm: the builtin's memory operand carries no type info, so
            // hipcc's waitcnt pass would make it wait for every LDS-DMA tile in flight (vmcnt(0)); asm
            // reads are invisible to that pass, hence the explicit wait, which takes the eight registers
            // through it so that no MFMA is scheduled above it
            s16x4 lo[4], hi[4];
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
              const int row0 = k4 * 16 + 4 * hh + qq;
              const uint32_t alo = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(vb + v_swz(row0, ch) + sub));
              const uint32_t ahi = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(vb + v_swz(row0 + 8, ch) + sub));
              asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo[k4]) : "v"(alo));
              asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi[k4]) : "v"(ahi));
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(lo[0]), "+v"(hi[0]), "+v"(lo[1]), "+v"(hi[1]), "+v"(lo[2]), "+v"(hi[2]), "+v"(lo[3]),
                           "+v"(hi[3]));
#pragma unroll
            for (int k4 = 0; k4 < 4; ++k4) {
              bf16x8 a;
              a[0] = lo[k4][0]; a[1] = lo[k4][1]; a[2] = lo[k4][2]; a[3] = lo[k4][3];
              a[4] = hi[k4][0]; a[5] = hi[k4][1]; a[6] = hi[k4][2]; a[7] = hi[k4][3];
              acc_o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pf[k4], acc_o[dt], 0, 0, 0);
            }
          } else {
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
      }
  };

  if constexpr (DMA) {
    // LDS-DMA staging (buffer_load ... lds): the tile's K / V land in LDS without a VGPR round trip,
    // so the lookahead is bounded by LDS (kDmaSlots tiles), not by staging registers. The LDS
    // image is lane-linear (instruction u of wave w writes bytes (u NT + 64 w + lane) x 16), so each
    // lane loads the source chunk that k_swz / v_swz put at its position: the XOR swizzle inverted
    // on the source side (rows of 256 B = 16 chunks). One counted wait + one barrier per tile.
    static_assert(NL == 2, "DMA staging: 2 instructions per lane per tensor");
    uint32_t dk[2], dv[2];  // fixed size: a template-dependent operand type drops the host stub
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int idx = u * NT + tid, row = idx >> 4, pc = idx & 15;
      dk[u] = static_cast<uint32_t>(row * kRowBytes + ((pc ^ (row & 15)) << 4));
      dv[u] = static_cast<uint32_t>(row * kRowBytes + ((pc ^ ((row & 3) << 2)) << 4));
    }
    auto issue_dma = [&](int t, int slot) {
      const int tu = __builtin_amdgcn_readfirstlane(t);
      const int64_t base = (static_cast<int64_t>(ld_scalar(bt + tu)) * nkv + kvh) * head_stride;
      const int bytes = min(kKT, ctx - tu * kKT) * D * 2;  // rows past ctx - 1 land as zeros
      const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)(k_cache + base), 0, bytes, 0x00020000);
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)(v_cache + base), 0, bytes, 0x00020000);
      char* sk = smem + slot * 2 * kTileBytes + wave * 1024;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, (__attribute__((address_space(3))) void*)(sk + u * 8192), 16, dk[u], 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (__attribute__((address_space(3))) void*)(sk + kTileBytes + u * 8192), 16,
                                                 dv[u], 0, 0, 0);
      }
    };
    if (halves) {
      // key halves: step s stages tile s of the first half (slot 2 (s & 1)) and tile t_mid + s of
      // the second (slot 2 (s & 1) + 1); step s + 1 is fetched into the slots of step s - 1 right
      // after the barrier that retires them, so it lands while step s computes
      const int t_mid = (ntiles + 1) / 2;  // unsplit: t_lo = 0
      auto issue_step = [&](int st) {
        issue_dma(st, 2 * (st & 1));
        if (t_mid + st < ntiles) issue_dma(t_mid + st, 2 * (st & 1) + 1);
      };
      issue_step(0);
      for (int st = 0; st < t_mid; ++st) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step st (the only one in flight)
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        if (st + 1 < t_mid) issue_step(st + 1);
        const int t = khalf ? t_mid + st : st;
        const char* kb = smem + (2 * (st & 1) + khalf) * 2 * kTileBytes;
        if (t < (khalf ? ntiles : t_mid)) tile_compute(t, kb, kb + kTileBytes);
      }
    } else {
#pragma unroll
    for (int j = 0; j < kDmaSlots - 1; ++j)
      if (t_lo + j < ntiles) issue_dma(t_lo + j, (t_lo + j) % kDmaSlots);
    for (int t = t_lo; t < ntiles; ++t) {
      // tile t landed (this wave's 4 loads of it; the next tiles' may stay in flight), then the
      // barrier: every wave's tile t landed and every wave finished reading slot (t - 1) % slots
      const int ahead = min(ntiles - 1 - t, kDmaSlots - 2);
      if (ahead >= 2) {
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else if (ahead == 1) {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // a bare s_barrier: __syncthreads()'s fence would drain every tile in flight (vmcnt(0))
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (t + kDmaSlots - 1 < ntiles) issue_dma(t + kDmaSlots - 1, (t + kDmaSlots - 1) % kDmaSlots);  // the slot just retired
      const char* kb = smem + (t % kDmaSlots) * 2 * kTileBytes;
      tile_compute(t, kb, kb + kTileBytes);
    }
    }
  } else {
  if (t_lo < ntiles) {
    issue(t_lo, 0);
#pragma unroll
    for (int j = 1; j < LA; ++j)
      if (t_lo + j < ntiles) issue(t_lo + j, j);
    commit(t_lo & 1, 0);
  }
  __syncthreads();

  // unrolled by LA so that every staging-set index is a compile-time constant (a runtime index into
  // a register array would go through scratch)
  for (int t0 = t_lo; t0 < ntiles; t0 += LA) {
#pragma unroll
  for (int j = 0; j < LA; ++j) {
    const int t = t0 + j;
    if (t >= ntiles) break;
    const int buf = t & 1;
    // the set tile t was staged in (j) is free again (committed): tile t + LA goes into it
    if (t + LA < ntiles) issue(t + LA, j);
    tile_compute(t, smem + buf * 2 * kTileBytes, smem + buf * 2 * kTileBytes + kTileBytes);
    if (t + 1 < ntiles) commit(buf ^ 1, (j + 1) % LA);
    __syncthreads();
  }
  }
  }

  if (halves) {
    // the second half's waves hand (O, m, l) to the first half's (same rows and head: wave - WPB / 2)
    // through LDS (the drained staging ring: [WPB / 2 waves][DT x 16 + 2][64 lanes] floats, lane
    // innermost so that every access is one float per lane, conflict-free)
    constexpr int NV = DT * 16 + 2;
    static_assert(!DMA || (WPB / 2) * NV * 64 * 4 <= kSmemMain, "halves hand-off fits the ring");
    float* xo = reinterpret_cast<float*>(smem) + (wave % (WPB / 2)) * NV * 64 + lane;
    __syncthreads();  // every wave past its last tile read
    if (khalf) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) xo[(dt * 16 + i) * 64] = acc_o[dt][i];
      xo[(DT * 16) * 64] = m_run;
      xo[(DT * 16 + 1) * 64] = l_run;
    }
    __syncthreads();
    if (khalf) return;  // after the block's last barrier
    const float m1 = xo[(DT * 16) * 64], l1 = xo[(DT * 16 + 1) * 64];
    const float M = fmaxf(m_run, m1);
    const float a0 = l_run > 0.f ? __builtin_amdgcn_exp2f(m_run - M) : 0.f;
    const float a1 = l1 > 0.f ? __builtin_amdgcn_exp2f(m1 - M) : 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc_o[dt][i] = fmaf(xo[(dt * 16 + i) * 64], a1, acc_o[dt][i] * a0);
    l_run = fmaf(l1, a1, l_run * a0);
  }
  const bool live = wvalid && row_i < qlen;
  if (nsplit > 1) {
    // split hand-off: every split writes (unnormalised O, m, l) in f32, the last to arrive merges
    // all of them in split order (its own from registers: the same values; every step an explicit
    // fmaf, so register and loaded terms round alike) -> deterministic, and one launch. Lanes
    // read back exactly the elements they wrote, so the layout is lane-private.
    const int64_t so = static_cast<int64_t>(T_all) * nh;  // (row, head) pairs per split slot
    // Inter-workgroup hand-off, MI355X_MICROARCH.md "Valid forms" table row 1: every byte stored
    // and loaded sc1 (16-/8-B buffer ops), every storing wave drains (vmcnt(0)) before the barrier,
    // ONE lane adds to the group's counter, the block whose add comes last merges after a barrier.
    // (A __threadfence pair here - L2 write-back + invalidate per block - cost 2.8x at 2k tokens.)
    // Per-wave resources: rows q0 + pb*32 .. +31 of head h; lane offset r * nh * {D, 2} floats.
    const int64_t wrow = static_cast<int64_t>(q0 + pb * 32) * nh + h;
    auto o_rsrc = [&](int slot) {
      return __builtin_amdgcn_make_buffer_rsrc(part + (slot * so + wrow) * D, 0, 32 * nh * D * 4, 0x00020000);
    };
    auto ml_rsrc = [&](int slot) {
      return __builtin_amdgcn_make_buffer_rsrc(part + ksplit * so * D + (slot * so + wrow) * 2, 0, 32 * nh * 2 * 4,
                                               0x00020000);
    };
    const int o_lane = r * nh * D * 4, ml_lane = r * nh * 2 * 4;
    if (live) {
      const __amdgpu_buffer_rsrc_t ro = o_rsrc(sp);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int d = dt * 32 + 8 * i4 + 4 * hh;
          const f32x4 v{acc_o[dt][4 * i4 + 0], acc_o[dt][4 * i4 + 1], acc_o[dt][4 * i4 + 2], acc_o[dt][4 * i4 + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ro, o_lane + d * 4, 0, 16);
        }
      if (hh == 0)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f32x2{m_run, l_run}), ml_rsrc(sp), ml_lane, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its partial is out
    __syncthreads();
    int& is_last = *reinterpret_cast<int*>(smem + kSmemMain);
    if (tid == 0) {
      int* ctr = counters + (static_cast<int64_t>(b) * ngrp + grp) * nkv + kvh;
      is_last = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
      if (is_last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    __syncthreads();
    if (!is_last || !live) return;
    // merge, latency-shaped: every split's (m, l) in one round trip, then the O partials (own
    // included: re-read, so the sequence of fmaf is the same whichever block is last) with the
    // next split's 16 loads in flight while the current one is summed
    f32x2 ml[kMaxSplit];
#pragma unroll
    for (int s2 = 0; s2 < kMaxSplit; ++s2)
      ml[s2] = __builtin_bit_cast(
          f32x2, __builtin_amdgcn_raw_buffer_load_b64(ml_rsrc(min(s2, nsplit - 1)), ml_lane, 0, 16));
    float M = -1e30f;
#pragma unroll
    for (int s2 = 0; s2 < kMaxSplit; ++s2)
      if (s2 < nsplit) M = fmaxf(M, ml[s2][0]);
    f32x4 ob[2][DT * 4];
    auto load_o = [&](int slot, f32x4* dst) {
      const __amdgpu_buffer_rsrc_t ro = o_rsrc(slot);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4)
          dst[dt * 4 + i4] = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(ro, o_lane + (dt * 32 + 8 * i4 + 4 * hh) * 4, 0, 16));
    };
    load_o(0, ob[0]);
    float L = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < kMaxSplit; ++s2) {
      if (s2 >= nsplit) break;
      if (s2 + 1 < nsplit) load_o(s2 + 1, ob[(s2 + 1) & 1]);
      const float sc = ml[s2][1] > 0.f ? __builtin_amdgcn_exp2f(ml[s2][0] - M) : 0.f;
      L = fmaf(ml[s2][1], sc, L);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc_o[dt][4 * i4 + j] = s2 == 0 ? ob[0][dt * 4 + i4][j] * sc
                                            : fmaf(ob[s2 & 1][dt * 4 + i4][j], sc, acc_o[dt][4 * i4 + j]);
    }
    l_run = L;
  } else if (!live) {
    return;
  }
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

// KV-split plan for a prefill launch: the grid is modelled as blocks of whole 64-key tiles
// dispatched longest-first onto one block per CU (248 VGPRs: 2 waves/SIMD = one 8-wave block), and
// the (ksplit, kmin) pair with the shortest greedy makespan wins: groups with >= 2 kmin tiles are
// split into min(ksplit, tiles / kmin) blocks. Costs in tile units (below). Assumes B sequences of
// the max shape.
extern "C" int llmc_attn_prefill_plan(int B, int max_qlen, int max_ctx, int nh, int nkv, int D, int bs, int* kmin_out) {
  *kmin_out = 1 << 30;
  if (nkv <= 0 || nh % nkv != 0 || max_qlen <= 0 || max_ctx < max_qlen) return 1;
  const int G = nh / nkv, npb = (max_qlen + 31) / 32, ngrp = (G * npb + 7) / 8, rows_pg = 8 / G > 0 ? 8 / G : 1;
  const int64_t units = static_cast<int64_t>(ngrp) * nkv * B;
  if (units > 4096) return 1;  // many rounds of blocks: the grid already balances
  std::vector<int> len(ngrp);
  for (int g = 0; g < ngrp; ++g) {  // group g's last row: rows_pg row tiles of 32 (causal key range)
    const int last_row = std::min(max_qlen, (g + 1) * rows_pg * 32);
    len[g] = (max_ctx - max_qlen + last_row + 63) / 64;
  }
  constexpr int kSlots = 256;
  // fitted to the r5 microbench sweep (profiles/r5_prefill_attention.md, 10 shapes x 7 splits): a
  // block's fixed cost is ~4 tiles (Q load, pipeline fill, launch share) and a split block's
  // hand-off 6 + 2 n more (sc1 partial write-through + drain, counter round trip, the merger's
  // reads of n partials)
  constexpr float kBlockCost = 4.f, kMergeCost = 6.f, kMergePerSplit = 2.f;
  auto makespan = [&](int S, int kmin) {
    std::vector<float> jobs;
    for (int g = ngrp - 1; g >= 0; --g) {  // dispatch order: longest group first
      const int n = S > 1 ? std::min(S, std::max(1, len[g] / kmin)) : 1;
      for (int r = 0; r < nkv * B; ++r)
        for (int sp = 0; sp < n; ++sp)
          jobs.push_back(static_cast<float>((sp + 1) * len[g] / n - sp * len[g] / n) + kBlockCost +
                         (n > 1 ? kMergeCost + kMergePerSplit * n : 0.f));
    }
    std::priority_queue<float, std::vector<float>, std::greater<float>> free_at;
    for (int i = 0; i < kSlots; ++i) free_at.push(0.f);
    float end = 0.f;
    for (float j : jobs) {
      const float t = free_at.top() + j;
      free_at.pop();
      free_at.push(t);
      end = std::max(end, t);
    }
    return end;
  };
  int best_s = 1, best_k = 1 << 30;
  // a split must win by > 3%; on a one-round grid by more: the unsplit grid then runs the key-halves
  // form (~0.6-0.7x of the 8-wave time this model prices; D = 128 on 64-key pages) or the paired /
  // 4-wave form (~0.83x) (llmc_attn_prefill_form). Measured: 4 / 1 heads at 8k keys still split
  // (model 0.52: 134-142 us vs halves 157); at 2k (0.72), 4k (0.68), 8 / 1 at 8k (0.71) halves wins.
  const bool halves_ok = D == 128 && bs == kKT;
  float best = makespan(1, 1 << 30) * (units <= 256 ? (halves_ok ? 0.62f : 0.80f) : 0.97f);
  // 4-way splits measured a loss everywhere but on grids of <= 128 blocks with >= 2 row tiles per
  // group (a TP=8 rank's single kv head) at >= 8k keys or on the smallest grids; the cost model
  // alone over-rates them elsewhere (8 / 2 heads at 4k keys: 0.56x predicted, 0.94x measured)
  const bool allow4 = G <= 4 && ((units <= 128 && max_ctx >= 8192) || units <= 32);
  for (int S : {2, 4})
    for (int kmin : {4, 8, 16}) {
      if (S == 4 && !allow4) continue;
      const float t = makespan(S, kmin);
      if (t < best) best = t, best_s = S, best_k = kmin;
    }
  *kmin_out = best_k;
  return best_s;
}

// Block form of a prefill launch: 0 = 8 waves (2 row tiles x 4 heads of one kv head share every
// staged K/V tile; one block per CU at 246 VGPRs), 1 = 8 waves with paired row tiles (a late and an
// early one per SIMD: mode 1 in the kernel), 2 = 4 waves, two blocks per CU (launch bound: <= 256
// VGPRs, so the one-tile lookahead; two tiles spill), 3 = key halves (8 waves = 4 row tiles x two
// halves of their key tiles, two tiles staged per step by LDS-DMA, the halves merged through LDS:
// mode 2; D = 128 on 64-key pages only). A split grid is form 0. On a grid of more than one round
// of the chip the longest-first order balances already and form 0 stays; when the 8-wave grid is
// ONE round (<= 256 blocks) its longest block (every key tile at 2 waves / SIMD) is the critical
// path, which the other forms shorten. Measured (MI355X, unsplit, us; two boxes ~5 % apart;
// profiles/r5_prefill_attention.md):
//   heads/kv  T      8 waves  paired  4 waves  halves
//   32/8     2048     76.6     58.5     69.2     61.8    (256 blocks, G <= 4: paired)
//   32/32    2048     69.9     57.0     63.3     57.3
//   32/8     1024     39.5     33.0     32.4     27.8    (<= 128 blocks: halves)
//   32/32    1024     39.4     35.3     32.4     26.9
//   16/2     2048     72.1      —       59.6     42.8    (G = 8: no pairs)
//   16/2     4096    129.3      —      115.7     92.1    (256 blocks, G = 8: halves)
//   32/8     8192     552      630      587      628     (4 rounds: 8 waves)
extern "C" int llmc_attn_prefill_form(int B, int max_qlen, int nh, int nkv, int ksplit, int D, int bs) {
  if (nkv <= 0 || nh % nkv != 0 || ksplit > 1) return 0;
  const int G = nh / nkv, npb = (max_qlen + 31) / 32;
  const int64_t units8 = static_cast<int64_t>((G * npb + 7) / 8) * nkv * B;
  if (units8 > 256) return 0;
  const bool halves_ok = D == 128 && bs == kKT, pairs_ok = G <= 4 && 8 % G == 0;
  if (units8 > 128 && pairs_ok) return 1;
  return halves_ok ? 3 : 2;
}

// Arrival counters a split launch needs: one per (sequence, row-tile group, kv head), where a split
// grid is the 8-wave form (ngrp = ceil(G * npb / 8), the kernel's gridDim.x / nkv / ksplit). The one
// size both the workspace allocator and the launch check use.
extern "C" int64_t llmc_attn_prefill_counters(int B, int max_qlen, int nh, int nkv) {
  if (nkv <= 0 || nh % nkv != 0 || max_qlen <= 0 || B <= 0) return 0;
  const int64_t npb = (max_qlen + 31) / 32, ngrp = ((nh / nkv) * npb + 7) / 8;
  return static_cast<int64_t>(B) * ngrp * nkv;
}

extern "C" int llmc_attn_prefill(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                 const void* block_tables, int bt_stride, const void* q_start, const void* q_lens,
                                 const void* ctx_lens, void* out, int out_stride, int B, int max_qlen, int nh, int nkv,
                                 int D, int bs, float scale, int ksplit, int kmin, void* part, void* counters,
                                 int T_all, int form_arg, hipStream_t s) {
  if (nh % nkv != 0 || ksplit < 1 || ksplit > kMaxSplit ||
      (ksplit > 1 && (part == nullptr || counters == nullptr || T_all < 1 || kmin < 1)))
    return -1;
  const int G = nh / nkv;
  const int npb = (max_qlen + 31) / 32;
  // block form: llmc_attn_prefill_form (its comment has the measurements)
  static const int form_env = [] {
    const char* e = getenv("LLMC_PREFILL_FORM");  // A/B runs: force form 0-3 (unsplit grids)
    return e ? atoi(e) : -1;
  }();
  // form_arg: -1 = llmc_attn_prefill_form's choice, 0-3 forced (tests; unsplit grids only)
  int form = llmc_attn_prefill_form(B, max_qlen, nh, nkv, ksplit, D, bs);
  if (form_env >= 0 && form_env <= 3 && ksplit == 1) form = form_env;
  if (form_arg >= 0 && form_arg <= 3 && ksplit == 1) form = form_arg;
  if (form == 1 && (G > 4 || 8 % G != 0)) form = 0;  // pairs need WPB / G >= 2 row tiles
  if (form == 3 && !(D == 128 && bs == kKT)) form = 2;  // key halves: LDS-DMA staging only
  const int wpb = form == 2 ? 4 : 8, mode = form == 1 ? 1 : form == 3 ? 2 : 0;
  static const int dma_env = [] {
    // LDS-DMA K/V staging (64-key pages, D = 128, 8-wave blocks): 2-5 % faster on every measured
    // shape (2k 65.8 -> 62.5 us, 8k 601 -> 587, 32k keys 3893 -> 3831; profiles/r5_prefill_attention.md)
    const char* e = getenv("LLMC_PREFILL_DMA");  // A/B runs: 0 = register staging
    return e ? atoi(e) : 1;
  }();
  const bool dma = (dma_env || mode == 2) && wpb == 8 && D == 128 && bs == kKT;
  dim3 grid((G * npb + (mode == 2 ? 4 : wpb) - 1) / (mode == 2 ? 4 : wpb) * ksplit * nkv, 1, B);
  const float sl2 = scale * 1.4426950408889634f;
  static const int la = [] {
    const char* e = getenv("LLMC_PREFILL_LOOKAHEAD");  // A/B runs: K/V tiles requested ahead
    return e ? atoi(e) : kPrefillLookahead;
  }();
#define LLMC_PF(DD, L)                                                                                           \
  do {                                                                                                           \
    if (bs == kKT) LLMC_PFP(DD, L, true);                                                                        \
    else LLMC_PFP(DD, L, false);                                                                                 \
  } while (0)
#define LLMC_PFW(DD, L, P, W)                                                                                    \
  attn_prefill_kernel<DD, W, L, P><<<grid, W * 64, 0, s>>>((const bf16_t*)q, q_stride, (const bf16_t*)k_cache,     \
                                               (const bf16_t*)v_cache, (const int32_t*)block_tables, bt_stride,   \
                                               (const int32_t*)q_start, (const int32_t*)q_lens,                  \
                                               (const int32_t*)ctx_lens, (bf16_t*)out, out_stride, nh, nkv, bs, sl2, \
                                               ksplit, kmin, (float*)part, (int*)counters, T_all, mode)
#define LLMC_PFP(DD, L, P)                         \
  do {                                             \
    if (L == 1 && wpb == 4) LLMC_PFW(DD, 1, P, 4); \
    else LLMC_PFW(DD, L, P, 8);                    \
  } while (0)
#define LLMC_PF_D(DD)                          \
  do {                                         \
    if (la >= 2 && wpb == 8) LLMC_PF(DD, 2);   \
    else LLMC_PF(DD, 1);                       \
  } while (0)
  if (dma) {
    attn_prefill_kernel<128, 8, 1, true, true><<<grid, 512, 0, s>>>(
        (const bf16_t*)q, q_stride, (const bf16_t*)k_cache, (const bf16_t*)v_cache, (const int32_t*)block_tables,
        bt_stride, (const int32_t*)q_start, (const int32_t*)q_lens, (const int32_t*)ctx_lens, (bf16_t*)out, out_stride,
        nh, nkv, bs, sl2, ksplit, kmin, (float*)part, (int*)counters, T_all, mode);
    return static_cast<int>(hipGetLastError());
  }
  switch (D) {
    case 64: LLMC_PF_D(64); break;
    case 96: LLMC_PF_D(96); break;
    case 128: LLMC_PF_D(128); break;
    default: return -2;
  }
#undef LLMC_PF_D
#undef LLMC_PF
#undef LLMC_PFP
#undef LLMC_PFW
  return static_cast<int>(hipGetLastError());
}
