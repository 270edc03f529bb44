// K5 + o_proj of a batch-1 decode step in ONE launch (host: llmc_attn_oproj):
//     h[n] += sum_k Wo[n, k] * attention(q, K/V cache)[k]   (or h[n] = ..., a TP rank's partial)
//
// Why (profiles/r2_dec2k_kernel_stats.md, 8B at 2k keys): as two launches the attention is a
// latency chain (10.6 us for ~10 MB of K/V) and o_proj pays its own boundary + ramp (7.2 us for
// 34 MB, 4.7 TB/s). Here the o_proj weights stream while the attention merges and hands off; when
// the merged head output arrives the projection is arithmetic on registers. Measured
// (profiles/r3_attn_oproj.md): faster than the two launches only where the attention is long
// (6k-8k keys: 18.9-21.5 vs 20.9-23.3 us), slower at <= 4k and on TP ranks; the engine takes it
// for 256-key blocks (ops.ATTN_OPROJ_MIN_CHUNK).
//
// Grid: (nc, nkv) blocks of 8 waves; block (c, g) = kv head g x the fixed key range
// [c * chunk, (c + 1) * chunk) (<= 256 keys: one 32-key MFMA sub-tile per wave, attn_core.h; <= 512:
// two, with the weights requested late so the second sub-tile's registers are free) AND
// the o_proj tile rows [c R, (c + 1) R) x input columns of head group g (its G query heads):
// R = H / nc rows, R / 4 per o wave (waves 0-3; waves 4-7 run the latency chain, see "Roles"),
// each lane one 16-B column chunk per row (G D = 512).
//
//   1. one round trip for Q, L, the wave's page id and the two epochs; K/V of the wave's
//      sub-tile; the block's o_proj weight tile (nt loads) right behind the K/V (mode 0) or after
//      the head ticket of step 2 (mode 1: the K/V never queue behind the weights) — except in the
//      head's merger with mode bit 1 (mode 3, the default), which requests its tile after step 3:
//      a CU's loads retire through one queue, so the merge's loads would wait behind 128 KB of
//      weights (1.1-1.4 us per launch, profiles/r4_attn_oproj_defer.md)
//   (mode bit 2, the default where the shape allows it: steps 4-5 become whole o_proj rows per
//   block over every head's output, see FR below — no tile partials and no reduce chain)
//   2. attention sub-tile -> block state -> partial granules (attn_core.h publish) and a ticket
//      on head g's counter (EVERY block of head g takes one, keys or not)
//   3. the last arriver of head g merges the partials and publishes head g's output (bf16) as
//      {value, tag} granules; every block of head g polls those (the merger is running: it took
//      the last ticket, so no wait is on a block that has not started — deadlock-free whatever
//      the residency, safe beside co-located engines)
//   4. o_proj partial of the tile over head g's columns (reduce-scatter across the lanes), as
//      {f32, tag} granules; a ticket on tile c's counter; its nkv-th arriver sums the nkv
//      partials in head order (deterministic) and adds them to the residual row h
//   5. the last tile reducer re-arms the exit counter and advances the tile epoch (every block
//      read it before arriving)
//
// Every spin is bounded: a give-up sets the fault word (checked by the engine like attn_decode's).
//
// MoE router in the same launch (whole-row form, an engine alone on its GPU; AoRouter): a Mixtral
// layer's decode router (RMSNorm -> E router logits -> top-k) was its own ~6.3-us launch between
// this one and the expert GEMVs. The logits are linear in the block's rows: logit_e =
// rsqrt(mean h^2 + eps) * sum_n Wr[e][n] norm_w[n] h[n], so each block publishes its 16 rows'
// share (E partial dots and the partial sum of squares, from router / norm weights it requested at
// its start) as data-tagged granules and block 0 sums them in block order and picks the top k
// (ao_router_tail).
#include "attn_core.h"
#include "car_proto.h"

namespace llmc {

constexpr int kAoThreads = 512, kAoWaves = kAoThreads / kWave;
constexpr int kAoLine = 16;  // int32 words per counter line (64 B)
constexpr int kAoMaxKv = 8;  // kv heads (= head groups summed per o_proj row) at most
constexpr unsigned kAoL2Polls = 16;  // polls of the same-XCD L2 copy of the partials before the write-through one

// Reduce-scatter of N per-lane row sums over the 64 lanes, one stage per lane bit M = 32, 16, ...:
// lanes with bit M keep the upper half of the live rows, the others the lower half, and add the
// partner's copy. Recursion keeps every index a constant (a loop over the stages left hipcc with
// runtime-indexed register arrays: thousands of selects, ~10 us per call).
template <int N, int M, int RWt>
__device__ __forceinline__ void ao_reduce_scatter(float (&s)[RWt], int lane) {
  if constexpr (N > 1) {
    const bool up = (lane & M) != 0;
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const float send = up ? s[i] : s[i + N / 2];
      const float keep = up ? s[i + N / 2] : s[i];
      s[i] = keep + xor_shfl<M>(send, lane);
    }
    ao_reduce_scatter<N / 2, M / 2, RWt>(s, lane);
  }
}

// Diagnostics (stamps != nullptr): 8 s_memrealtime stamps (100 MHz) per block, see llmc_attn_oproj.
__device__ __forceinline__ void ao_stamp(uint64_t* st, int k, bool who) {
  if (st != nullptr && who) st[k] = __builtin_amdgcn_s_memrealtime();
}

// The MoE router folded into the whole-row launch (see the header). Wr == nullptr: off.
struct AoRouter {
  const bf16_t* norm_w;  // the layer's post-attention RMSNorm weights [H]
  const bf16_t* Wr;      // router weights [E][H], E <= kAoRouterMaxE
  float eps;
  int E, k;              // top k of E
  float* w_out;          // [k] renormalised top-k weights
  int32_t* ids_out;      // [k] expert ids
  uint64_t* part;        // [9][kAoRouterMaxBlocks] {f32, tag} granules: per block its logit partials [8], sum of squares
  int* epoch;            // granule epoch (advanced by the merger)
};
constexpr int kAoRouterWave = 5;  // a control wave: no weight tile in its registers
constexpr int kAoRouterMaxE = 8, kAoRouterMaxBlocks = 256;

// Router partials, one wave (kAoRouterWave) of every block, after the block's 16 h rows are final:
// rv = those rows (bf16 values as stored, in f32), rw / rg = lane (e = lane / 4, q = lane % 4)'s
// router / norm weights of rows 4 q .. 4 q + 3 (requested at the block's start), tag = this
// launch's granule tag. The block's 9 values go out as data-tagged granules (no drain, no ticket).
// Block 0's router wave then merges: it re-polls the granule rows (by quantity, so a wave load
// reads 64 consecutive blocks' values: a few lines) until every tag is this launch's, sums them in
// block order and picks the top k. Block 0 waits on the grid's other blocks here, none of which
// ever waits on block 0 (no cycle, whatever the residency: a block not yet resident gets its CU
// when some kernel's block finishes); for an engine alone on its GPU the whole 256-block grid is
// resident and the wait ends with the last block's publish. Bounded (fault 4). (A ticketed
// last-arriver merge measured 5.1 us on the chain, the top-k as its own launch 4.9:
// profiles/r6_decode_experiments.md.)
__device__ __forceinline__ void ao_router_tail(const AoRouter& rt, const float* rv, u32x2 rw, u32x2 rg, uint32_t tag,
                                               int blk, int nblk, int H, int lane, int* fault) {
  float p = 0.f;
  if (lane < 32) {
    const int q4 = lane & 3;
    const float w[4] = {bf16_lo(rw[0]), bf16_hi(rw[0]), bf16_lo(rw[1]), bf16_hi(rw[1])};
    const float gm[4] = {bf16_lo(rg[0]), bf16_hi(rg[0]), bf16_lo(rg[1]), bf16_hi(rg[1])};
#pragma unroll
    for (int j = 0; j < 4; ++j) p += w[j] * (gm[j] * rv[4 * q4 + j]);
  }
  p += xor_shfl<1>(p, lane);
  p += xor_shfl<2>(p, lane);
  float sq = lane < 16 ? rv[lane] * rv[lane] : 0.f;
  sq += xor_shfl<1>(sq, lane);
  sq += xor_shfl<2>(sq, lane);
  sq += xor_shfl<4>(sq, lane);
  sq += xor_shfl<8>(sq, lane);
  const float pv = __shfl(p, (lane & 7) * 4, 64);  // every lane takes part in both shuffles
  const float sv = __shfl(sq, 0, 64);
  if (lane <= 8) {
    const uint64_t gv = static_cast<uint64_t>(__float_as_uint(lane < 8 ? pv : sv)) | (static_cast<uint64_t>(tag) << 32);
    __hip_atomic_store(rt.part + lane * kAoRouterMaxBlocks + blk, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (blk != 0) return;
  constexpr int NR = kAoRouterMaxBlocks / 64;
  uint64_t v[NR][9];
  for (unsigned spins = 0;; ++spins) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int b = min(r * 64 + lane, nblk - 1);  // clamped: loads in flight together, masked below
#pragma unroll
      for (int i = 0; i < 9; ++i)
        v[r][i] = __hip_atomic_load(rt.part + i * kAoRouterMaxBlocks + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int i = 0; i < 9; ++i) ok = ok && static_cast<uint32_t>(v[r][i] >> 32) == tag;
    if (__all(ok)) break;
    if (spins >= kSpinLimit) {
      if (lane == 0 && fault != nullptr) __hip_atomic_store(fault, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  float acc[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] = 0.f;
#pragma unroll
  for (int r = 0; r < NR; ++r)
    if (r * 64 + lane < nblk)
#pragma unroll
      for (int i = 0; i < 9; ++i) acc[i] += __uint_as_float(static_cast<uint32_t>(v[r][i]));
#pragma unroll
  for (int i = 0; i < 9; ++i) acc[i] = wave_sum(acc[i]);
  if (lane == 0) {
    // softmax over the E logits, top k (lowest index on ties), renormalised: moe_router_kernel's rule
    const float inv = rsqrtf(acc[8] / H + rt.eps);
    float lg[kAoRouterMaxE];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < kAoRouterMaxE; ++e) {
      lg[e] = acc[e] * inv;
      if (e < rt.E) mx = fmaxf(mx, lg[e]);
    }
    float z = 0.f;
#pragma unroll
    for (int e = 0; e < kAoRouterMaxE; ++e)
      if (e < rt.E) z += __expf(lg[e] - mx);
    uint32_t taken = 0;
    float sel[kAoRouterMaxE];
    float ssum = 0.f;
    for (int j = 0; j < rt.k; ++j) {
      int best = 0;
      float bv = -INFINITY;
      for (int e = 0; e < rt.E; ++e) {
        if ((taken >> e) & 1u) continue;
        if (lg[e] > bv) {
          bv = lg[e];
          best = e;
        }
      }
      taken |= 1u << best;
      sel[j] = __expf(bv - mx) / z;
      ssum += sel[j];
      rt.ids_out[j] = best;
    }
    for (int j = 0; j < rt.k; ++j) rt.w_out[j] = sel[j] / ssum;
    __hip_atomic_store(rt.epoch, static_cast<int>(tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// FR = 0: block (c, g) owns o_proj rows [c R, (c + 1) R) x head group g's columns, its partial
// summed over the nkv head groups by the tile's last arriver (step 4). FR = nkv (full rows, mode
// bit 2): block (c, g) owns R / nkv WHOLE rows [(g nc + c) R / nkv, ...) x every head group's
// columns, gathers every head's output and writes its rows itself — no tile partials, no tile
// ticket, no reduce chain after the dot (same weight bytes per block)
template <int G, int D, int RW, bool LATE, int SUBS, int FR = 0>
__global__ __launch_bounds__(kAoThreads) void attn_oproj_kernel(
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int32_t* __restrict__ block_table, int bt_len, const int32_t* __restrict__ seq_len,
    const bf16_t* __restrict__ w_o, int K_o, bf16_t* __restrict__ h, bf16_t* __restrict__ attn_out,
    float* __restrict__ part, uint32_t* __restrict__ handoff, uint64_t* __restrict__ tile_part, int* __restrict__ ctr,
    int* __restrict__ fault, int nkv, int bs, int nblocks, int chunk, float scale_log2,
    uint64_t* __restrict__ stamps, int defer, int add_resid, CarArgs ar, int gate, int prio, AoRouter rt,
    int l2copy) {
  static_assert(G * D == 512, "one 16-B column chunk per lane per row");
  static_assert(RW >= 1 && RW <= 32 && (RW & (RW - 1)) == 0, "rows per wave: power of two <= 32");
  static_assert(SUBS == 1 || (SUBS == 2 && LATE), "two sub-tiles per wave only with late weights (registers)");
  static_assert(FR == 0 || (LATE && RW % FR == 0 && FR <= kAoMaxKv), "full rows: late weights, RW / FR rows per o wave");
  using ST = SubTile<G, D>;
  constexpr int HQ = D / 4, RU = HQ + 1, Q = G * HQ;  // 16-B units: per head, per partial row, per group
  constexpr int R = 4 * RW;                              // o_proj rows per block (4 o waves)
  // block b = (c, g) with g = b % nkv: under the observed round-robin dispatch the nc blocks of a kv
  // head share one XCD (b % 8), so the head's merger can read their partials from that XCD's L2
  // (see step 2; placement only ever changes the speed)
  const int c = blockIdx.x / nkv, g = blockIdx.x % nkv, nc = gridDim.x / nkv;
  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  uint64_t* stp = stamps != nullptr ? stamps + (static_cast<int64_t>(g) * nc + c) * 8 : nullptr;
  ao_stamp(stp, 0, tid == 0);
  int* hctr = ctr + g * kAoLine;            // {-, head epoch, head ticket (u64: count + per-XCD counts)}
  int* tctr = ctr + (nkv + c) * kAoLine;    // {tile ticket}
  int* xctr = ctr + (nkv + nc) * kAoLine;   // {exit count, tile epoch}
  int* gctr = ctr + (nkv + nc + 1) * kAoLine;  // {attention arrivals, weight-gate epoch} (mode bit 3)

  // ---- 1. one round trip: epochs, L, this wave's page id (scalar), Q (vector) ----
  const uint32_t tag_h = static_cast<uint32_t>(__hip_atomic_load(hctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  const uint32_t tag_t = static_cast<uint32_t>(__hip_atomic_load(xctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  const int gate_e = gate ? __hip_atomic_load(gctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  const int L = ld_scalar(seq_len);
  const int key_lo = c * chunk;
  const int wk0 = key_lo + wave * 32 * SUBS;  // this wave's SUBS 32-key sub-tiles (one page: bs % (32 SUBS) == 0)
  const int pidx = __builtin_amdgcn_readfirstlane(min(wk0 / bs, bt_len - 1));
  const int page = min(max(ld_scalar(block_table + pidx), 0), nblocks - 1);  // clamped into the cache
  ST st;
  st.init(q + g * G * D, lane);
  // fused router (FR): the router wave requests its rows' router / norm weights now (tiny, behind
  // nothing), used only after the block's o_proj rows are final
  u32x2 rt_w = {0u, 0u}, rt_g = {0u, 0u};
  uint32_t rt_tag = 0;
  if constexpr (FR != 0) {
    if (rt.Wr != nullptr && wave == kAoRouterWave) {
      rt_tag = static_cast<uint32_t>(__hip_atomic_load(rt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
      if (lane < 32) {
        const int e = lane >> 2;
        const int rb = (g * nc + c) * (R / FR) + 4 * (lane & 3);
        if (e < rt.E) rt_w = *reinterpret_cast<const u32x2*>(rt.Wr + static_cast<int64_t>(e) * nc * R + rb);
        rt_g = *reinterpret_cast<const u32x2*>(rt.norm_w + rb);
      }
    }
  }
  const int key_hi = min(L, key_lo + chunk);
  const bool wave_keys = wk0 < key_hi;  // wave-uniform
  const bool block_keys = key_lo < L;   // block-uniform
  const int nsplit = (L + chunk - 1) / chunk;  // blocks of head g with keys (host: nc * chunk >= L)

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* vbuf = smem + wave * 32 * kVRowBytes;                              // per-wave V image
  float* red = reinterpret_cast<float*>(smem + kAoWaves * 32 * kVRowBytes);  // [8][G][D + 2]
  u32x4* xs = reinterpret_cast<u32x4*>(red + kAoWaves * G * (D + 2));      // head g's output, 64 chunks
  int* flag = reinterpret_cast<int*>(xs + (FR ? FR : 1) * 64);  // xs: head g's output (FR: every head's)

  bf16x8 kf[2][ST::KS], kf2[2][ST::KS];
  u32x4 vs[ST::NV], vs2[ST::NV];
  const int64_t kvbase = (static_cast<int64_t>(page) * nkv + g) * bs * D;
  // sub-tile t: keys [k0_t, k0_t + 32) of the wave. A sub-tile without keys issues its loads anyway,
  // all at one row of the page (L2 hits): loads under a branch would end in a register merge at
  // the join that waits for them before the weights issue; its scores are all masked (end = k0_t)
  const int k0_0 = wk0, k0_1 = wk0 + 32;
  const bool has0 = wave_keys, has1 = SUBS == 2 && k0_1 < key_hi;
  const int end_ld0 = has0 ? min(key_hi, k0_0 + 32) : k0_0 + 1, end_c0 = has0 ? min(key_hi, k0_0 + 32) : k0_0;
  const int end_ld1 = has1 ? min(key_hi, k0_1 + 32) : k0_1 + 1, end_c1 = has1 ? min(key_hi, k0_1 + 32) : k0_1;
  auto row0 = [&](const bf16_t* cache, int key) {
    return cache + kvbase + (has0 ? static_cast<int64_t>(key % bs) * D : 0);
  };
  auto row1 = [&](const bf16_t* cache, int key) {
    return cache + kvbase + (has1 ? static_cast<int64_t>(key % bs) * D : 0);
  };

  // Roles. The vector memory counter retires in order, so a wave with o_proj weights in flight
  // cannot use any later load's result (a ticket's return value, a merge or poll load) before its
  // weights have landed. Waves 0-3 (the "o waves") therefore carry the weights and nothing on the
  // latency chain; waves 4-7 (the "control waves", no weights) publish the partial, take the
  // tickets, merge, poll the hand-off and reduce the tile. Every wave computes one attention
  // sub-tile. The o_proj tile: rows n = c R + ow RW + j (ow = o wave), columns g G D + 8 lane .. + 8.
  const bool o_wave = wave < 4;  // wave-uniform
  // mode bit 4: the control waves (the latency chain: publish, tickets, merge, hand-off, tile
  // reduce) issue ahead of the o waves on their SIMDs (s_setprio 3 vs 0)
  if (prio && !o_wave) __builtin_amdgcn_s_setprio(3);
  const int ct = tid - 256;      // control-thread index (waves 4-7: 0..255)
  // tickets from wave 6: it has neither weights nor partial / hand-off stores in flight (stores
  // count in the same counter), so the returned value is usable at once
  constexpr int kTicketThread = 128;
  // The attention step is written out in each role's branch: with one shared copy after the
  // branches, hipcc's counter model at the join would make the o waves wait for their weights
  // before the MFMAs (it assumes the fewest loads in flight over both paths).
  u32x4 wt[RW];
  // FR: o wave rows (g nc + c) R / FR + wave RW / FR + j, element j FR + jj = head group jj's columns
  constexpr int RWF = FR ? RW / FR : RW;  // rows per o wave
  const bf16_t* wrow = FR ? w_o + static_cast<int64_t>((g * nc + c) * (R / (FR ? FR : 1)) + wave * RWF) * K_o + 8 * lane
                          : w_o + static_cast<int64_t>(c * R + wave * RW) * K_o + g * G * D + 8 * lane;
  auto load_tile = [&]() {
#pragma unroll
    for (int j = 0; j < RW; ++j)
      wt[j] = load16<true>(FR ? wrow + static_cast<int64_t>(j / (FR ? FR : 1)) * K_o + (j % (FR ? FR : 1)) * G * D
                              : wrow + static_cast<int64_t>(j) * K_o);  // nt: read once
  };
  if (o_wave) {
    st.issue(k0_0, end_ld0, lane, row0, k_cache, v_cache, kf, vs);
    if constexpr (SUBS == 2) st.issue(k0_1, end_ld1, lane, row1, k_cache, v_cache, kf2, vs2);
    __builtin_amdgcn_sched_barrier(0);  // every K/V load issues before the first weight load
    if constexpr (!LATE) {
      load_tile();
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- 2. attention sub-tile (K/V were issued before the weights: the wait leaves them in flight).
    // Unconditional: a wave without keys masks every score (its state stays empty); under a branch
    // hipcc would sink the last K/V load into it, behind the weights.
    st.compute(k0_0, end_c0, lane, vbuf, scale_log2, kf, vs);
    if constexpr (SUBS == 2) st.compute(k0_1, end_c1, lane, vbuf, scale_log2, kf2, vs2);
    ao_stamp(stp, 1, tid == 0);
  } else {
    st.issue(k0_0, end_ld0, lane, row0, k_cache, v_cache, kf, vs);
    if constexpr (SUBS == 2) st.issue(k0_1, end_ld1, lane, row1, k_cache, v_cache, kf2, vs2);
    st.compute(k0_0, end_c0, lane, vbuf, scale_log2, kf, vs);
    if constexpr (SUBS == 2) st.compute(k0_1, end_c1, lane, vbuf, scale_log2, kf2, vs2);
    ao_stamp(stp, 2, ct == 0);
  }
  // ---- ... -> block state -> partial -> head ticket ----
  st.to_lds(red, wave, lane);
  __syncthreads();
  // Two copies of the partial: write-through granules in `slab` (read by a merger anywhere) and
  // default-policy ones in `slab_l2` (they stay in this XCD's L2). The head ticket also counts the
  // arrivals per XCD (6 bits each above an 8-bit total), so the merger knows whether every producer
  // of its head ran on its own XCD; then it reads the L2 copy (L2 hits, not fabric round trips queued
  // behind the other blocks' weight stream), else the write-through one. Tags decide either way.
  const int slab_rows = nc;
  float* slab = part + static_cast<int64_t>(g) * slab_rows * G * RU * 4;
  float* slab_l2 = part + static_cast<int64_t>(nkv + g) * slab_rows * G * RU * 4;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(slab, 0, slab_rows * G * RU * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsrc_l2 =
      __builtin_amdgcn_make_buffer_rsrc(slab_l2, 0, slab_rows * G * RU * 16, 0x00020000);
  if (block_keys) {
    if (l2copy) publish_partial_dual<G, D, kAoWaves>(red, rsrc, rsrc_l2, c, tag_h, o_wave ? Q : ct);
    else publish_partial<G, D, kAoWaves>(red, rsrc, c, tag_h, o_wave ? Q : ct);
  }
  __syncthreads();  // every wave's stores are issued (the merger checks tags)
  if (ct == kTicketThread) {
    const uint32_t xcc = xcc_id();
    const uint64_t old = __hip_atomic_fetch_add(reinterpret_cast<uint64_t*>(hctr + 2),
                                                1ull + (1ull << (8 + 6 * xcc)), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    *flag = static_cast<int>(old & 255) == nc - 1;
    flag[1] = l2copy && nc <= 63 && static_cast<int>((old >> (8 + 6 * xcc)) & 63) == nc - 1;  // all on my XCD
    // weight gate (mode bit 3): the last block of the whole grid to finish its attention opens it
    if (gate && __hip_atomic_fetch_add(gctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nc * nkv - 1) {
      __hip_atomic_store(gctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gctr + 1, gate_e + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  ao_stamp(stp, 3, tid == 0);
  // Weight gate (mode bit 3, engines alone on their GPU): the o waves request their weight tile only
  // once EVERY block of the grid has streamed its K/V, so no head's last K/V loads (the merge chain's
  // start) queue behind other blocks' weight requests. Purely a scheduling device — no data depends
  // on it — so the wait is short-bounded and then goes ahead regardless (never a deadlock, e.g.
  // beside co-located engines whose blocks hold the CUs some of this grid's blocks need).
  auto weight_gate = [&]() {
    if (gate && lane == 0) {
      for (unsigned spins = 0; spins < (1u << 14) &&
                               __hip_atomic_load(gctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gate_e + 1;
           ++spins)
        __builtin_amdgcn_s_sleep(2);
    }
  };
  // defer (late weights only): the head's merger requests its weight tile after the merge instead,
  // so the merge's loads do not queue behind 128 KB of weights in this CU's memory pipeline
  const bool merger_defers = LATE && defer && *flag;  // block-uniform
  if constexpr (LATE) {
    // weights behind the whole attention step: the K/V loads never queue behind them, and a wave
    // stalled issuing 32 KB of loads holds no barrier the control waves need before the next one
    if (o_wave && !merger_defers) {
      weight_gate();
      load_tile();
    }
  }

  // ---- 3. the last arriver of head g merges (control waves) and publishes head g's output ----
  uint32_t* hoff = handoff + static_cast<int64_t>(g) * Q * 4;  // Q 16-B units {bf16x2, tag, bf16x2, tag}
  const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(hoff, 0, Q * 16, 0x00020000);
  if (*flag) {
    f32x4 ms, acc;
    // A deferring merger's o waves hold no weights yet: all 8 waves merge, so 32 partials are one
    // pass of 8 loads in flight per thread (one round trip on the critical path instead of two;
    // 16 rows per thread would spill the o waves' weight registers of the other blocks). Merge
    // thread mt < Q ends with output unit mt (dims 4 mt .. 4 mt + 3).
    int mt;
    const unsigned l2_polls = flag[1] ? kAoL2Polls : 0u;  // block-uniform
    if (merger_defers) {
      mt = tid;
      merge_rows<G, D, kAoThreads>(rsrc, reinterpret_cast<const char*>(slab), 0, nsplit, tag_h,
                                   reinterpret_cast<f32x4*>(smem), tid, ms, acc, fault, rsrc_l2,
                                   reinterpret_cast<const char*>(slab_l2), l2_polls);
    } else {
      mt = o_wave ? 256 + tid : ct;
      merge_rows<G, D, 256>(rsrc, reinterpret_cast<const char*>(slab), 0, nsplit, tag_h,
                            reinterpret_cast<f32x4*>(smem), mt, ms, acc, fault, rsrc_l2,
                            reinterpret_cast<const char*>(slab_l2), l2_polls);
    }
    if constexpr (FR != 0) ao_stamp(stp, 6, tid == 0);  // whole rows: 6 / 7 = the head merger's merge / publish
    if (mt < Q) {
      const float inv = 1.f / ms[1];
      const uint32_t lo = pack_bf16x2(acc[0] * inv, acc[1] * inv), hi = pack_bf16x2(acc[2] * inv, acc[3] * inv);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo, tag_h, hi, tag_h}, hr, mt * 16, 0, 16);
      const int gq = mt / HQ, u = mt % HQ;
      *reinterpret_cast<u32x2*>(attn_out + (g * G + gq) * D + 4 * u) = u32x2{lo, hi};
      if (merger_defers) {  // its own copy straight into LDS (units mt = dims 4 mt .. 4 mt + 3)
        uint32_t* xg = reinterpret_cast<uint32_t*>(xs + (FR ? g * 64 : 0));
        xg[2 * mt] = lo;
        xg[2 * mt + 1] = hi;
      }
    }
    if (ct == 0) {
      __hip_atomic_store(reinterpret_cast<uint64_t*>(hctr + 2), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
      __hip_atomic_store(hctr + 1, static_cast<int>(tag_h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // epoch
    }
    if constexpr (FR != 0) ao_stamp(stp, 7, tid == 0);
  }

  // FR: the merger's merge is done (its head output is in LDS): its weights go now, while its
  // control waves poll the other heads
  if constexpr (FR != 0) {
    if (merger_defers) {
      __syncthreads();
      if (o_wave) {
        weight_gate();
        load_tile();
      }
    }
  }
  // head outputs into LDS: head g only (FR = 0: wave 4) or every head (FR: control wave 4 + k
  // takes heads k, k + 4, ...), the merger's own head skipped (already there)
  if (!o_wave && (FR != 0 || wave == 4)) {
    for (int gg = FR ? wave - 4 : g; gg < (FR ? nkv : g + 1); gg += 4) {
      if (merger_defers && gg == g) continue;
      const uint32_t* ho = handoff + static_cast<int64_t>(gg) * Q * 4;
      // 8-B relaxed atomic loads, one granule each: ordered loads are re-issued on every poll
      // (plain buffer loads in this loop would look loop-invariant to hipcc and be hoisted out)
      const char* hb = reinterpret_cast<const char*>(ho) + 32 * lane;
      u32x2 a0, a1, b0, b1;
      // one lane polls one granule (256 blocks polling every granule flooded the memory path the
      // weights stream through); once it has landed the wave reads them all (re-read if any lags)
      if (lane == 0) {
        for (unsigned spins = 0; ld8_atomic(reinterpret_cast<const char*>(ho), 0)[1] != tag_h && spins < kSpinLimit;
             ++spins)
          __builtin_amdgcn_s_sleep(2);
      }
      for (unsigned spins = 0;; ++spins) {
        a0 = ld8_atomic(hb, 0);
        a1 = ld8_atomic(hb, 8);
        b0 = ld8_atomic(hb, 16);
        b1 = ld8_atomic(hb, 24);
        if (__all(a0[1] == tag_h && a1[1] == tag_h && b0[1] == tag_h && b1[1] == tag_h)) break;
        if (spins >= kSpinLimit) {
          if (lane == 0 && fault != nullptr) __hip_atomic_store(fault, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      xs[(FR ? gg * 64 : 0) + lane] = u32x4{a0[0], a1[0], b0[0], b1[0]};  // dims 8 lane .. + 7 of head group gg
    }
  }
  __syncthreads();
  ao_stamp(stp, 4, tid == 0);
  if constexpr (LATE && FR == 0) {
    if (o_wave && merger_defers) {
      weight_gate();
      load_tile();
    }
  }
  if constexpr (FR != 0) {
    // ---- 4'. whole rows: dot over every head group, reduce-scatter, residual add, done ----
    if (o_wave) {
      float s[RWF];
#pragma unroll
      for (int j = 0; j < RWF; ++j) {
        float a = 0.f;
#pragma unroll
        for (int jj = 0; jj < FR; ++jj) a = dot8_bf16(wt[j * FR + jj], xs[jj * 64 + lane], a);
        s[j] = a;
      }
      ao_reduce_scatter<RWF, 32>(s, lane);
      constexpr int LPR = 64 / RWF;
      s[0] = xor_tree_sum<LPR / 2>(s[0], lane);
      if ((lane % LPR) == 0) {
        bf16_t* hp = h + (g * nc + c) * (R / FR) + wave * RWF + lane / LPR;
        const bf16_t hv = f32_to_bf16((add_resid ? bf16_to_f32(*hp) : 0.f) + s[0]);
        *hp = hv;
        if (rt.Wr != nullptr) reinterpret_cast<float*>(flag + 4)[wave * RWF + lane / LPR] = bf16_to_f32(hv);
      }
      ao_stamp(stp, 5, tid == 0);
    }
    if (rt.Wr == nullptr) return;  // block-uniform
    __syncthreads();               // the block's 16 rows are in LDS
    if (wave == kAoRouterWave)
      ao_router_tail(rt, reinterpret_cast<const float*>(flag + 4), rt_w, rt_g, rt_tag, g * nc + c, nc * nkv, nc * R,
                     lane, fault);
    return;
  }

  // ---- 4. o_proj partial over head g's columns (o waves); reduce-scatter the RW row sums ----
  uint64_t* tp = tile_part + (static_cast<int64_t>(c) * nkv) * R;
  if (o_wave) {
    float s[RW];
    const u32x4 x = xs[lane];
#pragma unroll
    for (int j = 0; j < RW; ++j) s[j] = dot8_bf16(wt[j], x, 0.f);
    ao_reduce_scatter<RW, 32>(s, lane);
    constexpr int LPR = 64 / RW;  // lanes sharing one row after the stages (the low log2(LPR) bits)
    s[0] = xor_tree_sum<LPR / 2>(s[0], lane);
    if ((lane % LPR) == 0) {
      const int my_row = wave * RW + lane / LPR;  // row within the tile
      const uint64_t gv = static_cast<uint64_t>(__float_as_uint(s[0])) | (static_cast<uint64_t>(tag_t) << 32);
      __hip_atomic_store(tp + g * R + my_row, gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // 8-B sc1 store
    }
    ao_stamp(stp, 5, tid == 0);
  }
  __syncthreads();
  if (ct == kTicketThread) *flag = __hip_atomic_fetch_add(tctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nkv - 1;
  __syncthreads();
  ao_stamp(stp, 6, tid == 0);
  if (*flag == 0) return;

  // ---- the tile's nkv-th arriver (control waves): h[rows] += sum over heads, fixed order ----
  if (ct >= 0 && ct < R) {
    // every head's granule of this row in flight at once (nkv <= kAoMaxKv), re-polled until all
    // tags match; summed in head order
    uint64_t v[kAoMaxKv];
    for (unsigned spins = 0;; ++spins) {
      bool ok = true;
#pragma unroll
      for (int gg = 0; gg < kAoMaxKv; ++gg)
        if (gg < nkv) v[gg] = __hip_atomic_load(tp + gg * R + ct, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int gg = 0; gg < kAoMaxKv; ++gg)
        if (gg < nkv) ok = ok && static_cast<uint32_t>(v[gg] >> 32) == tag_t;
      if (ok) break;
      if (spins >= kSpinLimit) {
        if (fault != nullptr) __hip_atomic_store(fault, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    float sum = 0.f;
#pragma unroll
    for (int gg = 0; gg < kAoMaxKv; ++gg)
      if (gg < nkv) sum += __uint_as_float(static_cast<uint32_t>(v[gg]));
    bf16_t* hp = h + c * R + ct;
    const float val = (add_resid ? bf16_to_f32(*hp) : 0.f) + sum;
    if (ar.world > 1) {
      red[ct] = val;  // the tile's row values (the attention state area is free by now)
    } else {
      *hp = f32_to_bf16(val);
    }
    ao_stamp(stp, 7, ct == 0);
  }
  if (ar.world > 1) {
    // ---- a tensor-parallel rank: the all-reduce of the tile's R rows in this epilogue (car_proto.h
    // push protocol, gemv_core.h EPI_AR's exchange): every rank's reducer of tile c owns the same
    // rows, pushes its bf16 row pairs (rank 0's carry the residual) into every peer's buffer as
    // data-tagged granules and sums the peers' in rank order as they land — the bits of this
    // launch's partial + the one-shot all-reduce, without that launch. The tile's R / 2 granules are
    // R / 32 "virtual blocks" of kArGranulesPerBlock, vb = c R / 32 + i, each with its own epoch
    // word (the row-parallel GEMVs' EPI_AR blocks use the same buffer and words: every use of vb
    // advances its epoch by one on every rank, in the same stream order).
    __syncthreads();
    if (wave == 4) {
      constexpr int NG = R / 2, NVB = NG / kArGranulesPerBlock;
      static_assert(NG % kArGranulesPerBlock == 0 && NG <= kWave, "tile granules");
      const int gi = lane < NG ? lane : 0;
      const int vb = c * NVB + gi / kArGranulesPerBlock;
      const long gidx = static_cast<long>(vb) * kArGranulesPerBlock + gi % kArGranulesPerBlock;
      const uint32_t ep = __hip_atomic_load(car_ctr(ar.P.base[ar.rank]) + vb, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
      const uint32_t mine = pack_bf16x2(red[2 * gi], red[2 * gi + 1]);
      for (int base = 0; base < ar.world * NG; base += kWave) {  // push: (peer, granule); uniform trip count
        const int idx = base + lane;
        const bool live = idx < ar.world * NG;
        const int p = idx / NG, g2 = live ? idx % NG : 0;
        const uint32_t e2 = __shfl(ep, g2, 64);  // every lane takes part in both shuffles
        const uint32_t pay = __shfl(mine, g2, 64);
        const long gi2 = static_cast<long>(c * NVB + g2 / kArGranulesPerBlock) * kArGranulesPerBlock +
                         g2 % kArGranulesPerBlock;
        if (live && p != ar.rank) car_put(ar.P.base[p] + car_granule_off(e2, ar.cap, ar.rank, gi2), pay, e2);
      }
      if (lane < NG) {  // collect every peer's granule of my row pair, sum in rank order
        const long g[1] = {gidx};
        uint32_t in[kMaxRanks][1];
        car_collect<1>(ar.P, ar.rank, ar.world, ar.cap, ep, g, in);
        in[ar.rank][0] = mine;
        float lo = 0.f, hi = 0.f;
#pragma unroll
        for (int r = 0; r < kMaxRanks; ++r) {
          if (r < ar.world) {
            lo += bf16_lo(in[r][0]);
            hi += bf16_hi(in[r][0]);
          }
        }
        *reinterpret_cast<uint32_t*>(h + c * R + 2 * lane) = pack_bf16x2(lo, hi);
        if (lane % kArGranulesPerBlock == 0)
          __hip_atomic_store(car_ctr(ar.P.base[ar.rank]) + vb, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  if (ct == 0) {
    __hip_atomic_store(tctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm the tile ticket
    if (__hip_atomic_fetch_add(xctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nc - 1) {
      __hip_atomic_store(xctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(xctr + 1, static_cast<int>(tag_t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace llmc

using namespace llmc;

// > 64 KB of dynamic LDS (the per-wave V images): raise the kernel's limit once per instantiation
template <typename K>
static void ao_set_lds(K kern) {
  static bool done = false;  // one flag per instantiation
  if (!done) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    done = true;
  }
}

// Supported shape: G query heads per kv head and head dim D with G * D == 512, R = H / nc rows
// per block = 4 * RW (RW in {8, 16, 32}), chunk in {32, 64, ..., 256} keys per block, page size
// a multiple of 32. Returns 0 when (H, nh, nkv, D, nc) is supported.
extern "C" int llmc_attn_oproj_check(int H, int nh, int nkv, int D, int nc, int K_o) {
  if (nkv < 1 || nkv > kAoMaxKv || nh % nkv != 0 || nc < 1 || H % nc != 0) return -1;
  const int G = nh / nkv;
  if (G * D != 512 || K_o != nh * D) return -2;
  const int rw = H / nc / 4;
  if (rw * 4 * nc != H || (rw != 8 && rw != 16 && rw != 32)) return -3;
  if (!((G == 4 && D == 128) || (G == 8 && D == 64))) return -4;
  return 0;
}

// h += o_proj(attention). mode bit 0: issue the o_proj weights after the head ticket instead of
// right behind the K/V loads; bit 1 (with late weights): the head's merger issues its own after the
// merge; bit 2 (with late weights, 8 kv heads, G = 4, D = 128, 32-row tiles): whole o_proj rows per
// block (FR, see the kernel); bit 3 (with late weights): the weight gate — no block requests its
// weights before every block of the grid has streamed its K/V (lone engines); bit 4: the control
// waves run at a higher issue priority than the o waves (s_setprio); bit 5: no same-XCD L2 copy of
// the attention partials (the head merger always reads the write-through copy).
// fault codes: 1 a partial never arrived (merge), 2 the head output never arrived, 3 a tile partial,
// 4 a router granule (rt_*).
// stamps (nullable, diagnostics): uint64 [nkv][nc][8] s_memrealtime per block: 0 start, 1 o wave 0's
// attention done, 2 control wave 4's attention done, 3 head ticket taken, 4 head output in LDS,
// 5 o wave 0's tile partial published, 6 tile ticket taken, 7 tile reduced (reducer only); whole
// rows (mode bit 2): 6 the head merger's merge done, 7 its output stores issued (mergers only).
// Workspace (zeroed once): part f32 [2 nkv][nc][G][D/4 + 1][4] (write-through copy, then the L2 copy);
// handoff u32 [nkv][G D / 4][4];
// tile_part u64 [nc][nkv][H / nc]; ctr int32 [(nkv + nc + 2) * 16].
// Tensor-parallel ranks (h = this rank's row-parallel partial of the sum over ranks): add_resid = 0
// writes h = W_o . attention instead of adding (a rank != 0 whose all-reduce follows as its own
// launch); world > 1 runs the all-reduce in the tile reducers' epilogue (car_proto.h push protocol
// over `bases` = every rank's fused-all-reduce buffer, `cap` bytes per data parity, host status
// page `host`): h = sum over ranks, rank 0's term carrying the residual (add_resid = rank == 0).
// The whole-row form (mode bit 2) has no tile reducer: never with world > 1.
// Which form a launch of this shape and mode takes: 2 = whole rows (FR), 1 = tile partials, 0 = not
// covered. The fused MoE router (rt_wr != nullptr) needs the whole-row form.
extern "C" int llmc_attn_oproj_form(int H, int nh, int nkv, int D, int nc, int chunk, int mode, int world) {
  if (llmc_attn_oproj_check(H, nh, nkv, D, nc, nh * D) != 0) return 0;
  const bool two = chunk > kAoWaves * 32;
  const bool late = (mode & 1) != 0 || two;
  const int G = nh / nkv, rw = H / nc / 4;
  const bool fr = (mode & 4) != 0 && late && nkv == kAoMaxKv && G == 4 && D == 128 && rw == 32 && world <= 1;
  return fr ? 2 : 1;
}

// rt_* (nullable rt_wr = off; whole-row form, world 1, an engine alone on its GPU, E <= 8 experts):
// the layer's MoE decode router on the launch's output row — top rt_k ids (rt_ids int32 [k]) and
// renormalised weights (rt_w f32 [k]) as moe_router writes them; rt_part u64 [9][256] granules and
// rt_epoch int32 (one 64-B line), zeroed once. Fault code 4: the router merge gave up on a granule.
extern "C" int llmc_attn_oproj(const void* q, const void* k_cache, const void* v_cache, const void* block_table,
                               int bt_len, const void* seq_len, const void* w_o, void* h, void* attn_out, void* part,
                               void* handoff, void* tile_part, void* ctr, void* fault, int H, int nh, int nkv, int D,
                               int bs, int nblocks, int chunk, int nc, float scale, int mode, void* stamps,
                               int add_resid, const void* const* bases, void* host, int rank, int world, size_t cap,
                               const void* rt_norm, const void* rt_wr, float rt_eps, int rt_E, int rt_k, void* rt_w,
                               void* rt_ids, void* rt_part, void* rt_epoch, hipStream_t s) {
  const int K_o = nh * D;
  if (llmc_attn_oproj_check(H, nh, nkv, D, nc, K_o) != 0) return -1;
  AoRouter rt{};
  if (rt_wr != nullptr) {
    if (llmc_attn_oproj_form(H, nh, nkv, D, nc, chunk, mode, world) != 2 || rt_E < 1 || rt_E > kAoRouterMaxE ||
        rt_k < 1 || rt_k > rt_E || nc * nkv > kAoRouterMaxBlocks || rt_norm == nullptr || rt_w == nullptr ||
        rt_ids == nullptr || rt_part == nullptr || rt_epoch == nullptr)
      return -7;
    rt = AoRouter{static_cast<const bf16_t*>(rt_norm), static_cast<const bf16_t*>(rt_wr), rt_eps, rt_E, rt_k,
                  static_cast<float*>(rt_w), static_cast<int32_t*>(rt_ids), static_cast<uint64_t*>(rt_part),
                  static_cast<int*>(rt_epoch)};
  }
  CarArgs ar{};
  if (world > 1) {
    if (world > kMaxRanks || rank < 0 || rank >= world || bases == nullptr) return -1;
    const int vbs = nc * (H / nc / 2) / kArGranulesPerBlock;  // virtual blocks of the tiles' granules
    if ((H / nc / 2) % kArGranulesPerBlock != 0 || vbs > kMaxBlocks ||
        static_cast<size_t>(vbs) * kArGranulesPerBlock * 8 > cap / kMaxRanks)
      return -6;
    for (int r = 0; r < kMaxRanks; ++r) ar.P.base[r] = r < world ? static_cast<char*>(const_cast<void*>(bases[r])) : nullptr;
    ar.P.host = static_cast<uint32_t*>(host);
    ar.rank = rank;
    ar.world = world;
    ar.cap = static_cast<long>(cap);
  }
  // up to 256 keys per block: one 32-key sub-tile per wave; up to 512: two (late weights only)
  const bool two = chunk > kAoWaves * 32;
  if (chunk < 32 || chunk > kAoWaves * 64 || chunk % (two ? 64 : 32) != 0 || bs % (two ? 64 : 32) != 0 ||
      bt_len < 1 || nblocks < 1)
    return -1;
  const bool late = (mode & 1) != 0 || two;  // o_proj weights issued after the head ticket
  const int G = nh / nkv, rw = H / nc / 4;
  const bool fr = (mode & 4) != 0 && late && nkv == kAoMaxKv && G == 4 && D == 128 && rw == 32 &&
                  world <= 1;  // full rows (no tile reducer to run the all-reduce)
  const size_t lds = kAoWaves * 32 * kVRowBytes + static_cast<size_t>(kAoWaves) * G * (D + 2) * sizeof(float) +
                     (fr ? kAoMaxKv : 1) * 64 * 16 + 16 + 16 * sizeof(float);  // + flag, router rows
  dim3 grid(nc * nkv);  // block b = (c = b / nkv, g = b % nkv)
  const float sl2 = scale * 1.4426950408889634f;
#define LLMC_AO_K(KERN)                                                                                          \
  do {                                                                                                            \
    ao_set_lds(KERN);                                                                                             \
    KERN<<<grid, kAoThreads, lds, s>>>(                                                                           \
      (const bf16_t*)q, (const bf16_t*)k_cache, (const bf16_t*)v_cache, (const int32_t*)block_table, bt_len,       \
      (const int32_t*)seq_len, (const bf16_t*)w_o, K_o, (bf16_t*)h, (bf16_t*)attn_out, (float*)part,               \
      (uint32_t*)handoff, (uint64_t*)tile_part, (int*)ctr, (int*)fault, nkv, bs, nblocks, chunk, sl2, (uint64_t*)stamps, \
      (mode >> 1) & 1, add_resid, ar, late ? (mode >> 3) & 1 : 0, (mode >> 4) & 1, rt, ((mode >> 5) & 1) ^ 1); \
  } while (0)
#define LLMC_AO(GG, DD, RR)                                                                                      \
  do {                                                                                                            \
    if (two) LLMC_AO_K((attn_oproj_kernel<GG, DD, RR, true, 2>));                                                 \
    else if (late) LLMC_AO_K((attn_oproj_kernel<GG, DD, RR, true, 1>));                                           \
    else LLMC_AO_K((attn_oproj_kernel<GG, DD, RR, false, 1>));                                                    \
  } while (0)
  if (fr) {
    if (two) LLMC_AO_K((attn_oproj_kernel<4, 128, 32, true, 2, kAoMaxKv>));
    else LLMC_AO_K((attn_oproj_kernel<4, 128, 32, true, 1, kAoMaxKv>));
  } else if (G == 4 && D == 128) {
    if (rw == 8) LLMC_AO(4, 128, 8);
    else if (rw == 16) LLMC_AO(4, 128, 16);
    else LLMC_AO(4, 128, 32);
  } else {
    if (rw == 8) LLMC_AO(8, 64, 8);
    else if (rw == 16) LLMC_AO(8, 64, 16);
    else LLMC_AO(8, 64, 32);
  }
#undef LLMC_AO
#undef LLMC_AO_K
  return static_cast<int>(hipGetLastError());
}
