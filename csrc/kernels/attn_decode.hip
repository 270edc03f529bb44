// K5: paged decode attention with the GQA group on the matrix cores (one query token per
// sequence), ONE launch per step in both of its forms (host: llmc_attn_decode).
//
// Shared sub-tile step (a wave and 32 keys), mfma_f32_16x16x32_bf16:
//   S^T[key][h] = K . Q^T     A = K (16 keys x 32 dims: one 16-B global load per lane, no LDS),
//                             B = Q^T (32 dims x 16 heads; the G real heads, rest zero) in VGPRs.
//                             C puts head h = lane & 15 on the lane and 4 keys per 16x16 tile in
//                             registers -> per head, 8 of the 32 keys are lane-local and the
//                             row max / row sum need only 2 xor-shuffles (offsets 16, 32).
//   O^T[d][h] += V^T . P^T    B = P^T straight from the S^T accumulators (cvt to bf16; the
//                             k-order is permuted to match, guide §3 "accumulator tile as the next
//                             MFMA's operand"); A = V^T via ds_read_b64_tr_b16 (T10) from a per-wave
//                             LDS image of the 32 V rows, chunk-swizzled c ^ ((row & 7) << 1) so a
//                             half-wave's 8 rows x 32 B hit 64 distinct banks. O^T keeps the head on
//                             the lane, so the online-softmax rescale uses lane-local alpha.
//
// FUSED form (short contexts, <= 4k keys: responders): a block = 4 waves = one kv head x a FIXED
// 128- or 256-key chunk. The chunk does not depend on L, so a wave's page id (its 32/64 keys share
// a page), the length, the merge epoch and Q are loaded together in ONE round trip, then K/V.
// SPLIT form (long contexts: the judge): a block = 8 waves (4 without GQA) = one kv head x one balanced key range
// (the L keys split evenly, in 32-key units, over min(grid_chunks, L / min_chunk) blocks:
// common.h decode_nsplit / decode_range), so a graph captured for a bucket keeps every block
// equally busy whatever the actual L; the block's page ids are staged in LDS once; 8 waves put
// 2 x 16 KB of K/V per wave in flight (the 4-wave form of round 1 left the HBM queue half empty
// and needed a second, reduce launch).
//
// Cross-block merge, both forms, in the same launch, with no fence and no drain: every chunk block
// publishes its normalised partial (O/l per dim in bf16, lambda = m + log2 l per head in f32) as
// 8-byte {value, tag} granules (two per 16-B write-through store; MI355X_MICROARCH.md
// § visibility R2: the data IS the flag) and takes a ticket; the LAST arriver merges every
// partial with an online log-sum-exp, re-polling any granule whose tag is not yet this launch's
// (a store still in flight from a block that has already arrived — never a block that is not yet
// running, so nothing waits on scheduling and no CU is held while co-located engines need it;
// polling mergers that waited on unscheduled producers cost the 3-engine bench 8-20 %). The tag is
// a per-(row, kv head) epoch in device memory the merger advances (tag = epoch + 1: never 0,
// never reused), so a granule left by any earlier launch can never match. Spins are bounded.
#include "common.h"

namespace llmc {

typedef __attribute__((ext_vector_type(4))) short s16x4m;
typedef __attribute__((address_space(3))) s16x4m lds_s16x4m;

constexpr float kNegInfM = -1e30f;
constexpr int kVRowBytes = 256;              // LDS pitch of one V row (D <= 128)
constexpr unsigned kSpinLimit = 1u << 22;    // polls before a merger gives up (never in practice)

__device__ __forceinline__ int vswz(int row, int chunk) { return row * kVRowBytes + ((chunk ^ ((row & 7) << 1)) << 4); }

// Per-wave attention state over 32-key sub-tiles (head h = lane & 15 of the wave's kv head).
template <int G, int D>
struct SubTile {
  static constexpr int KS = D / 32;  // dim slabs for Q.K
  static constexpr int DT = D / 16;  // 16-dim tiles of O^T
  static constexpr int VCH = D / 8;  // 16-B chunks per V row
  static constexpr int NV = (32 * VCH + 63) / 64;  // 16-B V chunks per lane per sub-tile

  bf16x8 qf[KS];
  f32x4 acc[DT];
  float m_run, l_run;

  __device__ __forceinline__ void init(const bf16_t* qrow_kvh, int lane) {
    const int h = lane & 15, g4 = lane >> 4;
    const bool real = h < G;
    const bf16_t* qrow = qrow_kvh + (real ? h : 0) * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g4);
      qf[ks] = real ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run = kNegInfM;
    l_run = 0.f;
  }

  // K (A operand, registers) and V (staged for LDS) loads of keys [kbase, kbase + 32), clamped
  // to `end`; row(key) -> the key's K (or V) row.
  template <typename RowFn>
  __device__ __forceinline__ void issue(int kbase, int end, int lane, RowFn row, const bf16_t* kc, const bf16_t* vc,
                                        bf16x8 (&kf)[2][KS], u32x4 (&vst)[NV]) {
    const int h = lane & 15, g4 = lane >> 4;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      int key = kbase + kt * 16 + h;
      key = key < end ? key : end - 1;
      const bf16_t* kr = row(kc, key);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[kt][ks] = *reinterpret_cast<const bf16x8*>(kr + ks * 32 + 8 * g4);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int flat = u * 64 + lane;
      const int r = flat / VCH, ch = flat % VCH;
      if (r < 32) {
        int key = kbase + r;
        key = key < end ? key : end - 1;
        vst[u] = *reinterpret_cast<const u32x4*>(row(vc, key) + ch * 8);
      }
    }
  }

  __device__ __forceinline__ void compute(int kbase, int end, int lane, char* vbuf, float scale_log2,
                                          bf16x8 (&kf)[2][KS], u32x4 (&vst)[NV]) {
    const int g4 = lane >> 4;
    // ---- S^T = K . Q^T ----
    f32x4 s[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[kt][ks], qf[ks], s[kt], 0, 0, 0);
    }
    // V rows -> LDS (swizzled), visible to this wave's tr reads after lgkmcnt(0)
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int flat = u * 64 + lane;
      const int r = flat / VCH, ch = flat % VCH;
      if (r < 32) *reinterpret_cast<u32x4*>(vbuf + vswz(r, ch)) = vst[u];
    }
    // ---- online softmax over this sub-tile (keys 4*g4+i and 16+4*g4+i of the lane's head) ----
    float mx = kNegInfM;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kbase + kt * 16 + 4 * g4 + i;
        const float v = key < end ? s[kt][i] * scale_log2 : kNegInfM;
        s[kt][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = exp2f(m_run - m_new);
    float rs = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = s[kt][i] <= -1e29f ? 0.f : exp2f(s[kt][i] - m_new);
        s[kt][i] = p;
        rs += p;
      }
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    l_run = l_run * alpha + rs;
    m_run = m_new;
    // P^T fragment: k = 8*g4 + j  <->  key 4*g4 + j (j < 4), 16 + 4*g4 + (j - 4) (j >= 4)
    bf16x8 pf;
    {
      u32x4 pk;
      pk[0] = pack_bf16x2(s[0][0], s[0][1]);
      pk[1] = pack_bf16x2(s[0][2], s[0][3]);
      pk[2] = pack_bf16x2(s[1][0], s[1][1]);
      pk[3] = pack_bf16x2(s[1][2], s[1][3]);
      pf = __builtin_bit_cast(bf16x8, pk);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's V rows are in LDS
    // ---- O^T += V^T . P^T ; A = V^T rows d = dt*16 + (lane & 15), keys via two tr reads ----
    const int qq = (lane & 15) >> 2, p4 = lane & 3;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int ch = 2 * dt + (p4 >> 1);
      const int sub = (p4 & 1) * 8;
      const s16x4m lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4m*)(vbuf + vswz(4 * g4 + qq, ch) + sub));
      const s16x4m hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4m*)(vbuf + vswz(16 + 4 * g4 + qq, ch) + sub));
      bf16x8 a;
      a[0] = lo[0]; a[1] = lo[1]; a[2] = lo[2]; a[3] = lo[3];
      a[4] = hi[0]; a[5] = hi[1]; a[6] = hi[2]; a[7] = hi[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[dt][i] *= alpha;
      acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pf, acc[dt], 0, 0, 0);
    }
    // the next sub-tile overwrites vbuf: make sure every tr read of this one has returned
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  // wave state -> red[wave][h][D + 2] (O^T column h, then m, l; only lanes with h < G)
  __device__ __forceinline__ void to_lds(float* red, int wave, int lane) const {
    const int h = lane & 15, g4 = lane >> 4;
    if (h < G) {
      float* r = red + (wave * G + h) * (D + 2);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) r[dt * 16 + 4 * g4 + i] = acc[dt][i];
      if (g4 == 0) {
        r[D] = m_run;
        r[D + 1] = l_run;
      }
    }
  }
};

// Merge the NW waves' states of head hh at dim d (log2 domain): o (unnormalised), m, l.
template <int G, int D, int NW>
__device__ __forceinline__ void merge_waves(const float* red, int hh, int d, float& o, float& m, float& l) {
  constexpr int stride = D + 2;
  float mx = kNegInfM;
#pragma unroll
  for (int w = 0; w < NW; ++w) mx = fmaxf(mx, red[(w * G + hh) * stride + D]);
  float ls = 0.f, oo = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const float* r = red + (w * G + hh) * stride;
    const float sc = exp2f(r[D] - mx);
    ls += r[D + 1] * sc;
    oo += r[d] * sc;
  }
  o = oo;
  m = mx;
  l = ls;
}

// The block's own result when it is the sequence's only chunk.
template <int G, int D, int NW>
__device__ __forceinline__ void store_direct(const float* red, bf16_t* out_row, int tid) {
  for (int idx = tid; idx < G * D; idx += NW * 64) {
    const int hh = idx / D, d = idx % D;
    float o, m, l;
    merge_waves<G, D, NW>(red, hh, d, o, m, l);
    out_row[hh * D + d] = f32_to_bf16(o / l);
  }
}

// ---- partial granules -------------------------------------------------------------------------
// Per (row, kv head) slab: [max_chunks][G][D/4 + 1] 16-B units. Unit u < D/4 = {bf16x2 O[4u..4u+1]/l,
// tag, bf16x2 O[4u+2..4u+3]/l, tag}; unit D/4 = {lambda, tag, lambda, tag}. Every 8-B half is ONE
// granule of one write-through (sc1) store (MI355X_MICROARCH.md § visibility R2: 16-B sc1 halves
// untorn), so a reader needs no ordering: it checks every tag. Normalised partials in bf16 (as the
// output; the weights and lambda stay f32).
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t rsrc, int byte_off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, byte_off, 0, 16);
}
__device__ __forceinline__ u32x4 ld16_sc1(__amdgpu_buffer_rsrc_t rsrc, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc, byte_off, 0, 16);
}
// lambda granule: an 8-B relaxed agent-scope atomic load (global_load_dwordx2 sc1). Being an
// ordered load it also keeps the compiler from hoisting the O-unit buffer loads out of a re-poll
// (a loop with no ordered access looks loop-invariant to it).
__device__ __forceinline__ u32x2 ld8_atomic(const char* base, int byte_off) {
  const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(base + byte_off), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return u32x2{static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32)};
}

template <int G, int D, int NW>
__device__ __forceinline__ void publish_partial(const float* red, __amdgpu_buffer_rsrc_t rsrc, int c, uint32_t tag,
                                                int tid) {
  constexpr int HQ = D / 4, RU = HQ + 1;
  for (int p = tid; p < G * HQ; p += NW * 64) {
    const int g = p / HQ, u = p % HQ;
    float o[4], m, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) merge_waves<G, D, NW>(red, g, 4 * u + e, o[e], m, l);
    const float inv = 1.f / l;
    const int row = (c * G + g) * RU;
    st16_sc1(rsrc, (row + u) * 16, u32x4{pack_bf16x2(o[0] * inv, o[1] * inv), tag, pack_bf16x2(o[2] * inv, o[3] * inv), tag});
    if (u == 0) {
      const uint32_t lam = __float_as_uint(m + __log2f(l));
      st16_sc1(rsrc, (row + HQ) * 16, u32x4{lam, tag, lam, tag});
    }
  }
}

// Merge the partial rows [r0, r0 + n) of a granule slab: thread = (output quad, row group), up to 8
// rows' {O quad, lambda} loads in flight per thread, re-polled until every tag matches (a
// straggler is a store already issued by a block that has arrived: no wait on any block that is
// not running), folded with an online log-sum-exp; row groups meet in LDS. On return threads
// tid < G * D / 4 hold their quad's (M, S) in ms[0..1] and the unnormalised sums in acc.
template <int G, int D, int NT>
__device__ __forceinline__ void merge_rows(__amdgpu_buffer_rsrc_t rsrc, const char* base, int r0, int n, uint32_t tag,
                                           f32x4* scratch, int tid, f32x4& ms, f32x4& acc, int* fault) {
  constexpr int HQ = D / 4, RU = HQ + 1, Q = G * HQ;
  static_assert(Q <= NT, "one pass");
  const int ngr = max(1, min(NT / Q, n));
  const int gr = tid / Q;
  float M = kNegInfM, S = 0.f, a[4] = {0.f, 0.f, 0.f, 0.f};
  if (gr < ngr) {
    const int g = (tid % Q) / HQ, u = (tid % Q) % HQ;
    for (int c0 = gr; c0 < n; c0 += 8 * ngr) {
      u32x4 ov[8];
      u32x2 lv[8];
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int cc = r0 + min(c0 + j * ngr, n - 1);  // clamped: every load in flight, masked below
          const int row = (cc * G + g) * RU;
          ov[j] = ld16_sc1(rsrc, (row + u) * 16);
          lv[j] = ld8_atomic(base, (row + HQ) * 16);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (c0 + j * ngr < n) ok = ok && ov[j][1] == tag && ov[j][3] == tag && lv[j][1] == tag;
        if (__all(ok)) break;
        if (spins >= kSpinLimit) {
          // gave up on a granule that never arrived: the output is wrong, so say so (the
          // engine reads this word after its sync points and fails the request)
          if (fault != nullptr && (tid & 63) == 0) __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (c0 + j * ngr < n) {
          const float lam = __uint_as_float(lv[j][0]);
          const float mn = fmaxf(M, lam);
          const float so = exp2f(M - mn), sn = exp2f(lam - mn);
          S = S * so + sn;
          a[0] = a[0] * so + bf16_lo(ov[j][0]) * sn;
          a[1] = a[1] * so + bf16_hi(ov[j][0]) * sn;
          a[2] = a[2] * so + bf16_lo(ov[j][2]) * sn;
          a[3] = a[3] * so + bf16_hi(ov[j][2]) * sn;
          M = mn;
        }
      }
    }
  }
  scratch[2 * tid] = f32x4{M, S, 0.f, 0.f};
  scratch[2 * tid + 1] = f32x4{a[0], a[1], a[2], a[3]};
  __syncthreads();
  if (tid < Q) {
    ms = scratch[2 * tid];
    acc = scratch[2 * tid + 1];
    for (int k = 1; k < ngr; ++k) {
      const f32x4 ms2 = scratch[2 * (tid + k * Q)], acc2 = scratch[2 * (tid + k * Q) + 1];
      const float mn = fmaxf(ms[0], ms2[0]);
      const float so = exp2f(ms[0] - mn), sn = exp2f(ms2[0] - mn);
      ms = f32x4{mn, ms[1] * so + ms2[1] * sn, 0.f, 0.f};
      acc = acc * so + acc2 * sn;
    }
  }
  __syncthreads();  // scratch is reused by the caller's next merge
}

// Publish this chunk's partial and take a ticket in its GROUP of `gsize` consecutive chunks; the
// group's last arriver merges the group. With one group that is the output; otherwise the group
// result is published as one more granule row (slab row max_chunks + group) and the last group
// merger merges those (two levels: a 256-block split merges 16 rows twice instead of 256 rows in
// one block). The last merger re-arms the tickets it took and advances the epoch (every block of
// this launch read the epoch before it arrived). ctr = {top ticket, epoch, group tickets...};
// `flag` is one LDS word. Every block but the last returns inside.
template <int G, int D, int NW>
__device__ __forceinline__ void publish_and_merge(const float* red, float* part, int* ctr, int b, int nkv, int kvh,
                                                  int c, int nchunks, int gsize, int max_chunks, int max_groups,
                                                  uint32_t tag, bf16_t* out_row, char* smem, int* flag, int tid,
                                                  int* fault) {
  constexpr int HQ = D / 4, RU = HQ + 1, Q = G * HQ;
  const int rows = max_chunks + max_groups;
  float* slab = part + (static_cast<int64_t>(b) * nkv + kvh) * rows * G * RU * 4;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(slab, 0, rows * G * RU * 16, 0x00020000);
  const char* base = reinterpret_cast<const char*>(slab);
  f32x4* scratch = reinterpret_cast<f32x4*>(smem);
  publish_partial<G, D, NW>(red, rsrc, c, tag, tid);
  const int grp = c / gsize, ngroups = (nchunks + gsize - 1) / gsize;
  const int g0 = grp * gsize, gn = min(gsize, nchunks - g0);
  int* gctr = ngroups == 1 ? ctr : ctr + 2 + grp;
  __syncthreads();  // every wave's stores are issued (not drained: the merger checks tags)
  if (tid == 0) *flag = __hip_atomic_fetch_add(gctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gn - 1;
  __syncthreads();
  if (*flag == 0) return;
  f32x4 ms, acc;
  merge_rows<G, D, NW * 64>(rsrc, base, g0, gn, tag, scratch, tid, ms, acc, fault);
  if (ngroups > 1) {
    // publish the group result as a granule row, then the top-level ticket
    if (tid < Q) {
      const int g = tid / HQ, u = tid % HQ;
      const float inv = 1.f / ms[1];
      const int row = ((max_chunks + grp) * G + g) * RU;
      st16_sc1(rsrc, (row + u) * 16,
               u32x4{pack_bf16x2(acc[0] * inv, acc[1] * inv), tag, pack_bf16x2(acc[2] * inv, acc[3] * inv), tag});
      if (u == 0) {
        const uint32_t lam = __float_as_uint(ms[0] + __log2f(ms[1]));
        st16_sc1(rsrc, (row + HQ) * 16, u32x4{lam, tag, lam, tag});
      }
    }
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store(gctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm the group ticket
      *flag = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
    }
    __syncthreads();
    if (*flag == 0) return;
    merge_rows<G, D, NW * 64>(rsrc, base, max_chunks, ngroups, tag, scratch, tid, ms, acc, fault);
  }
  if (tid < Q) {
    const int g = tid / HQ, u = tid % HQ;
    const float inv = 1.f / ms[1];
    *reinterpret_cast<u32x2*>(out_row + g * D + 4 * u) =
        u32x2{pack_bf16x2(acc[0] * inv, acc[1] * inv), pack_bf16x2(acc[2] * inv, acc[3] * inv)};
  }
  if (tid == 0) {
    __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);                          // re-arm
    __hip_atomic_store(ctr + 1, static_cast<int>(tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // epoch
  }
}

// ---------------------------------------------------------------------------------------------
template <int G, int D, int NW>
__global__ __launch_bounds__(NW * 64) void attn_decode_split_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters, bf16_t* __restrict__ out,
    int out_stride, int nkv, int bs, int nblocks, int min_chunk, int max_chunks, int gsize, int max_groups,
    float scale_log2, int* __restrict__ fault) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  using ST = SubTile<G, D>;
  constexpr int NT = NW * 64;
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  int* ctr = counters + (b * nkv + kvh) * (2 + max_groups);  // {ticket, epoch, group tickets}
  const uint32_t tag = static_cast<uint32_t>(__hip_atomic_load(ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  const int L = seq_lens[b];
  const int nchunks = decode_nsplit(L, gridDim.x, -min_chunk);
  if (c >= nchunks) return;
  int start, end;
  decode_range(L, nchunks, c, -min_chunk, start, end);

  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* vbuf = smem + wave * 32 * kVRowBytes;  // per-wave V image [32][256 B]
  float* red = reinterpret_cast<float*>(smem + NW * 32 * kVRowBytes);
  int* pages = reinterpret_cast<int*>(red + NW * G * (D + 2));  // this block's page ids

  ST st;
  st.init(q + static_cast<int64_t>(b) * q_stride + kvh * G * D, lane);
  // stage the block's page ids once (no dependent block-table load per key)
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int p0 = start / bs;
  const int npages = (end - 1) / bs - p0 + 1;
  // page ids clamped into the cache: a corrupt block table reads a wrong page, never a wild address
  for (int i = tid; i < npages; i += NT) pages[i] = min(max(bt[min(p0 + i, bt_stride - 1)], 0), nblocks - 1);
  __syncthreads();
  const int64_t head_stride = static_cast<int64_t>(bs) * D;
  auto row = [&](const bf16_t* cache, int key) {
    const int64_t page = pages[key / bs - p0];
    return cache + (page * nkv + kvh) * head_stride + static_cast<int64_t>(key % bs) * D;
  };

  const int per_wave = (((end - start + NW - 1) / NW) + 31) & ~31;  // 32-key sub-tiles per wave
  const int wbase = start + wave * per_wave;
  bf16x8 kfA[2][ST::KS], kfB[2][ST::KS];
  u32x4 vsA[ST::NV], vsB[ST::NV];
  auto valid = [&](int k) { return k - wbase < per_wave && k < end; };  // wave-uniform
  // two named register sets, hand-unrolled (no runtime-indexed register arrays, guide rule 20):
  // the next sub-tile's loads are in flight while the current one computes
  if (valid(wbase)) st.issue(wbase, end, lane, row, k_cache, v_cache, kfA, vsA);
  for (int k0 = wbase;; k0 += 64) {
    if (!valid(k0)) break;
    if (valid(k0 + 32)) st.issue(k0 + 32, end, lane, row, k_cache, v_cache, kfB, vsB);
    st.compute(k0, end, lane, vbuf, scale_log2, kfA, vsA);
    if (!valid(k0 + 32)) break;
    if (valid(k0 + 64)) st.issue(k0 + 64, end, lane, row, k_cache, v_cache, kfA, vsA);
    st.compute(k0 + 32, end, lane, vbuf, scale_log2, kfB, vsB);
  }
  st.to_lds(red, wave, lane);
  __syncthreads();
  bf16_t* out_row = out + static_cast<int64_t>(b) * out_stride + kvh * G * D;
  if (nchunks == 1) {
    store_direct<G, D, NW>(red, out_row, tid);
    return;
  }
  publish_and_merge<G, D, NW>(red, part, ctr, b, nkv, kvh, c, nchunks, gsize, max_chunks, max_groups, tag, out_row, smem,
                              reinterpret_cast<int*>(pages), tid, fault);
}

// ---------------------------------------------------------------------------------------------
template <int G, int D>
__global__ __launch_bounds__(256) void attn_decode_fused_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters,
    bf16_t* __restrict__ out, int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize,
    int max_groups, float scale_log2, int* __restrict__ fault) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  using ST = SubTile<G, D>;
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  const int per_wave = chunk / 4;  // keys per wave (32 or 64): inside one page (host-checked)
  // ONE round trip for everything that does not depend on the sequence length: the length, this
  // wave's page id (wave-uniform: scalar cache), the merge epoch and Q (vector)
  const int key0 = c * chunk + wave * per_wave;
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int pidx = __builtin_amdgcn_readfirstlane(min(key0 / bs, bt_stride - 1));
  const int page = min(max(ld_scalar(bt + pidx), 0), nblocks - 1);  // clamped into the cache
  const int L = ld_scalar(seq_lens + b);
  int* ctr = counters + (b * nkv + kvh) * (2 + max_groups);  // {ticket, epoch, group tickets}
  const uint32_t tag = static_cast<uint32_t>(__hip_atomic_load(ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
  ST st;
  st.init(q + static_cast<int64_t>(b) * q_stride + kvh * G * D, lane);
  if (c * chunk >= L) return;  // block-uniform
  const int nchunks = (L + chunk - 1) / chunk;
  const int end = min(L, key0 + per_wave);

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* vbuf = smem + wave * 32 * kVRowBytes;
  float* red = reinterpret_cast<float*>(smem + 4 * 32 * kVRowBytes);
  if (key0 < L) {  // wave-uniform
    const int64_t base = (static_cast<int64_t>(page) * nkv + kvh) * bs * D;
    auto row = [&](const bf16_t* cache, int key) { return cache + base + static_cast<int64_t>(key % bs) * D; };
    bf16x8 kfA[2][ST::KS], kfB[2][ST::KS];
    u32x4 vsA[ST::NV], vsB[ST::NV];
    st.issue(key0, end, lane, row, k_cache, v_cache, kfA, vsA);
    if (key0 + 32 < end) st.issue(key0 + 32, end, lane, row, k_cache, v_cache, kfB, vsB);
    st.compute(key0, end, lane, vbuf, scale_log2, kfA, vsA);
    if (key0 + 32 < end) st.compute(key0 + 32, end, lane, vbuf, scale_log2, kfB, vsB);
  }
  st.to_lds(red, wave, lane);
  __syncthreads();
  bf16_t* out_row = out + static_cast<int64_t>(b) * out_stride + kvh * G * D;
  if (nchunks == 1) {
    store_direct<G, D, 4>(red, out_row, tid);
    return;
  }
  publish_and_merge<G, D, 4>(red, part, ctr, b, nkv, kvh, c, nchunks, gsize, max_chunks, max_groups, tag, out_row, smem,
                             reinterpret_cast<int*>(red + 4 * G * (D + 2)), tid, fault);
}

// Split blocks: 8 waves when a block's balanced range at the table's full length is >= 512 keys
// (2 x 16 KB of K/V in flight per wave), 4 otherwise (wide TP grids: a TP=8 rank's one kv head
// over 256 blocks has ~130 keys per block) and always without GQA (G = 1: Phi-3's 32 kv heads
// already give 512 blocks, and 8-wave blocks at 212 VGPRs would halve the blocks resident per CU).
template <int G, int D, int NW>
static int launch_split_nw(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                           const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out,
                           int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize,
                           int max_groups, int max_chunk_keys, float scale, int* fault) {
  const size_t lds = NW * 32 * kVRowBytes + static_cast<size_t>(NW) * G * (D + 2) * sizeof(float) +
                     static_cast<size_t>((max_chunk_keys + bs - 1) / bs + 2) * sizeof(int);
  if (lds > 160 * 1024) return -4;
  auto kern = attn_decode_split_kernel<G, D, NW>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr_set = true;
  }
  kern<<<grid, NW * 64, lds, s>>>((const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc,
                                  (const int32_t*)bt, bt_stride, (const int32_t*)sl, (float*)part, (int*)ctr,
                                  (bf16_t*)out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups,
                                  scale * 1.4426950408889634f, fault);
  return static_cast<int>(hipGetLastError());
}

template <int G, int D>
static int launch_split(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                        const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out, int out_stride,
                        int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize, int max_groups,
                        float scale, int* fault) {
  // page-id staging sized for the largest balanced range any sequence of this table can get
  const int grid_chunks = static_cast<int>(grid.x);
  const int units = (bt_stride * bs + 31) / 32;
  const int bal = 32 * ((units + grid_chunks - 1) / grid_chunks) + 32;
  const int max_chunk = bal > 2 * chunk ? bal : 2 * chunk;
  // a minimum block range of >= 512 keys (the length-only split of batching engines) always takes
  // 8 waves, so a row's per-wave key partition never depends on the bucket its batch selected
  if (G > 1 && (bal >= 512 || chunk >= 512))
    return launch_split_nw<G, D, 8>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, nkv,
                                    bs, nblocks, chunk, max_chunks, gsize, max_groups, max_chunk, scale, fault);
  return launch_split_nw<G, D, 4>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, nkv, bs,
                                  nblocks, chunk, max_chunks, gsize, max_groups, max_chunk, scale, fault);
}

template <int G, int D>
static int launch_fused(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                        const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out, int out_stride,
                        int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize, int max_groups,
                        float scale, int* fault) {
  const size_t lds = 4 * 32 * kVRowBytes + static_cast<size_t>(4) * G * (D + 2) * sizeof(float) + 16;  // + flag
  if (lds > 64 * 1024) return -4;
  attn_decode_fused_kernel<G, D><<<grid, 256, lds, s>>>(
      (const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, (const int32_t*)bt, bt_stride,
      (const int32_t*)sl, (float*)part, (int*)ctr, (bf16_t*)out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize,
      max_groups, scale * 1.4426950408889634f, fault);
  return static_cast<int>(hipGetLastError());
}

template <int G>
static int launch_g(bool fused, int D, dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc,
                    const void* vc, const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out,
                    int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks, int gsize,
                    int max_groups, float scale, int* fault) {
#define LLMC_ATTN_D(DD)                                                                                          \
  case DD:                                                                                                       \
    return fused ? launch_fused<G, DD>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, \
                                       nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, fault)     \
                 : launch_split<G, DD>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, \
                                       nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, fault);
  switch (D) {
    LLMC_ATTN_D(64)
    LLMC_ATTN_D(96)
    LLMC_ATTN_D(128)
    default: return -2;
  }
#undef LLMC_ATTN_D
}

}  // namespace llmc

using namespace llmc;

// Attention of one decode step for rows 0..B-1, one launch.
// part: f32 [B, nkv, max_chunks + max_groups, G, D + 4] partial granules (zeroed once); counters:
// int32 [B, nkv, 2 + max_groups] {top ticket, epoch, group tickets} (zeroed once; the kernel re-arms
// the tickets and advances the epoch); max_groups = attn_decode_groups(max_chunks).
// fused = 1 (short contexts): grid_chunks fixed chunk-key blocks (chunk 128 or 256; bs % (chunk/4) == 0).
// fused = 0 (long contexts): balanced split over <= grid_chunks blocks of >= chunk keys (multiple of 128).
// Chunk partials are merged in one level up to kAttnOneLevel chunks, else in groups of kAttnGroup.
// fault (nullable int32): set to 1 when a merger gave up waiting for a partial (bounded spin): the
// step's attention output is then invalid and the caller must fail the request.
constexpr int kAttnOneLevel = 32, kAttnGroup = 16;  // one-level merges of 64 rows measured 1.3-1.5x slower

extern "C" int llmc_attn_decode_groups(int max_chunks) {
  return max_chunks > kAttnOneLevel ? (max_chunks + kAttnGroup - 1) / kAttnGroup : 0;
}

extern "C" int llmc_attn_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                const void* block_tables, int bt_stride, const void* seq_lens, void* part,
                                void* counters, void* out, int out_stride, int B, int nh, int nkv, int D, int bs,
                                int nblocks, int chunk, int grid_chunks, int max_chunks, float scale, int fused,
                                void* fault, hipStream_t s) {
  if (nh % nkv != 0 || grid_chunks > max_chunks || grid_chunks < 1 || nblocks < 1 || counters == nullptr ||
      bt_stride < 1)
    return -1;
  if (fused ? ((chunk != 128 && chunk != 256) || bs % (chunk / 4) != 0) : (chunk % 128 != 0)) return -1;
  const int G = nh / nkv;
  const int max_groups = llmc_attn_decode_groups(max_chunks);
  const int gsize = grid_chunks > kAttnOneLevel ? kAttnGroup : grid_chunks;
  if (static_cast<int64_t>(max_chunks + max_groups) * G * (D / 4 + 1) * 16 >= (1ll << 31)) return -4;
  dim3 grid(grid_chunks, nkv, B);
  const bool f = fused != 0;
  switch (G) {
    case 1: return launch_g<1>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    case 2: return launch_g<2>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    case 4: return launch_g<4>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    case 8: return launch_g<8>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, gsize, max_groups, scale, static_cast<int*>(fault));
    default: return -3;
  }
}
