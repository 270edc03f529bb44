// Decode-attention building blocks shared by attn_decode.hip (K5, its own launch) and
// attn_oproj.hip (the same attention feeding the o_proj tile in one launch): the MFMA sub-tile
// step, the wave/block merges and the in-launch partial publish + last-arriver merge.
// Design notes: attn_decode.hip's header.
#pragma once
#include "common.h"

namespace llmc {

typedef __attribute__((ext_vector_type(4))) short s16x4m;
typedef __attribute__((address_space(3))) s16x4m lds_s16x4m;

constexpr float kNegInfM = -1e30f;
constexpr int kVRowBytes = 256;              // LDS pitch of one V row (D <= 128)
constexpr unsigned kSpinLimit = 1u << 22;    // polls before a merger gives up (never in practice)
// Decode-attention counters: every word (top ticket, epoch, group tickets) of a (row, kv head) on
// its own 128-B line. Returning atomics on one line serialise (MI355X_MICROARCH.md dequeue / fanin:
// ~11-13 ns each), and with the words of all kv heads packed in one line every block of the grid
// (256-512) queued its ticket behind the others'.
constexpr int kCtrPitch = 32;  // int32 words per counter line
// Chunk partials are merged in one level up to kAttnOneLevel chunks, else in groups of kAttnGroup
// (one-level merges of 64 rows measured 1.3-1.5x slower)
constexpr int kAttnOneLevel = 32, kAttnGroup = 16;

__device__ __forceinline__ int vswz(int row, int chunk) { return row * kVRowBytes + ((chunk ^ ((row & 7) << 1)) << 4); }

struct PlainLd16 {
  __device__ __forceinline__ u32x4 operator()(const bf16_t* p) const { return *reinterpret_cast<const u32x4*>(p); }
};

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

  // ld(p) loads the 16 B at p (plain by default; a caller whose operands are produced inside its
  // own launch passes write-through-coherent sc1 loads)
  template <typename Ld = PlainLd16>
  __device__ __forceinline__ void init(const bf16_t* qrow_kvh, int lane, Ld ld = Ld{}) {
    // columns h >= G of the 16-head MFMA tile carry a copy of head 0 (finite; every column's
    // scores, softmax state and output stay in that column and to_lds drops them). No select on
    // the loaded value: a select would make hipcc wait for Q here, before the K/V loads issue.
    const int h = lane & 15, g4 = lane >> 4;
    const bf16_t* qrow = qrow_kvh + (h < G ? h : 0) * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, ld(qrow + ks * 32 + 8 * g4));
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run = kNegInfM;
    l_run = 0.f;
  }

  // K (A operand, registers) and V (staged for LDS) loads of keys [kbase, kbase + 32), clamped
  // to `end`; row(key) -> the key's K (or V) row.
  template <typename RowFn, typename LdK = PlainLd16, typename LdV = PlainLd16>
  __device__ __forceinline__ void issue(int kbase, int end, int lane, RowFn row, const bf16_t* kc, const bf16_t* vc,
                                        bf16x8 (&kf)[2][KS], u32x4 (&vst)[NV], LdK ldk = LdK{}, LdV ldv = LdV{}) {
    const int h = lane & 15, g4 = lane >> 4;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      int key = kbase + kt * 16 + h;
      key = key < end ? key : end - 1;
      const bf16_t* kr = row(kc, key);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[kt][ks] = __builtin_bit_cast(bf16x8, ldk(kr + ks * 32 + 8 * g4));
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int flat = u * 64 + lane;
      const int r = flat / VCH, ch = flat % VCH;
      if (r < 32) {
        int key = kbase + r;
        key = key < end ? key : end - 1;
        vst[u] = ldv(row(vc, key) + ch * 8);
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
    mx = xor16_max(mx);
    mx = xor32_max(mx);
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
    rs = xor16_add(rs);
    rs = xor32_add(rs);
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
// ... written through as 4-B pairs, for a consumer in the same launch
template <int G, int D, int NW>
__device__ __forceinline__ void store_direct_sc1(const float* red, bf16_t* out_row, int tid) {
  for (int idx = tid; idx < G * D / 2; idx += NW * 64) {
    const int hh = (2 * idx) / D, d = (2 * idx) % D;
    float o0, o1, m, l;
    merge_waves<G, D, NW>(red, hh, d, o0, m, l);
    merge_waves<G, D, NW>(red, hh, d + 1, o1, m, l);
    __hip_atomic_store(reinterpret_cast<uint32_t*>(out_row + hh * D + d), pack_bf16x2(o0 / l, o1 / l), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
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
// default-policy 16-B store: the line stays in this XCD's L2 (a same-XCD reader's sc1 load hits it
// there; a reader on another XCD may see a stale line: only ever an additional copy, see
// publish_partial's `rsrc_l2`)
__device__ __forceinline__ void st16_l2(__amdgpu_buffer_rsrc_t rsrc, int byte_off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, byte_off, 0, 0);
}
// this wave's XCD (0-7): for choosing a faster same-XCD path only, never for correctness
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}
// lambda granule: an 8-B relaxed agent-scope atomic load (global_load_dwordx2 sc1). Being an
// ordered load it also keeps the compiler from hoisting the O-unit buffer loads out of a re-poll
// (a loop with no ordered access looks loop-invariant to it).
__device__ __forceinline__ u32x2 ld8_atomic(const char* base, int byte_off) {
  const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(base + byte_off), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return u32x2{static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32)};
}

// DUAL: the same granules also into a second slab (`rsrc_l2`) with default-policy stores, whose
// lines stay in this XCD's L2 — a merger that knows every producer ran on its own XCD reads that
// copy from L2 instead of the write-through copy from memory (attn_oproj.hip)
template <int G, int D, int NW, bool DUAL>
__device__ __forceinline__ void publish_partial_x(const float* red, __amdgpu_buffer_rsrc_t rsrc, int c, uint32_t tag,
                                                  int tid, __amdgpu_buffer_rsrc_t rsrc_l2) {
  constexpr int HQ = D / 4, RU = HQ + 1;
  for (int p = tid; p < G * HQ; p += NW * 64) {
    const int g = p / HQ, u = p % HQ;
    float o[4], m, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) merge_waves<G, D, NW>(red, g, 4 * u + e, o[e], m, l);
    const float inv = 1.f / l;
    const int row = (c * G + g) * RU;
    const u32x4 ov{pack_bf16x2(o[0] * inv, o[1] * inv), tag, pack_bf16x2(o[2] * inv, o[3] * inv), tag};
    if constexpr (DUAL) st16_l2(rsrc_l2, (row + u) * 16, ov);
    st16_sc1(rsrc, (row + u) * 16, ov);
    if (u == 0) {
      const uint32_t lam = __float_as_uint(m + __log2f(l));
      if constexpr (DUAL) st16_l2(rsrc_l2, (row + HQ) * 16, u32x4{lam, tag, lam, tag});
      st16_sc1(rsrc, (row + HQ) * 16, u32x4{lam, tag, lam, tag});
    }
  }
}

template <int G, int D, int NW>
__device__ __forceinline__ void publish_partial(const float* red, __amdgpu_buffer_rsrc_t rsrc, int c, uint32_t tag,
                                                int tid) {
  publish_partial_x<G, D, NW, false>(red, rsrc, c, tag, tid, rsrc);
}
template <int G, int D, int NW>
__device__ __forceinline__ void publish_partial_dual(const float* red, __amdgpu_buffer_rsrc_t rsrc,
                                                     __amdgpu_buffer_rsrc_t rsrc_l2, int c, uint32_t tag, int tid) {
  publish_partial_x<G, D, NW, true>(red, rsrc, c, tag, tid, rsrc_l2);
}

// Merge the partial rows [r0, r0 + n) of a granule slab: thread = (output quad, row group), up to
// BATCH rows' {O quad, lambda} loads in flight per thread, re-polled until every tag matches (a
// straggler is a store already issued by a block that has arrived: no wait on any block that is
// not running), folded with an online log-sum-exp; row groups meet in LDS. On return threads
// tid < G * D / 4 hold their quad's (M, S) in ms[0..1] and the unnormalised sums in acc.
// first_polls > 0: the first polls read the copy at (rsrc_first, base_first) instead (a same-XCD
// L2 copy, publish_partial's DUAL), then the write-through copy
template <int G, int D, int NT, int BATCH = 8>
__device__ __forceinline__ void merge_rows(__amdgpu_buffer_rsrc_t rsrc, const char* base, int r0, int n, uint32_t tag,
                                           f32x4* scratch, int tid, f32x4& ms, f32x4& acc, int* fault,
                                           __amdgpu_buffer_rsrc_t rsrc_first, const char* base_first,
                                           unsigned first_polls) {
  constexpr int HQ = D / 4, RU = HQ + 1, Q = G * HQ;
  static_assert(Q <= NT, "one pass");
  const int ngr = max(1, min(NT / Q, n));
  const int gr = tid / Q;
  float M = kNegInfM, S = 0.f, a[4] = {0.f, 0.f, 0.f, 0.f};
  if (gr < ngr) {
    const int g = (tid % Q) / HQ, u = (tid % Q) % HQ;
    for (int c0 = gr; c0 < n; c0 += BATCH * ngr) {
      u32x4 ov[BATCH];
      u32x2 lv[BATCH];
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
        const bool first = spins < first_polls;  // wave-uniform
        const __amdgpu_buffer_rsrc_t rs = first ? rsrc_first : rsrc;
        const char* bs = first ? base_first : base;
#pragma unroll
        for (int j = 0; j < BATCH; ++j) {
          const int cc = r0 + min(c0 + j * ngr, n - 1);  // clamped: every load in flight, masked below
          const int row = (cc * G + g) * RU;
          ov[j] = ld16_sc1(rs, (row + u) * 16);
          lv[j] = ld8_atomic(bs, (row + HQ) * 16);
        }
#pragma unroll
        for (int j = 0; j < BATCH; ++j)
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
      for (int j = 0; j < BATCH; ++j) {
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
  if (tid < NT) {  // tid >= NT: a thread of the block that only meets the barriers (attn_oproj.hip)
    scratch[2 * tid] = f32x4{M, S, 0.f, 0.f};
    scratch[2 * tid + 1] = f32x4{a[0], a[1], a[2], a[3]};
  }
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

template <int G, int D, int NT, int BATCH = 8>
__device__ __forceinline__ void merge_rows(__amdgpu_buffer_rsrc_t rsrc, const char* base, int r0, int n, uint32_t tag,
                                           f32x4* scratch, int tid, f32x4& ms, f32x4& acc, int* fault) {
  merge_rows<G, D, NT, BATCH>(rsrc, base, r0, n, tag, scratch, tid, ms, acc, fault, rsrc, base, 0u);
}

// Publish this chunk's partial and take a ticket in its GROUP (returns true in the block that wrote
// the output; SC1OUT: the output is written through for a consumer in the same launch) of `gsize` consecutive chunks; the
// group's last arriver merges the group. With one group that is the output; otherwise the group
// result is published as one more granule row (slab row max_chunks + group) and the last group
// merger merges those (two levels: a 256-block split merges 16 rows twice instead of 256 rows in
// one block). The last merger re-arms the tickets it took and advances the epoch (every block of
// this launch read the epoch before it arrived). ctr = {top ticket, epoch, group tickets...}, one
// kCtrPitch line each;
// `flag` is one LDS word. Every block but the last returns inside.
template <int G, int D, int NW, bool SC1OUT = false>
__device__ __forceinline__ bool publish_and_merge(const float* red, float* part, int* ctr, int b, int nkv, int kvh,
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
  int* gctr = ngroups == 1 ? ctr : ctr + (2 + grp) * kCtrPitch;
  __syncthreads();  // every wave's stores are issued (not drained: the merger checks tags)
  if (tid == 0) *flag = __hip_atomic_fetch_add(gctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gn - 1;
  __syncthreads();
  if (*flag == 0) return false;
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
    if (*flag == 0) return false;
    merge_rows<G, D, NW * 64>(rsrc, base, max_chunks, ngroups, tag, scratch, tid, ms, acc, fault);
  }
  if (tid < Q) {
    const int g = tid / HQ, u = tid % HQ;
    const float inv = 1.f / ms[1];
    const u32x2 o2{pack_bf16x2(acc[0] * inv, acc[1] * inv), pack_bf16x2(acc[2] * inv, acc[3] * inv)};
    if constexpr (SC1OUT) {  // consumed inside the launch: one 8-B write-through store
      __hip_atomic_store(reinterpret_cast<uint64_t*>(out_row + g * D + 4 * u),
                         static_cast<uint64_t>(o2[0]) | (static_cast<uint64_t>(o2[1]) << 32), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    } else {
      *reinterpret_cast<u32x2*>(out_row + g * D + 4 * u) = o2;
    }
  }
  if (tid == 0) {
    __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);                          // re-arm
    __hip_atomic_store(ctr + kCtrPitch, static_cast<int>(tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // epoch
  }
  return true;
}

}  // namespace llmc
