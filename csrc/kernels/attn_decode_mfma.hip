// K5: paged decode attention with the GQA group on the matrix cores (one query token per
// sequence), in two forms chosen by the context bucket (host: llmc_attn_decode).
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
// SPLIT form (long contexts: judge, > 4k keys): grid (grid_chunks, nkv, B), a block = 4 waves =
// one kv head x one balanced key range (the L keys split evenly, in 32-key units, over
// min(grid_chunks, L / min_chunk) blocks: common.h decode_nsplit / decode_range), so a graph
// captured for a bucket keeps every block equally busy whatever the actual L; the block's page
// ids are staged in LDS once; per-block partials (O, m, l) go to the reduce kernel
// (attn_decode.hip), one extra launch that is noise next to tens of µs of K/V streaming.
//
// FUSED form (short contexts, <= 4k keys: responders): a block = 4 waves = one kv head x a FIXED
// 128- or 256-key chunk, one or two 32-key sub-tiles per wave. At 2k keys the whole layer is 8 MB (~1.5 µs of
// HBM) and the split form's cost was its chain of dependent round trips plus a second launch
// (7 + 5 µs, profiles/r1_bench_n1_kernel_stats.md). Here the chunk does not depend on L, so a
// wave's page id (bs % 32 == 0: its 32 keys share a page), the length and Q are loaded together
// through the scalar cache in ONE round trip, then K/V in a second; the chunks' partials are merged
// in the same launch by the last-arriving block (write-through partials + an agent-scope ticket,
// L1-bypassing loads in the reducer: no fence, see st16_sc1).
#include "common.h"

namespace llmc {

typedef __attribute__((ext_vector_type(4))) short s16x4m;
typedef __attribute__((address_space(3))) s16x4m lds_s16x4m;

constexpr float kNegInfM = -1e30f;
constexpr int kVRowBytes = 256;    // LDS pitch of one V row (D <= 128)

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

// Merge the 4 waves' states of head hh at dim d (log2 domain): o (unnormalised), m, l.
template <int G, int D>
__device__ __forceinline__ void merge_waves(const float* red, int hh, int d, float& o, float& m, float& l) {
  constexpr int stride = D + 2;
  float mx = kNegInfM;
#pragma unroll
  for (int w = 0; w < 4; ++w) mx = fmaxf(mx, red[(w * G + hh) * stride + D]);
  float ls = 0.f, oo = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const float* r = red + (w * G + hh) * stride;
    const float sc = exp2f(r[D] - mx);
    ls += r[D + 1] * sc;
    oo += r[d] * sc;
  }
  o = oo;
  m = mx;
  l = ls;
}

// ---------------------------------------------------------------------------------------------
template <int G, int D>
__global__ __launch_bounds__(256) void attn_decode_split_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, bf16_t* __restrict__ out, int out_stride,
    int nkv, int bs, int nblocks, int min_chunk, int max_chunks, float scale_log2) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  using ST = SubTile<G, D>;
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int L = seq_lens[b];
  const int nchunks = decode_nsplit(L, gridDim.x, -min_chunk);
  if (c >= nchunks) return;
  int start, end;
  decode_range(L, nchunks, c, -min_chunk, start, end);

  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* vbuf = smem + wave * 32 * kVRowBytes;  // per-wave V image [32][256 B]
  float* red = reinterpret_cast<float*>(smem + 4 * 32 * kVRowBytes);
  int* pages = reinterpret_cast<int*>(red + 4 * G * (D + 2));  // this block's page ids

  // stage the block's page ids once (no dependent block-table load per key)
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int p0 = start / bs;
  const int npages = (end - 1) / bs - p0 + 1;
  // page ids clamped into the cache: a corrupt block table reads a wrong page, never a wild address
  for (int i = tid; i < npages; i += 256) pages[i] = min(max(bt[p0 + i], 0), nblocks - 1);
  __syncthreads();
  const int64_t head_stride = static_cast<int64_t>(bs) * D;
  auto row = [&](const bf16_t* cache, int key) {
    const int64_t page = pages[key / bs - p0];
    return cache + (page * nkv + kvh) * head_stride + static_cast<int64_t>(key % bs) * D;
  };

  ST st;
  st.init(q + static_cast<int64_t>(b) * q_stride + kvh * G * D, lane);
  const int per_wave = (((end - start + 3) / 4) + 31) & ~31;  // 32-key sub-tiles per wave
  const int wbase = start + wave * per_wave;
  bf16x8 kfA[2][ST::KS], kfB[2][ST::KS];
  u32x4 vsA[ST::NV], vsB[ST::NV];
  auto valid = [&](int k) { return k - wbase < per_wave && k < end; };  // wave-uniform
  // two named register sets, hand-unrolled (no runtime-indexed register arrays, guide rule 20):
  // the next sub-tile's loads are in flight while the current one computes. (A third set, two
  // sub-tiles ahead, measured no faster at 16k-65k keys: profiles/r1_attn_decode_microbench.md.)
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
  constexpr int stride = D + 2;
  float* pb = part + ((static_cast<int64_t>(b) * nkv + kvh) * max_chunks) * G * stride;
  bf16_t* out_row = out + static_cast<int64_t>(b) * out_stride + kvh * G * D;
  for (int idx = tid; idx < G * D; idx += 256) {
    const int hh = idx / D, d = idx % D;
    float o, m, l;
    merge_waves<G, D>(red, hh, d, o, m, l);
    if (nchunks == 1) {
      out_row[hh * D + d] = f32_to_bf16(o / l);
    } else {  // partials in the natural-log domain expected by the reduce kernel
      float* pc = pb + (static_cast<int64_t>(c) * G + hh) * stride;
      pc[d] = o;
      if (d == 0) {
        pc[D] = m * 0.6931471805599453f;
        pc[D + 1] = l;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// 16-B write-through (sc1) store / L1-bypassing (sc1) load of the fused form's partials: the
// hand-off to the last-arriving block needs no release or acquire fence (≈1.7 µs each at this
// occupancy: MI355X_MICROARCH.md § visibility, fence table) — valid form row 1: every payload store
// and every payload load sc1, every storing wave drained before one lane's agent-scope ticket add,
// the last adder's workgroup loading after a barrier it joins.
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t rsrc, int byte_off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc, byte_off, 0, 16);
}
__device__ __forceinline__ f32x4 ld16_sc1(__amdgpu_buffer_rsrc_t rsrc, int byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, byte_off, 0, 16));
}

template <int G, int D>
__global__ __launch_bounds__(256) void attn_decode_fused_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters,
    bf16_t* __restrict__ out, int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks,
    float scale_log2) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  using ST = SubTile<G, D>;
  constexpr int PS = D + 4;  // partial row: O[D], then {m (log2), l, 0, 0} (16-B aligned rows)
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  const int per_wave = chunk / 4;  // keys per wave (32 or 64): inside one page (host-checked)
  // ONE round trip for everything that does not depend on the sequence length: the length, this
  // wave's page id (wave-uniform: scalar cache) and Q (vector)
  const int key0 = c * chunk + wave * per_wave;
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int pidx = __builtin_amdgcn_readfirstlane(min(key0 / bs, bt_stride - 1));
  const int page = min(max(ld_scalar(bt + pidx), 0), nblocks - 1);  // clamped into the cache
  const int L = ld_scalar(seq_lens + b);
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
    for (int idx = tid; idx < G * D; idx += 256) {
      const int hh = idx / D, d = idx % D;
      float o, m, l;
      merge_waves<G, D>(red, hh, d, o, m, l);
      out_row[hh * D + d] = f32_to_bf16(o / l);
    }
    return;
  }
  // this chunk's partial, 16 B per store, write-through
  const int64_t pbase = (static_cast<int64_t>(b) * nkv + kvh) * max_chunks * G * PS;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(part + pbase, 0, max_chunks * G * PS * 4, 0x00020000);
  for (int i4 = tid; i4 < G * D / 4; i4 += 256) {
    const int hh = (4 * i4) / D, d = (4 * i4) % D;
    f32x4 o;
    float m, l;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float oe;
      merge_waves<G, D>(red, hh, d + e, oe, m, l);
      o[e] = oe;
    }
    const int row_off = (c * G + hh) * PS * 4;
    st16_sc1(rsrc, row_off + d * 4, o);
    if (d == 0) st16_sc1(rsrc, row_off + D * 4, f32x4{m, l, 0.f, 0.f});
  }
  // ---- ticket: the last-arriving chunk block merges (every storing wave drained first) ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int* flag = reinterpret_cast<int*>(red + 4 * G * (D + 2));
  int* ctr = counters + b * nkv + kvh;
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = old == nchunks - 1;
  }
  __syncthreads();
  if (*flag == 0) return;
  float* sc = reinterpret_cast<float*>(smem);  // [G][max_chunks]: m, then 2^(m - M)
  float* lv = sc + G * max_chunks;             // [G][max_chunks]: l
  float* Lg = lv + G * max_chunks;             // [G]: total l
  for (int i = tid; i < G * nchunks; i += 256) {
    const int g = i / nchunks, cc = i % nchunks;
    const f32x4 ml = ld16_sc1(rsrc, ((cc * G + g) * PS + D) * 4);
    sc[g * max_chunks + cc] = ml[0];
    lv[g * max_chunks + cc] = ml[1];
  }
  __syncthreads();
  if (tid < G) {
    float mx = kNegInfM;
    for (int cc = 0; cc < nchunks; ++cc) mx = fmaxf(mx, sc[tid * max_chunks + cc]);
    float ls = 0.f;
    for (int cc = 0; cc < nchunks; ++cc) {
      const float e = exp2f(sc[tid * max_chunks + cc] - mx);
      sc[tid * max_chunks + cc] = e;
      ls += lv[tid * max_chunks + cc] * e;
    }
    Lg[tid] = ls;
  }
  __syncthreads();
  // 4 dims per thread, 8 chunks' loads in flight per batch
  for (int i4 = tid; i4 < G * D / 4; i4 += 256) {
    const int hh = (4 * i4) / D, d = (4 * i4) % D;
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nchunks; c0 += 8) {
      f32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cc = min(c0 + j, nchunks - 1);  // clamped: loads stay batched
        v[j] = ld16_sc1(rsrc, ((cc * G + hh) * PS + d) * 4);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float w = c0 + j < nchunks ? sc[hh * max_chunks + c0 + j] : 0.f;
        o += v[j] * w;
      }
    }
    const float inv = 1.f / Lg[hh];
    const uint32_t lo = pack_bf16x2(o[0] * inv, o[1] * inv), hi = pack_bf16x2(o[2] * inv, o[3] * inv);
    *reinterpret_cast<u32x2*>(out_row + hh * D + d) = u32x2{lo, hi};
  }
  if (tid == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

template <int G, int D>
static int launch_split(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                        const void* bt, int bt_stride, const void* sl, void* part, void* out, int out_stride, int nkv,
                        int bs, int nblocks, int chunk, int max_chunks, float scale) {
  // page-id staging sized for the largest balanced range any sequence of this table can get
  const int grid_chunks = static_cast<int>(grid.x);
  const int units = (bt_stride * bs + 31) / 32;
  const int bal = 32 * ((units + grid_chunks - 1) / grid_chunks) + 32;
  const int max_chunk = bal > 2 * chunk ? bal : 2 * chunk;
  const size_t lds = 4 * 32 * kVRowBytes + static_cast<size_t>(4) * G * (D + 2) * sizeof(float) +
                     static_cast<size_t>((max_chunk + bs - 1) / bs + 2) * sizeof(int);
  if (lds > 64 * 1024) return -4;
  attn_decode_split_kernel<G, D><<<grid, 256, lds, s>>>(
      (const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, (const int32_t*)bt, bt_stride,
      (const int32_t*)sl, (float*)part, (bf16_t*)out, out_stride, nkv, bs, nblocks, chunk, max_chunks,
      scale * 1.4426950408889634f);
  return static_cast<int>(hipGetLastError());
}

template <int G, int D>
static int launch_fused(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                        const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out, int out_stride,
                        int nkv, int bs, int nblocks, int chunk, int max_chunks, float scale) {
  const size_t red = static_cast<size_t>(4) * G * (D + 2) * sizeof(float) + 16;  // + the ticket flag
  const size_t merge = (static_cast<size_t>(2) * G * max_chunks + G) * sizeof(float);
  const size_t lds = 4 * 32 * kVRowBytes + red;
  if (merge > 4 * 32 * kVRowBytes || lds > 64 * 1024) return -4;
  if ((static_cast<int64_t>(max_chunks) * G * (D + 4) * 4) >= (1ll << 31)) return -4;
  attn_decode_fused_kernel<G, D><<<grid, 256, lds, s>>>(
      (const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, (const int32_t*)bt, bt_stride,
      (const int32_t*)sl, (float*)part, (int*)ctr, (bf16_t*)out, out_stride, nkv, bs, nblocks, chunk, max_chunks,
      scale * 1.4426950408889634f);
  return static_cast<int>(hipGetLastError());
}

template <int G>
static int launch_g(bool fused, int D, dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc,
                    const void* vc, const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out,
                    int out_stride, int nkv, int bs, int nblocks, int chunk, int max_chunks, float scale) {
#define LLMC_ATTN_D(DD)                                                                                          \
  case DD:                                                                                                       \
    return fused ? launch_fused<G, DD>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, \
                                       nkv, bs, nblocks, chunk, max_chunks, scale)                               \
                 : launch_split<G, DD>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, out, out_stride, nkv, \
                                       bs, nblocks, chunk, max_chunks, scale);
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

// Attention kernel of one decode step (the reduce of the split form: attn_decode.hip).
// fused = 1: grid_chunks fixed 128-key chunks (bucket capacity / 128), part = [B, nkv, max_chunks,
// G, D + 4] f32, counters [B, nkv] int32 zeroed once (re-armed by every merge); needs bs % 32 == 0.
// fused = 0: balanced split over <= grid_chunks blocks of >= chunk keys (multiple of 128), part =
// [B, nkv, max_chunks, G, D + 2].
extern "C" int llmc_attn_decode_mfma(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                     const void* block_tables, int bt_stride, const void* seq_lens, void* part,
                                     void* counters, void* out, int out_stride, int B, int nh, int nkv, int D, int bs,
                                     int nblocks, int chunk, int grid_chunks, int max_chunks, float scale, int fused,
                                     hipStream_t s) {
  if (nh % nkv != 0 || grid_chunks > max_chunks || grid_chunks < 1 || nblocks < 1) return -1;
  // fused: 128- or 256-key chunks, each wave's keys (chunk / 4) inside one page
  if (fused ? ((chunk != 128 && chunk != 256) || bs % (chunk / 4) != 0 || counters == nullptr)
            : (chunk % 128 != 0))
    return -1;
  dim3 grid(grid_chunks, nkv, B);
  const bool f = fused != 0;
  switch (nh / nkv) {
    case 1: return launch_g<1>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, scale);
    case 2: return launch_g<2>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, scale);
    case 4: return launch_g<4>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, scale);
    case 8: return launch_g<8>(f, D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, nblocks, chunk, max_chunks, scale);
    default: return -3;
  }
}
