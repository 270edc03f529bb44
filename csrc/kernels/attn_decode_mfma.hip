// K5 (MFMA form): paged decode attention with the GQA group on the matrix cores.
//
// The VALU form (attn_decode.hip) spends 4 cross-lane shuffles + 2 exps per (key, head); at long
// judge contexts (33k tokens: 135 MB of K/V per layer) that, not HBM, bounds it. Here a wave
// processes 32-key sub-tiles with mfma_f32_16x16x32_bf16:
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
// Grid (grid_chunks, nkv, B); a block = 4 waves = one kv head x one balanced key range: the L keys
// of the sequence are split evenly, in 32-key units, over min(grid_chunks, L / min_chunk) blocks
// (common.h decode_nsplit / decode_range), so a graph captured for a context bucket keeps every
// block equally busy whatever the actual L (one block per CU at long judge contexts, no tail).
// The cross-chunk merge reuses attn_decode.hip's partial layout and reduce kernel.
#include "attn_reduce.h"

namespace llmc {

typedef __attribute__((ext_vector_type(4))) short s16x4m;
typedef __attribute__((address_space(3))) s16x4m lds_s16x4m;

constexpr float kNegInfM = -1e30f;
constexpr int kVRowBytes = 256;  // LDS pitch of one V row (D <= 128)

__device__ __forceinline__ int vswz(int row, int chunk) { return row * kVRowBytes + ((chunk ^ ((row & 7) << 1)) << 4); }

template <int G, int D, bool TICKET>
__global__ __launch_bounds__(256) void attn_decode_mfma_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters,
    bf16_t* __restrict__ out, int out_stride, int nkv, int bs, int min_chunk, int max_chunks, float scale_log2) {
  static_assert(G <= 16 && D % 32 == 0 && D <= 128, "shape");
  constexpr int KS = D / 32;  // dim slabs for Q.K
  constexpr int DT = D / 16;  // 16-dim tiles of O^T
  constexpr int VCH = D / 8;  // 16-B chunks per V row
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int L = seq_lens[b];
  const int nchunks = decode_nsplit(L, gridDim.x, -min_chunk);
  if (c >= nchunks) return;
  int start, end;
  decode_range(L, nchunks, c, -min_chunk, start, end);

  const int tid = threadIdx.x, wave = tid / 64, lane = tid % 64;
  const int h = lane & 15, g4 = lane >> 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* vbuf = smem + wave * 32 * kVRowBytes;  // per-wave V image [32][256 B]
  float* red = reinterpret_cast<float*>(smem + 4 * 32 * kVRowBytes);
  int* pages = reinterpret_cast<int*>(red + 4 * G * (D + 2));  // this block's page ids

  // stage the block's page ids once (no dependent block-table load per key)
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const int p0 = start / bs;
  const int npages = (end - 1) / bs - p0 + 1;
  for (int i = tid; i < npages; i += 256) pages[i] = bt[p0 + i];
  __syncthreads();
  const int64_t head_stride = static_cast<int64_t>(bs) * D;
  auto row_ptr = [&](const bf16_t* cache, int key) {
    const int64_t page = pages[key / bs - p0];
    return cache + (page * nkv + kvh) * head_stride + static_cast<int64_t>(key % bs) * D;
  };

  // Q^T fragments (B operand): lane holds Q[h][ks*32 + 8*g4 .. +8] for the real heads, else 0
  bf16x8 qf[KS];
  {
    const bool real = h < G;
    const bf16_t* qrow = q + static_cast<int64_t>(b) * q_stride + (kvh * G + (real ? h : 0)) * D;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g4);
      qf[ks] = real ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }

  f32x4 acc[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = kNegInfM, l_run = 0.f;

  constexpr int NV = (32 * VCH + 63) / 64;  // 16-B V chunks per lane per sub-tile
  // issue one sub-tile's K (A operand, registers) and V (staged for LDS) loads
  auto issue = [&](int kbase, bf16x8 (&kf)[2][KS], u32x4 (&vst)[NV]) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      int key = kbase + kt * 16 + h;
      key = key < end ? key : end - 1;
      const bf16_t* kr = row_ptr(k_cache, key);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[kt][ks] = *reinterpret_cast<const bf16x8*>(kr + ks * 32 + 8 * g4);
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int flat = u * 64 + lane;
      const int row = flat / VCH, ch = flat % VCH;
      if (row < 32) {
        int key = kbase + row;
        key = key < end ? key : end - 1;
        vst[u] = *reinterpret_cast<const u32x4*>(row_ptr(v_cache, key) + ch * 8);
      }
    }
  };

  auto compute = [&](int kbase, bf16x8 (&kf)[2][KS], u32x4 (&vst)[NV]) {
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
      const int row = flat / VCH, ch = flat % VCH;
      if (row < 32) *reinterpret_cast<u32x4*>(vbuf + vswz(row, ch)) = vst[u];
    }
    // ---- online softmax over this sub-tile (head h on the lane, keys 4*g4+i and 16+4*g4+i) ----
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
  };

  const int per_wave = (((end - start + 3) / 4) + 31) & ~31;  // 32-key sub-tiles per wave
  const int wbase = start + wave * per_wave;
  bf16x8 kfA[2][KS], kfB[2][KS];
  u32x4 vsA[NV], vsB[NV];
  auto valid = [&](int k) { return k - wbase < per_wave && k < end; };  // wave-uniform
  // two named register sets, hand-unrolled (no runtime-indexed register arrays, guide rule 20):
  // the next sub-tile's loads are in flight while the current one computes. (A third set, two
  // sub-tiles ahead, measured no faster at 16k-65k keys: profiles/r1_attn_decode_microbench.md.)
  if (valid(wbase)) issue(wbase, kfA, vsA);
  for (int k0 = wbase;; k0 += 64) {
    if (!valid(k0)) break;
    if (valid(k0 + 32)) issue(k0 + 32, kfB, vsB);
    compute(k0, kfA, vsA);
    if (!valid(k0 + 32)) break;
    if (valid(k0 + 64)) issue(k0 + 64, kfA, vsA);
    compute(k0 + 32, kfB, vsB);
  }

  // ---- merge the 4 waves: red[wave][h][D + 2] (only lanes with h < G carry data) ----
  const int stride = D + 2;
  if (h < G) {
    float* r = red + (wave * G + h) * stride;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) r[dt * 16 + 4 * g4 + i] = acc[dt][i];
    if (g4 == 0) {
      r[D] = m_run;
      r[D + 1] = l_run;
    }
  }
  __syncthreads();
  float* pb = part + ((static_cast<int64_t>(b) * nkv + kvh) * max_chunks) * G * stride;
  bf16_t* out_row = out + static_cast<int64_t>(b) * out_stride + kvh * G * D;
  for (int idx = tid; idx < G * D; idx += 256) {
    const int hh = idx / D, d = idx % D;
    float mxw = kNegInfM;
#pragma unroll
    for (int w = 0; w < 4; ++w) mxw = fmaxf(mxw, red[(w * G + hh) * stride + D]);
    float lsum = 0.f, o = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float* r = red + (w * G + hh) * stride;
      const float sc = exp2f(r[D] - mxw);
      lsum += r[D + 1] * sc;
      o += r[d] * sc;
    }
    if (nchunks == 1) {
      out_row[hh * D + d] = f32_to_bf16(o / lsum);
    } else {
      // partials in the natural-log domain expected by the reducers
      float* pc = pb + (static_cast<int64_t>(c) * G + hh) * stride;
      if constexpr (TICKET) {
        st_sc1(pc + d, o);
        if (d == 0) {
          st_sc1(pc + D, mxw * 0.6931471805599453f);
          st_sc1(pc + D + 1, lsum);
        }
      } else {
        pc[d] = o;
        if (d == 0) {
          pc[D] = mxw * 0.6931471805599453f;
          pc[D + 1] = lsum;
        }
      }
    }
  }
  if constexpr (TICKET) {
    // last-arriving chunk block of this (sequence, kv head) merges all partials in-launch
    if (nchunks == 1) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are done
    __syncthreads();
    int* flag = pages;  // page ids are no longer needed
    int* ctr = counters + b * nkv + kvh;
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (old == nchunks - 1) ? 1 : 0;
    }
    __syncthreads();
    if (*flag == 0) return;
    reduce_chunks<G, true>(pb, nchunks, D, reinterpret_cast<float*>(smem), out_row);  // reuses the V images
    if (tid == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int G, int D>
static int launch_mfma(dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                       const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out, int out_stride,
                       int nkv, int bs, int chunk, int max_chunks, float scale, bool ticket) {
  // page-id staging sized for the largest balanced range any sequence of this table can get
  const int grid_chunks = static_cast<int>(grid.x);
  const int units = (bt_stride * bs + 31) / 32;
  const int bal = 32 * ((units + grid_chunks - 1) / grid_chunks) + 32;
  const int max_chunk = bal > 2 * chunk ? bal : 2 * chunk;
  const size_t lds = 4 * 32 * kVRowBytes + static_cast<size_t>(4) * G * (D + 2) * sizeof(float) +
                     static_cast<size_t>((max_chunk + bs - 1) / bs + 2) * sizeof(int);
  if (lds > 64 * 1024) return -4;
  // the in-launch reduce stages 2 * G * nchunks + 2 * G floats in the (32 KB) V-image region
  if (ticket && (2 * G * grid_chunks + 2 * G) * sizeof(float) > 4 * 32 * kVRowBytes) return -5;
  auto kern = ticket ? attn_decode_mfma_kernel<G, D, true> : attn_decode_mfma_kernel<G, D, false>;
  kern<<<grid, 256, lds, s>>>((const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, (const int32_t*)bt,
                              bt_stride, (const int32_t*)sl, (float*)part, (int*)ctr, (bf16_t*)out, out_stride, nkv,
                              bs, chunk, max_chunks, scale * 1.4426950408889634f);
  return static_cast<int>(hipGetLastError());
}

template <int G>
static int launch_mfma_d(int D, dim3 grid, hipStream_t s, const void* q, int q_stride, const void* kc, const void* vc,
                         const void* bt, int bt_stride, const void* sl, void* part, void* ctr, void* out,
                         int out_stride, int nkv, int bs, int chunk, int max_chunks, float scale, bool ticket) {
  switch (D) {
    case 64: return launch_mfma<G, 64>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, nkv, bs, chunk, max_chunks, scale, ticket);
    case 96: return launch_mfma<G, 96>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, nkv, bs, chunk, max_chunks, scale, ticket);
    case 128: return launch_mfma<G, 128>(grid, s, q, q_stride, kc, vc, bt, bt_stride, sl, part, ctr, out, out_stride, nkv, bs, chunk, max_chunks, scale, ticket);
    default: return -2;
  }
}

}  // namespace llmc

using namespace llmc;

// Same workspace/contract as llmc_attn_decode; chunk (the minimum balanced chunk) must be a
// multiple of 128. ticket: merge in-launch (last arriver) instead of leaving partials for the
// reduce kernel.
extern "C" int llmc_attn_decode_mfma(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                     const void* block_tables, int bt_stride, const void* seq_lens, void* part,
                                     void* counters, void* out, int out_stride, int B, int nh, int nkv, int D, int bs,
                                     int chunk, int grid_chunks, int max_chunks, float scale, int ticket,
                                     hipStream_t s) {
  if (nh % nkv != 0 || chunk % 128 != 0 || grid_chunks > max_chunks) return -1;
  dim3 grid(grid_chunks, nkv, B);
  switch (nh / nkv) {
    case 1: return launch_mfma_d<1>(D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, chunk, max_chunks, scale, ticket != 0);
    case 2: return launch_mfma_d<2>(D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, chunk, max_chunks, scale, ticket != 0);
    case 4: return launch_mfma_d<4>(D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, chunk, max_chunks, scale, ticket != 0);
    case 8: return launch_mfma_d<8>(D, grid, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, nkv, bs, chunk, max_chunks, scale, ticket != 0);
    default: return -3;
  }
}
