// K5: paged attention DECODE (one query token per sequence), split-KV.
//
// Batch-1 decode attention on an 8-kv-head model is LATENCY-bound (a 1k-token context is 4 MB of
// K/V: < 1 µs of HBM time), so the design minimises the serial chain of memory round trips:
//   grid (grid_chunks, nkv, B), 256 threads = 4 waves; a block owns one kv head and one chunk of
//   `chunk` context tokens and ALL G = nh/nkv query heads of that kv head (GQA: K/V read once).
//   * page lookup: when chunk divides the page size the whole block lives in ONE page -> one
//     uniform (scalar) block-table load; otherwise per token;
//   * every K/V load of a wave is issued before any math (UN tokens per 16-lane group, 16 B per
//     lane, a 16-lane group holds one D <= 128 key row) -> one HBM round trip per block;
//   * each 16-lane group runs an online softmax over its keys; groups merge by xor-shuffles,
//     waves through LDS; a single live chunk writes the bf16 output directly.
// Cross-chunk merge, two selectable forms (measured, see profiles/):
//   REDUCE_KERNEL (default): partials with plain stores, then attn_decode_reduce_kernel —
//     inside a HIP graph the kernel boundary (~1.2 µs) is cheaper than an in-launch hand-off;
//   TICKET: write-through (sc1) partial stores + agent-scope ticket; the last-arriving block
//     reduces with sc1 loads (Guideline 16 valid form, row 1) — no second launch.
// Grid sized per context bucket by the host (one captured decode graph per bucket); chunks past
// seq_len exit immediately.
#include "attn_reduce.h"

namespace llmc {

template <int G, bool TICKET>
__global__ __launch_bounds__(256) void attn_decode_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part, int* __restrict__ counters,
    bf16_t* __restrict__ out, int out_stride, int nkv, int D, int bs, int chunk, int max_chunks, float scale) {
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int L = seq_lens[b];
  const int start = c * chunk;
  if (start >= L) return;
  const int end = min(start + chunk, L);
  const int nchunks = (L + chunk - 1) / chunk;

  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const int grp = lane / 16, sub = lane % 16;
  const bool active = sub * 8 < D;
  const int d0 = active ? sub * 8 : 0;
  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  const bool one_page = (bs % chunk) == 0;
  const int64_t page0 = bt[start / bs];  // uniform

  // q for the G heads of this kv head, pre-scaled, as packed bf16 for v_dot2.
  u32x4 qv[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bf16_t* qp = q + static_cast<int64_t>(b) * q_stride + (kvh * G + g) * D + d0;
    u32x4 raw = *reinterpret_cast<const u32x4*>(qp);
    float f[8];
    unpack8(raw, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = active ? f[j] * scale : 0.f;
    qv[g] = pack8(f);
  }

  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = kNegBig;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }

  // token t handled by (wave, grp): t = start + wave*4 + grp + 16*u
  constexpr int UN = 4;
  for (int t0 = start + wave * 4; t0 < end; t0 += 16 * UN) {
    u32x4 kv[UN], vv[UN];
    bool ok[UN];
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      const int t = t0 + grp + u * 16;
      ok[u] = t < end;
      const int tt = ok[u] ? t : start;
      const int64_t page = one_page ? page0 : static_cast<int64_t>(bt[tt / bs]);
      const int64_t off = ((page * nkv + kvh) * bs + (tt % bs)) * D + d0;
      kv[u] = *reinterpret_cast<const u32x4*>(k_cache + off);
      vv[u] = *reinterpret_cast<const u32x4*>(v_cache + off);
    }
#pragma unroll
    for (int u = 0; u < UN; ++u) {
      float vf[8];
      unpack8(vv[u], vf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float s = dot8_bf16(qv[g], kv[u], 0.f);
        s = group_sum<16>(s);
        if (!ok[u]) s = kNegBig;
        const float mn = fmaxf(m[g], s);
        const float alpha = __expf(m[g] - mn);
        const float p = __expf(s - mn);
        l[g] = l[g] * alpha + p;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[g][j] = acc[g][j] * alpha + p * vf[j];
        m[g] = mn;
      }
    }
  }

  // merge the 4 lane-groups of the wave (lanes sub, sub+16, sub+32, sub+48)
#pragma unroll
  for (int o = 16; o <= 32; o <<= 1) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float mo = __shfl_xor(m[g], o, 64);
      const float lo = __shfl_xor(l[g], o, 64);
      const float mn = fmaxf(m[g], mo);
      const float a = __expf(m[g] - mn), bb = __expf(mo - mn);
      l[g] = l[g] * a + lo * bb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float ao = __shfl_xor(acc[g][j], o, 64);
        acc[g][j] = acc[g][j] * a + ao * bb;
      }
      m[g] = mn;
    }
  }

  // merge the 4 waves through LDS: red[wave][g][D + 2]
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);
  const int stride = D + 2;
  if (grp == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float* r = red + (wave * G + g) * stride;
      if (active) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[d0 + j] = acc[g][j];
      }
      if (sub == 0) {
        r[D] = m[g];
        r[D + 1] = l[g];
      }
    }
  }
  __syncthreads();
  float* pb = part + ((static_cast<int64_t>(b) * nkv + kvh) * max_chunks) * G * stride;
  bf16_t* out_row = out + static_cast<int64_t>(b) * out_stride + kvh * G * D;
  for (int idx = tid; idx < G * D; idx += 256) {
    const int g = idx / D, d = idx % D;
    float mx = kNegBig;
#pragma unroll
    for (int w = 0; w < 4; ++w) mx = fmaxf(mx, red[(w * G + g) * stride + D]);
    float lsum = 0.f, o = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float* r = red + (w * G + g) * stride;
      const float sc = __expf(r[D] - mx);
      lsum += r[D + 1] * sc;
      o += r[d] * sc;
    }
    if (nchunks == 1) {
      out_row[g * D + d] = f32_to_bf16(o / lsum);
    } else {
      float* pc = pb + (static_cast<int64_t>(c) * G + g) * stride;
      if constexpr (TICKET) {
        st_sc1(pc + d, o);
        if (d == 0) {
          st_sc1(pc + D, mx);
          st_sc1(pc + D + 1, lsum);
        }
      } else {
        pc[d] = o;
        if (d == 0) {
          pc[D] = mx;
          pc[D + 1] = lsum;
        }
      }
    }
  }
  if constexpr (TICKET) {
    if (nchunks == 1) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    int* flag = reinterpret_cast<int*>(red + 4 * G * stride);
    int* ctr = counters + b * nkv + kvh;
    if (tid == 0) {
      const int old = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (old == nchunks - 1) ? 1 : 0;
    }
    __syncthreads();
    if (*flag == 0) return;
    reduce_chunks<G, true>(pb, nchunks, D, red + 4 * G * stride + 4, out_row);
    if (tid == 0) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// grid (nkv * G, B, ceil(D / DB)), 256 threads: one query head x DB dims per block; the 256
// threads are DB dims x (256 / DB) chunk groups. ONE memory round trip for up to 16 * 256 / DB
// chunks: every thread issues its (up to 16) partial-value loads and the block its m / l loads
// together — the values do not depend on the softmax max — then the max, the scale factors and
// the weighted sums are formed from registers and LDS; chunk groups meet in LDS. The host picks
// DB from the grid's chunk count (64 / 32 / 16 for <= 64 / 128 / 256 chunks) so a wide split
// (a TP rank's single kv head spread over 256 blocks) still merges in one round trip, on 4x the
// blocks, instead of 4 dependent batches.
template <int G, int DB>
__global__ __launch_bounds__(256) void attn_decode_reduce_kernel(const float* __restrict__ part,
                                                                 const int32_t* __restrict__ seq_lens,
                                                                 bf16_t* __restrict__ out, int out_stride, int nkv,
                                                                 int D, int chunk_arg, int gc, int max_chunks) {
  static_assert(DB == 16 || DB == 32 || DB == 64, "DB");
  constexpr int CG = 256 / DB;  // chunk groups
  const int kvh = blockIdx.x / G, g = blockIdx.x % G, b = blockIdx.y;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sc = reinterpret_cast<float*>(smem);  // [max_chunks]: m, then exp(m - M)
  float* lv = sc + max_chunks;                 // [max_chunks]: l
  float* red = lv + max_chunks;                // [CG][DB] + 8 scratch
  const int tid = threadIdx.x, stride = D + 2;
  const float* pb = part + ((static_cast<int64_t>(b) * nkv + kvh) * max_chunks * G + g) * stride;
  const int64_t cstride = static_cast<int64_t>(G) * stride;  // between consecutive chunks
  const int dl = tid % DB, cg = tid / DB;
  const int d = blockIdx.z * DB + dl;
  const bool live = d < D;
  // The partial values and this thread's (m, l) words are loaded for the GRID's chunk count gc
  // before the sequence length arrives: they do not depend on it, so the length's round trip
  // and theirs overlap. Slots past the sequence's own chunk count hold finite stale partials
  // (the workspace starts zeroed) and are masked below, never multiplied in.
  float v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int c = min(cg + CG * j, gc - 1);  // clamped: all loads in flight, masked below
    v[j] = live ? pb[c * cstride + d] : 0.f;
  }
  float m0 = kNegBig, l0 = 0.f;
  if (tid < gc) {
    m0 = pb[tid * cstride + D];
    l0 = pb[tid * cstride + D + 1];
  }
  const int L = seq_lens[b];
  const int nchunks = decode_nsplit(L, gc, chunk_arg);
  if (nchunks <= 1) return;
  float mx = kNegBig;
  for (int c = tid; c < nchunks; c += 256) {
    const float m = c == tid ? m0 : pb[c * cstride + D];
    sc[c] = m;
    lv[c] = c == tid ? l0 : pb[c * cstride + D + 1];
    mx = fmaxf(mx, m);
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[256 + tid / 64] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[256], red[257]), fmaxf(red[258], red[259]));
  float ls = 0.f;
  for (int c = tid; c < nchunks; c += 256) {
    const float e = __expf(sc[c] - mx);
    sc[c] = e;
    ls += lv[c] * e;
  }
  ls = wave_sum(ls);
  if ((tid & 63) == 0) red[260 + tid / 64] = ls;
  __syncthreads();
  const float lsum = red[260] + red[261] + red[262] + red[263];
  float o = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) o += (cg + CG * j < nchunks) ? v[j] * sc[cg + CG * j] : 0.f;
  for (int c0 = cg + 16 * CG; c0 < nchunks; c0 += 16 * CG) {  // beyond one round trip: further batches
    float w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = min(c0 + CG * j, nchunks - 1);
      w[j] = live ? pb[c * cstride + d] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) o += (c0 + CG * j < nchunks) ? w[j] * sc[c0 + CG * j] : 0.f;
  }
  red[cg * DB + dl] = o;
  __syncthreads();
  if (cg == 0 && live) {
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < CG; ++i) tot += red[i * DB + dl];
    out[static_cast<int64_t>(b) * out_stride + (kvh * G + g) * D + d] = f32_to_bf16(tot / lsum);
  }
}

// One reduce launch; DB (dims per block) from the largest chunk count this grid can produce.
template <int G>
static int launch_reduce(int B, int nkv, int D, int chunk, int gc, int max_chunks, hipStream_t s, const void* part,
                         const void* sl, void* out, int out_stride);

static size_t reduce_lds(int max_chunks) { return (2 * static_cast<size_t>(max_chunks) + 256 + 8) * sizeof(float); }

template <int G>
static int launch_decode(int B, int nkv, int grid_chunks, hipStream_t s, const void* q, int q_stride, const void* kc,
                         const void* vc, const void* bt, int bt_stride, const void* sl, void* part, void* ctr,
                         void* out, int out_stride, int D, int bs, int chunk, int max_chunks, float scale,
                         bool ticket) {
  const size_t red_lds = static_cast<size_t>(4) * G * (D + 2) * sizeof(float);
  const size_t scl_lds = (static_cast<size_t>(G) * (2 * max_chunks + 2)) * sizeof(float);
  if (red_lds + 16 + scl_lds > 160 * 1024) return -3;
  dim3 grid(grid_chunks, nkv, B);
  if (ticket) {
    auto kern = attn_decode_kernel<G, true>;
    const size_t lds = red_lds + 16 + scl_lds;
    static bool attr = false;
    if (lds > 64 * 1024 && !attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024);
      attr = true;
    }
    kern<<<grid, 256, lds, s>>>((const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, (const int32_t*)bt,
                                bt_stride, (const int32_t*)sl, (float*)part, (int*)ctr, (bf16_t*)out, out_stride, nkv,
                                D, bs, chunk, max_chunks, scale);
    return static_cast<int>(hipGetLastError());
  }
  attn_decode_kernel<G, false><<<grid, 256, red_lds, s>>>(
      (const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc, (const int32_t*)bt, bt_stride,
      (const int32_t*)sl, (float*)part, (int*)ctr, (bf16_t*)out, out_stride, nkv, D, bs, chunk, max_chunks, scale);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return static_cast<int>(e);
  if (grid_chunks > 1) {
    return launch_reduce<G>(B, nkv, D, chunk, grid_chunks, max_chunks, s, part, sl, out, out_stride);
  }
  return static_cast<int>(hipGetLastError());
}

}  // namespace llmc

using namespace llmc;

// part: f32 workspace [B, nkv, max_chunks, G, D + 2]; counters: int32 [B, nkv], zero-initialised
// once (the TICKET form re-arms them every launch). grid_chunks <= max_chunks bounds the context
// of this launch. mode: 0 = VALU partials + reduce kernel, 1 = VALU in-launch ticket reduce,
// 2 = MFMA balanced split + reduce kernel, 3 = MFMA balanced split + in-launch ticket reduce
// (modes 2/3: chunk = minimum keys per block, a multiple of 128).
extern "C" int llmc_attn_decode_mfma(const void*, int, const void*, const void*, const void*, int, const void*, void*,
                                     void*, void*, int, int, int, int, int, int, int, int, int, float, int,
                                     hipStream_t);

namespace llmc {
template <int G>
static int launch_reduce(int B, int nkv, int D, int chunk, int gc, int max_chunks, hipStream_t s, const void* part,
                         const void* sl, void* out, int out_stride) {
  // chunks this grid can produce: gc (balanced form) or ceil(context / chunk) (fixed chunks: gc
  // is the bucket's chunk count as well)
  const int nmax = gc;
  const size_t lds = reduce_lds(max_chunks);
  if (nmax <= 64) {
    attn_decode_reduce_kernel<G, 64><<<dim3(nkv * G, B, (D + 63) / 64), 256, lds, s>>>(
        (const float*)part, (const int32_t*)sl, (bf16_t*)out, out_stride, nkv, D, chunk, gc, max_chunks);
  } else if (nmax <= 128) {
    attn_decode_reduce_kernel<G, 32><<<dim3(nkv * G, B, (D + 31) / 32), 256, lds, s>>>(
        (const float*)part, (const int32_t*)sl, (bf16_t*)out, out_stride, nkv, D, chunk, gc, max_chunks);
  } else {
    attn_decode_reduce_kernel<G, 16><<<dim3(nkv * G, B, (D + 15) / 16), 256, lds, s>>>(
        (const float*)part, (const int32_t*)sl, (bf16_t*)out, out_stride, nkv, D, chunk, gc, max_chunks);
  }
  return static_cast<int>(hipGetLastError());
}
}  // namespace llmc

template <int G>
static int launch_reduce_only(int B, int nkv, int D, int chunk, int gc, int max_chunks, hipStream_t s, const void* part,
                              const void* sl, void* out, int out_stride) {
  return launch_reduce<G>(B, nkv, D, chunk, gc, max_chunks, s, part, sl, out, out_stride);
}

extern "C" int llmc_attn_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                const void* block_tables, int bt_stride, const void* seq_lens, void* part,
                                void* counters, void* out, int out_stride, int B, int nh, int nkv, int D, int bs,
                                int chunk, int grid_chunks, int max_chunks, float scale, int mode, hipStream_t s) {
  if (D % 8 != 0 || D > 128 || nh % nkv != 0 || grid_chunks > max_chunks) return -1;
  if (mode == 2 || mode == 3 || mode == 4) {  // MFMA (attn_decode_mfma.hip) [+ reduce kernel]
    int rc = llmc_attn_decode_mfma(q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters,
                                   out, out_stride, B, nh, nkv, D, bs, chunk, grid_chunks, max_chunks, scale,
                                   mode == 3, s);
    // mode 4: partials are left for the consumer (o_proj GEMV with the PRO_MERGE prologue)
    if (rc != 0 || grid_chunks <= 1 || mode >= 3) return rc;
    switch (nh / nkv) {
      case 1: return launch_reduce_only<1>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
      case 2: return launch_reduce_only<2>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
      case 4: return launch_reduce_only<4>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
      case 8: return launch_reduce_only<8>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
      default: return -2;
    }
  }
  const bool ticket = mode == 1;
  switch (nh / nkv) {
    case 1: return launch_decode<1>(B, nkv, grid_chunks, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, D, bs, chunk, max_chunks, scale, ticket);
    case 2: return launch_decode<2>(B, nkv, grid_chunks, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, D, bs, chunk, max_chunks, scale, ticket);
    case 4: return launch_decode<4>(B, nkv, grid_chunks, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, D, bs, chunk, max_chunks, scale, ticket);
    case 8: return launch_decode<8>(B, nkv, grid_chunks, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters, out, out_stride, D, bs, chunk, max_chunks, scale, ticket);
    default: return -2;
  }
}
