// K5: paged attention DECODE (one query token per sequence), split-KV + reduce.
//
// Memory-bound on the K/V stream (cdna_hip_programming.md App. B "Attention decode"): K/V go
// straight to VGPRs, 16 B per lane. Geometry:
//   grid (max_chunks, nkv, B), 256 threads = 4 waves; a block owns one kv head and one chunk of
//   CHUNK context tokens, and ALL G = nh/nkv query heads of that kv head (GQA: K/V read once for
//   the group). A 16-lane group holds one key row (D <= 128 -> 8 bf16 per lane), so a wave
//   scores 4 keys per instruction; each 16-lane group runs its own online softmax, merged at
//   the end with xor-shuffles (across groups) and LDS (across waves).
// The grid is sized for the engine's maximum context so the launch is HIP-graph replayable;
// chunks past seq_len exit immediately. With a single live chunk the block writes the final
// bf16 output itself; otherwise f32 partials (unnormalised acc, running max m, sum l) go to a
// workspace and attn_decode_reduce merges them.
#include "common.h"

namespace llmc {

constexpr float kNegBig = -1e30f;

template <int G>
__global__ __launch_bounds__(256) void attn_decode_kernel(
    const bf16_t* __restrict__ q, int q_stride, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int32_t* __restrict__ block_tables, int bt_stride,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part_o, float* __restrict__ part_ml,
    bf16_t* __restrict__ out, int out_stride, int nkv, int D, int bs, int chunk, int max_chunks, float scale) {
  const int c = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int L = seq_lens[b];
  const int start = c * chunk;
  if (start >= L) return;
  const int end = min(start + chunk, L);
  const int nchunks = (L + chunk - 1) / chunk;
  const int nh = nkv * G;

  const int tid = threadIdx.x, wave = tid / kWave, lane = tid % kWave;
  const int grp = lane / 16, sub = lane % 16;
  const bool active = sub * 8 < D;
  const int d0 = active ? sub * 8 : 0;

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

  const int32_t* bt = block_tables + static_cast<int64_t>(b) * bt_stride;
  // token t handled by (wave, grp): t = start + wave*4 + grp + 16*i
  for (int t0 = start + wave * 4; t0 < end; t0 += 32) {
    u32x4 kv[2], vv[2];
    bool ok[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = t0 + grp + u * 16;
      ok[u] = t < end;
      const int tt = ok[u] ? t : start;
      const int64_t page = bt[tt / bs];
      const int64_t off = ((page * nkv + kvh) * bs + (tt % bs)) * D + d0;
      kv[u] = *reinterpret_cast<const u32x4*>(k_cache + off);
      vv[u] = *reinterpret_cast<const u32x4*>(v_cache + off);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
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

  // merge the 4 waves through LDS: [wave][g][D + 2]
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
  // thread -> (g, d) pairs
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
    const int h = kvh * G + g;
    if (nchunks == 1) {
      out[static_cast<int64_t>(b) * out_stride + h * D + d] = f32_to_bf16(o / lsum);
    } else {
      const int64_t pi = (static_cast<int64_t>(b) * nh + h) * max_chunks + c;
      part_o[pi * D + d] = o;
      if (d == 0) {
        part_ml[pi * 2] = mx;
        part_ml[pi * 2 + 1] = lsum;
      }
    }
  }
}

// grid (nh, B), 128 threads: merge chunk partials of sequences with > 1 live chunk.
__global__ __launch_bounds__(128) void attn_decode_reduce_kernel(const float* __restrict__ part_o,
                                                                 const float* __restrict__ part_ml,
                                                                 const int32_t* __restrict__ seq_lens,
                                                                 bf16_t* __restrict__ out, int out_stride, int nh,
                                                                 int D, int chunk, int max_chunks) {
  const int h = blockIdx.x, b = blockIdx.y;
  const int L = seq_lens[b];
  const int nchunks = (L + chunk - 1) / chunk;
  if (nchunks <= 1) return;
  const int64_t base = (static_cast<int64_t>(b) * nh + h) * max_chunks;
  float mx = kNegBig;
  for (int c = 0; c < nchunks; ++c) mx = fmaxf(mx, part_ml[(base + c) * 2]);
  for (int d = threadIdx.x; d < D; d += 128) {
    float lsum = 0.f, o = 0.f;
    for (int c = 0; c < nchunks; ++c) {
      const float sc = __expf(part_ml[(base + c) * 2] - mx);
      lsum += part_ml[(base + c) * 2 + 1] * sc;
      o += part_o[(base + c) * D + d] * sc;
    }
    out[static_cast<int64_t>(b) * out_stride + h * D + d] = f32_to_bf16(o / lsum);
  }
}

template <int G>
static void launch_decode(dim3 grid, size_t lds, hipStream_t s, const void* q, int q_stride, const void* kc,
                          const void* vc, const void* bt, int bt_stride, const void* sl, void* po, void* pml,
                          void* out, int out_stride, int nkv, int D, int bs, int chunk, int max_chunks, float scale) {
  attn_decode_kernel<G><<<grid, 256, lds, s>>>((const bf16_t*)q, q_stride, (const bf16_t*)kc, (const bf16_t*)vc,
                                               (const int32_t*)bt, bt_stride, (const int32_t*)sl, (float*)po,
                                               (float*)pml, (bf16_t*)out, out_stride, nkv, D, bs, chunk,
                                               max_chunks, scale);
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_attn_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                const void* block_tables, int bt_stride, const void* seq_lens, void* part_o,
                                void* part_ml, void* out, int out_stride, int B, int nh, int nkv, int D, int bs,
                                int chunk, int max_chunks, float scale, hipStream_t s) {
  if (D % 8 != 0 || D > 128 || nh % nkv != 0) return -1;
  const int G = nh / nkv;
  dim3 grid(max_chunks, nkv, B);
  const size_t lds = static_cast<size_t>(4) * G * (D + 2) * sizeof(float);
  switch (G) {
    case 1: launch_decode<1>(grid, lds, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part_o, part_ml, out, out_stride, nkv, D, bs, chunk, max_chunks, scale); break;
    case 2: launch_decode<2>(grid, lds, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part_o, part_ml, out, out_stride, nkv, D, bs, chunk, max_chunks, scale); break;
    case 4: launch_decode<4>(grid, lds, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part_o, part_ml, out, out_stride, nkv, D, bs, chunk, max_chunks, scale); break;
    case 8: launch_decode<8>(grid, lds, s, q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part_o, part_ml, out, out_stride, nkv, D, bs, chunk, max_chunks, scale); break;
    default: return -2;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return static_cast<int>(e);
  attn_decode_reduce_kernel<<<dim3(nh, B), 128, 0, s>>>((const float*)part_o, (const float*)part_ml,
                                                         (const int32_t*)seq_lens, (bf16_t*)out, out_stride, nh, D,
                                                         chunk, max_chunks);
  return static_cast<int>(hipGetLastError());
}
