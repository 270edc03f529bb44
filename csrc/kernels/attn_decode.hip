// K5 (long contexts): cross-chunk merge of the SPLIT form of decode attention
// (attn_decode_mfma.hip: per-block partials O, m (natural log), l in [B, nkv, max_chunks, G, D + 2])
// and the host entry point that picks the form per context bucket.
#include "common.h"

namespace llmc {

constexpr float kNegBig = -1e30f;

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

static size_t reduce_lds(int max_chunks) { return (2 * static_cast<size_t>(max_chunks) + 256 + 8) * sizeof(float); }

// One reduce launch; DB (dims per block) from the largest chunk count this grid can produce, so
// even a 256-way split merges in one round trip.
template <int G>
static int launch_reduce(int B, int nkv, int D, int chunk_arg, int gc, int max_chunks, hipStream_t s, const void* part,
                         const void* sl, void* out, int out_stride) {
  const size_t lds = reduce_lds(max_chunks);
  if (gc <= 64) {
    attn_decode_reduce_kernel<G, 64><<<dim3(nkv * G, B, (D + 63) / 64), 256, lds, s>>>(
        (const float*)part, (const int32_t*)sl, (bf16_t*)out, out_stride, nkv, D, chunk_arg, gc, max_chunks);
  } else if (gc <= 128) {
    attn_decode_reduce_kernel<G, 32><<<dim3(nkv * G, B, (D + 31) / 32), 256, lds, s>>>(
        (const float*)part, (const int32_t*)sl, (bf16_t*)out, out_stride, nkv, D, chunk_arg, gc, max_chunks);
  } else {
    attn_decode_reduce_kernel<G, 16><<<dim3(nkv * G, B, (D + 15) / 16), 256, lds, s>>>(
        (const float*)part, (const int32_t*)sl, (bf16_t*)out, out_stride, nkv, D, chunk_arg, gc, max_chunks);
  }
  return static_cast<int>(hipGetLastError());
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_attn_decode_mfma(const void*, int, const void*, const void*, const void*, int, const void*, void*,
                                     void*, void*, int, int, int, int, int, int, int, int, int, int, float, int,
                                     hipStream_t);

// One decode step's attention for rows 0..B-1. fused = 1 (short contexts): fixed 128-key chunks,
// grid_chunks = bucket capacity / 128, merged in the same launch (part [B, nkv, max_chunks, G, D + 4],
// counters [B, nkv] int32 zeroed once). fused = 0 (long contexts): balanced split over <= grid_chunks
// blocks of >= chunk keys (a multiple of 128) + the reduce launch (part [B, nkv, max_chunks, G, D + 2]).
extern "C" int llmc_attn_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                                const void* block_tables, int bt_stride, const void* seq_lens, void* part,
                                void* counters, void* out, int out_stride, int B, int nh, int nkv, int D, int bs,
                                int nblocks, int chunk, int grid_chunks, int max_chunks, float scale, int fused,
                                hipStream_t s) {
  if (D % 32 != 0 || D > 128 || nh % nkv != 0 || grid_chunks > max_chunks) return -1;
  int rc = llmc_attn_decode_mfma(q, q_stride, k_cache, v_cache, block_tables, bt_stride, seq_lens, part, counters,
                                 out, out_stride, B, nh, nkv, D, bs, nblocks, chunk, grid_chunks, max_chunks, scale,
                                 fused, s);
  if (rc != 0 || fused || grid_chunks <= 1) return rc;
  switch (nh / nkv) {
    case 1: return launch_reduce<1>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
    case 2: return launch_reduce<2>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
    case 4: return launch_reduce<4>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
    case 8: return launch_reduce<8>(B, nkv, D, -chunk, grid_chunks, max_chunks, s, part, seq_lens, out, out_stride);
    default: return -2;
  }
}
