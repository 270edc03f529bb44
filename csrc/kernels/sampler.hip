// K8: sampler + device-resident decode-state advance.
//
// Fast path (greedy, or plain temperature sampling): Gumbel-max  argmax(logit/T + g),
// g = -log(-log(u)), u from Philox4x32-10(key = seed[b], counter = (vocab idx, position)).
// Two launches: stage 1 spreads the 128k-wide row over 64 blocks (full-chip bandwidth), stage 2
// (one wave per row) finishes the argmax and ADVANCES the decode state on device:
//   out_tokens[b][count] = tok; count++; tokens_in[b] = tok; pos++; seq_len = pos + 1;
//   slot = block_table[pos / bs] * bs + pos % bs.
// Because positions, seeds and slots live in device memory, the whole decode step (embedding ->
// layers -> logits -> sample -> advance) replays from a HIP graph with no host work per token.
//
// Top-k / top-p path: one 1024-thread block per row, exact radix select (4 x 8-bit passes over
// the order-preserving uint image of the float logits) for the top-k threshold, then the same
// radix walk over probability MASS for the top-p threshold, then Gumbel-max over survivors.
#include "common.h"

namespace llmc {

struct Philox {
  __device__ static inline void round(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint64_t p0 = static_cast<uint64_t>(M0) * c[0];
    const uint64_t p1 = static_cast<uint64_t>(M1) * c[2];
    const uint32_t hi0 = p0 >> 32, lo0 = static_cast<uint32_t>(p0);
    const uint32_t hi1 = p1 >> 32, lo1 = static_cast<uint32_t>(p1);
    c[0] = hi1 ^ c[1] ^ k0;
    c[1] = lo1;
    c[2] = hi0 ^ c[3] ^ k1;
    c[3] = lo0;
  }
  __device__ static inline uint32_t draw(uint64_t key, uint32_t idx, uint32_t step) {
    uint32_t c[4] = {idx, step, 0x5eedu, 0u};
    uint32_t k0 = static_cast<uint32_t>(key), k1 = static_cast<uint32_t>(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      round(c, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    return c[0];
  }
};

__device__ __forceinline__ float gumbel(uint64_t key, uint32_t idx, uint32_t step) {
  const uint32_t r = Philox::draw(key, idx, step);
  const float u = (static_cast<float>(r >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
  return -__logf(-__logf(u));
}

// better(a) if larger value, ties -> smaller index
__device__ __forceinline__ void argmax_merge(float& v, int& i, float ov, int oi) {
  if (ov > v || (ov == v && oi < i)) {
    v = ov;
    i = oi;
  }
}

__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(i, o, 64);
    argmax_merge(v, i, ov, oi);
  }
}

constexpr int kParts = 64;

// grid (kParts, B), 256 threads
__global__ __launch_bounds__(256) void sample_stage1_kernel(const float* __restrict__ logits, int64_t row_stride,
                                                            int V, const float* __restrict__ inv_temp,
                                                            const int64_t* __restrict__ seeds,
                                                            const int32_t* __restrict__ positions,
                                                            float* __restrict__ part_v, int* __restrict__ part_i) {
  const int p = blockIdx.x, b = blockIdx.y;
  const float* row = logits + b * row_stride;
  const float it = inv_temp[b];
  const bool greedy = it <= 0.f;
  const uint64_t key = static_cast<uint64_t>(seeds[b]);
  const uint32_t step = static_cast<uint32_t>(positions[b]);
  const int per = (V + kParts - 1) / kParts;
  const int lo = p * per, hi = min(V, lo + per);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = lo + threadIdx.x; i < hi; i += 256) {
    float v = row[i];
    if (!greedy) v = v * it + gumbel(key, static_cast<uint32_t>(i), step);
    argmax_merge(bv, bi, v, i);
  }
  wave_argmax(bv, bi);
  __shared__ float sv[4];
  __shared__ int si[4];
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = bv;
    si[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k) argmax_merge(bv, bi, sv[k], si[k]);
    part_v[b * kParts + p] = bv;
    part_i[b * kParts + p] = bi;
  }
}

struct DecodeState {
  int32_t* tokens_in;     // [B]
  int32_t* positions;     // [B]
  int32_t* seq_lens;      // [B]
  int32_t* slots;         // [B]
  const int32_t* block_tables;  // [B, bt_stride]
  int bt_stride;
  int bs;
  int32_t* out_tokens;    // [B, cap]
  int32_t* out_count;     // [B]
  int cap;
};

// No-op unless tokens_in is given (a bare sample call must not move the position/step counter).
__device__ __forceinline__ void advance(const DecodeState& st, int b, int tok) {
  if (st.tokens_in == nullptr) return;
  if (st.out_tokens != nullptr) {
    const int cnt = st.out_count[b];
    if (cnt < st.cap) st.out_tokens[static_cast<int64_t>(b) * st.cap + cnt] = tok;
    st.out_count[b] = cnt + 1;
  }
  if (st.tokens_in != nullptr) st.tokens_in[b] = tok;
  if (st.positions != nullptr) {
    const int pos = st.positions[b] + 1;
    st.positions[b] = pos;
    if (st.seq_lens != nullptr) st.seq_lens[b] = pos + 1;
    if (st.slots != nullptr && st.block_tables != nullptr) {
      const int blk = st.block_tables[static_cast<int64_t>(b) * st.bt_stride + pos / st.bs];
      st.slots[b] = blk * st.bs + pos % st.bs;
    }
  }
}

// grid B, 64 threads
__global__ __launch_bounds__(64) void sample_stage2_kernel(const float* __restrict__ part_v,
                                                           const int* __restrict__ part_i, int32_t* __restrict__ next,
                                                           DecodeState st) {
  const int b = blockIdx.x;
  float v = part_v[b * kParts + threadIdx.x];
  int i = part_i[b * kParts + threadIdx.x];
  wave_argmax(v, i);
  if (threadIdx.x == 0) {
    next[b] = i;
    advance(st, b, i);
  }
}

// ------------------------------------------------------------------------------------------
// top-k / top-p (exact radix select), one 1024-thread block per row
__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int kTKThreads = 1024;

__global__ __launch_bounds__(kTKThreads) void sample_topkp_kernel(const float* __restrict__ logits, int64_t row_stride,
                                                                  int V, const float* __restrict__ inv_temp,
                                                                  const int* __restrict__ top_k,
                                                                  const float* __restrict__ top_p,
                                                                  const int64_t* __restrict__ seeds,
                                                                  int32_t* __restrict__ next, DecodeState st) {
  const int b = blockIdx.x;
  const float* row = logits + b * row_stride;
  const float it_raw = inv_temp[b];
  const bool greedy = it_raw <= 0.f;
  const float it = greedy ? 1.f : it_raw;
  const int k = top_k[b];
  const float pp = top_p[b];
  const uint64_t key = static_cast<uint64_t>(seeds[b]);
  const uint32_t step = static_cast<uint32_t>(st.positions != nullptr ? st.positions[b] : 0);
  __shared__ float red[kTKThreads / 64];
  __shared__ unsigned cnt[256];
  __shared__ float mass[256];
  __shared__ uint32_t sh_prefix, sh_mask;
  __shared__ float sh_rem;
  __shared__ float sv[kTKThreads / 64];
  __shared__ int si[kTKThreads / 64];

  // max
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < V; i += kTKThreads) mx = fmaxf(mx, row[i]);
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = mx;
  __syncthreads();
  mx = -INFINITY;
  for (int w = 0; w < kTKThreads / 64; ++w) mx = fmaxf(mx, red[w]);
  __syncthreads();

  uint32_t thr = 0;  // keep elements with fkey(logit) >= thr
  // ---- top-k radix select ----
  if (k > 0 && k < V) {
    if (threadIdx.x == 0) {
      sh_prefix = 0;
      sh_mask = 0;
      sh_rem = static_cast<float>(k);
    }
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int j = threadIdx.x; j < 256; j += kTKThreads) cnt[j] = 0;
      __syncthreads();
      const uint32_t prefix = sh_prefix, mask = sh_mask;
      for (int i = threadIdx.x; i < V; i += kTKThreads) {
        const uint32_t kk = fkey(row[i]);
        if ((kk & mask) == prefix) atomicAdd(&cnt[(kk >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        float rem = sh_rem;
        int bin = 255;
        for (; bin > 0; --bin) {
          if (static_cast<float>(cnt[bin]) >= rem) break;
          rem -= static_cast<float>(cnt[bin]);
        }
        sh_rem = rem;
        sh_prefix = prefix | (static_cast<uint32_t>(bin) << shift);
        sh_mask = mask | (255u << shift);
      }
      __syncthreads();
    }
    thr = sh_prefix;
  }
  // ---- top-p radix select over probability mass ----
  if (pp < 1.f && !greedy) {
    float z = 0.f;
    for (int i = threadIdx.x; i < V; i += kTKThreads) {
      const float l = row[i];
      if (fkey(l) >= thr) z += __expf((l - mx) * it);
    }
    z = block_sum<kTKThreads>(z, red);
    if (threadIdx.x == 0) {
      sh_prefix = 0;
      sh_mask = 0;
      sh_rem = pp * z;
    }
    __syncthreads();
    for (int shift = 24; shift >= 0; shift -= 8) {
      for (int j = threadIdx.x; j < 256; j += kTKThreads) mass[j] = 0.f;
      __syncthreads();
      const uint32_t prefix = sh_prefix, mask = sh_mask;
      for (int i = threadIdx.x; i < V; i += kTKThreads) {
        const float l = row[i];
        const uint32_t kk = fkey(l);
        if (kk >= thr && (kk & mask) == prefix) atomicAdd(&mass[(kk >> shift) & 255u], __expf((l - mx) * it));
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        float rem = sh_rem;
        int bin = 255;
        for (; bin > 0; --bin) {
          if (mass[bin] >= rem) break;
          rem -= mass[bin];
        }
        sh_rem = rem;
        sh_prefix = prefix | (static_cast<uint32_t>(bin) << shift);
        sh_mask = mask | (255u << shift);
      }
      __syncthreads();
    }
    thr = max(thr, sh_prefix);
  }
  // ---- Gumbel-max over survivors ----
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += kTKThreads) {
    const float l = row[i];
    if (fkey(l) < thr) continue;
    const float v = greedy ? l : l * it + gumbel(key, static_cast<uint32_t>(i), step);
    argmax_merge(bv, bi, v, i);
  }
  wave_argmax(bv, bi);
  if ((threadIdx.x & 63) == 0) {
    sv[threadIdx.x / 64] = bv;
    si[threadIdx.x / 64] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kTKThreads / 64; ++w) argmax_merge(bv, bi, sv[w], si[w]);
    next[b] = bi;
    advance(st, b, bi);
  }
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_sample(const void* logits, int64_t row_stride, int B, int V, const void* inv_temp,
                           const void* top_k, const void* top_p, const void* seeds, const void* positions,
                           void* workspace_v, void* workspace_i, void* next, void* tokens_in, void* seq_lens,
                           void* slots, const void* block_tables, int bt_stride, int bs, void* out_tokens,
                           void* out_count, int cap, int use_topkp, hipStream_t s) {
  DecodeState st;
  st.tokens_in = (int32_t*)tokens_in;
  st.positions = (int32_t*)positions;
  st.seq_lens = (int32_t*)seq_lens;
  st.slots = (int32_t*)slots;
  st.block_tables = (const int32_t*)block_tables;
  st.bt_stride = bt_stride;
  st.bs = bs;
  st.out_tokens = (int32_t*)out_tokens;
  st.out_count = (int32_t*)out_count;
  st.cap = cap;
  if (use_topkp) {
    sample_topkp_kernel<<<B, kTKThreads, 0, s>>>((const float*)logits, row_stride, V, (const float*)inv_temp,
                                                 (const int*)top_k, (const float*)top_p, (const int64_t*)seeds,
                                                 (int32_t*)next, st);
    return static_cast<int>(hipGetLastError());
  }
  sample_stage1_kernel<<<dim3(kParts, B), 256, 0, s>>>((const float*)logits, row_stride, V, (const float*)inv_temp,
                                                       (const int64_t*)seeds, (const int32_t*)positions,
                                                       (float*)workspace_v, (int*)workspace_i);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return static_cast<int>(e);
  sample_stage2_kernel<<<B, 64, 0, s>>>((const float*)workspace_v, (const int*)workspace_i, (int32_t*)next, st);
  return static_cast<int>(hipGetLastError());
}

extern "C" int llmc_sample_parts() { return kParts; }
