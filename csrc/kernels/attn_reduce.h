// Cross-chunk merge of split-KV decode attention partials, shared by the VALU (attn_decode.hip)
// and MFMA (attn_decode_mfma.hip) kernels' in-launch "last arriver reduces" (TICKET) form.
// Partial layout per (sequence, kv head): [chunk][G][D + 2] f32 = unnormalised O, m (natural-log
// domain), l. sc1 (write-through, agent scope) stores/loads make partials written on one XCD's
// L2 visible to the last-arriving block on another (Guideline 16 valid form).
#pragma once
#include "common.h"

namespace llmc {

constexpr float kNegBig = -1e30f;

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Merge chunk partials [nchunks][G][D + 2] into bf16 out rows of the G heads. `lds` holds
// 2 * G * nchunks + 2 * G floats. LOADER is plain or sc1.
template <int G, bool SC1>
__device__ __forceinline__ void reduce_chunks(const float* __restrict__ pb, int nchunks, int D, float* lds,
                                              bf16_t* __restrict__ out_row) {
  const int tid = threadIdx.x;
  const int stride = D + 2;
  auto ld = [](const float* p) { return SC1 ? ld_sc1(p) : *p; };
  float* scl = lds;                // [G][nchunks]: m, then exp(m - M)
  float* lv = scl + G * nchunks;   // [G][nchunks]: l
  float* Mg = lv + G * nchunks;    // [G]
  float* Lg = Mg + G;              // [G]
  for (int i = tid; i < G * nchunks; i += 256) {
    const int g = i / nchunks, cc = i % nchunks;
    const float* pc = pb + (static_cast<int64_t>(cc) * G + g) * stride;
    scl[i] = ld(pc + D);
    lv[i] = ld(pc + D + 1);
  }
  __syncthreads();
  if (tid < G) {
    float mx = kNegBig;
    for (int cc = 0; cc < nchunks; ++cc) mx = fmaxf(mx, scl[tid * nchunks + cc]);
    float ls = 0.f;
    for (int cc = 0; cc < nchunks; ++cc) ls += lv[tid * nchunks + cc] * __expf(scl[tid * nchunks + cc] - mx);
    Mg[tid] = mx;
    Lg[tid] = ls;
  }
  __syncthreads();
  for (int i = tid; i < G * nchunks; i += 256) scl[i] = __expf(scl[i] - Mg[i / nchunks]);
  __syncthreads();
  for (int idx = tid; idx < G * D; idx += 256) {
    const int g = idx / D, d = idx % D;
    float o = 0.f;
    for (int c0 = 0; c0 < nchunks; c0 += 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int cc = min(c0 + j, nchunks - 1);  // clamped: branch-free, all 16 loads in flight
        v[j] = ld(pb + (static_cast<int64_t>(cc) * G + g) * stride + d);
      }
#pragma unroll
      for (int j = 0; j < 16; ++j) o += (c0 + j < nchunks) ? v[j] * scl[g * nchunks + c0 + j] : 0.f;
    }
    out_row[g * D + d] = f32_to_bf16(o / Lg[g]);
  }
}

}  // namespace llmc
