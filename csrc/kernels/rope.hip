// K3: RoPE (rotate-half, Llama/Mixtral/Phi-3) on q and k + paged-KV write.
//
// Input: fused qkv rows [T, (nh + 2 nkv) * D] straight out of the qkv projection, with every Q and
// K head PAIR-INTERLEAVED ([x0, x_{D/2}, x1, x_{D/2+1}, ...], models/transformer.py). Rotated q
// is written in canonical order to q_out [T, nh * D]; rotated k and raw v are scattered into the
// paged caches at slot[t] (block * bs + offset; slot < 0 = do not cache). This is the PREFILL
// path; decode applies the same rotation in the qkv GEMV epilogue (gemv_core.h, EPI_ROPE). cos/sin come from a host-precomputed f32 table [max_pos][D/2]
// (cdna_hip_programming.md App. B: no on-device trig). Positions and slots are read from device
// memory, so the same launch is replayable inside a decode HIP graph.
// KV cache layout: [num_blocks][nkv][bs][D] bf16 (one page = bs contiguous D-rows per head).
#include "common.h"

namespace llmc {

__global__ __launch_bounds__(256) void rope_kv_write_kernel(const bf16_t* __restrict__ qkv, int qkv_stride,
                                                            bf16_t* __restrict__ q_out, int q_stride,
                                                            const int32_t* __restrict__ positions,
                                                            const float* __restrict__ cos_t,
                                                            const float* __restrict__ sin_t,
                                                            bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                                                            const int32_t* __restrict__ slots, int nh, int nkv, int D,
                                                            int bs) {
  const int t = blockIdx.x;
  const int half = D / 2;
  const int quads = half / 4;  // 4 rotation pairs per item
  const int pos = positions[t];
  const int slot = slots != nullptr ? slots[t] : -1;
  const bf16_t* row = qkv + static_cast<int64_t>(t) * qkv_stride;
  const float* cr = cos_t + static_cast<int64_t>(pos) * half;
  const float* sr = sin_t + static_cast<int64_t>(pos) * half;
  const int64_t page = slot >= 0 ? slot / bs : 0;
  const int off = slot >= 0 ? slot % bs : 0;

  const int rot_items = (nh + nkv) * quads;
  for (int it = threadIdx.x; it < rot_items; it += blockDim.x) {
    const int head = it / quads;
    const int i = (it % quads) * 4;
    const bf16_t* base = row + head * D;  // q heads then k heads are contiguous in qkv
    // pairs (i..i+3) live interleaved at [2i .. 2i+7]: one 16-B load
    const u32x4 pr = *reinterpret_cast<const u32x4*>(base + 2 * i);
    const f32x4 c = *reinterpret_cast<const f32x4*>(cr + i);
    const f32x4 s = *reinterpret_cast<const f32x4*>(sr + i);
    float x1[4] = {bf16_lo(pr[0]), bf16_lo(pr[1]), bf16_lo(pr[2]), bf16_lo(pr[3])};
    float x2[4] = {bf16_hi(pr[0]), bf16_hi(pr[1]), bf16_hi(pr[2]), bf16_hi(pr[3])};
    float o1[4], o2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o1[j] = x1[j] * c[j] - x2[j] * s[j];
      o2[j] = x2[j] * c[j] + x1[j] * s[j];
    }
    u32x2 ra, rb;
    ra[0] = pack_bf16x2(o1[0], o1[1]);
    ra[1] = pack_bf16x2(o1[2], o1[3]);
    rb[0] = pack_bf16x2(o2[0], o2[1]);
    rb[1] = pack_bf16x2(o2[2], o2[3]);
    if (head < nh) {
      bf16_t* qo = q_out + static_cast<int64_t>(t) * q_stride + head * D;
      *reinterpret_cast<u32x2*>(qo + i) = ra;
      *reinterpret_cast<u32x2*>(qo + i + half) = rb;
    } else if (slot >= 0) {
      const int kh = head - nh;
      bf16_t* dst = k_cache + ((page * nkv + kh) * bs + off) * D;
      *reinterpret_cast<u32x2*>(dst + i) = ra;
      *reinterpret_cast<u32x2*>(dst + i + half) = rb;
    }
  }
  if (slot >= 0) {
    const int vchunks = nkv * (D / 8);
    const bf16_t* vrow = row + (nh + nkv) * D;
    for (int it = threadIdx.x; it < vchunks; it += blockDim.x) {
      const int kh = it / (D / 8);
      const int i = (it % (D / 8)) * 8;
      bf16_t* dst = v_cache + ((page * nkv + kh) * bs + off) * D;
      *reinterpret_cast<u32x4*>(dst + i) = *reinterpret_cast<const u32x4*>(vrow + kh * D + i);
    }
  }
}

}  // namespace llmc

using namespace llmc;

extern "C" int llmc_rope_kv_write(const void* qkv, int qkv_stride, void* q_out, int q_stride, const void* positions,
                                  const void* cos_t, const void* sin_t, void* k_cache, void* v_cache, const void* slots,
                                  int T, int nh, int nkv, int D, int bs, hipStream_t s) {
  if (D % 8 != 0 || (D / 2) % 4 != 0) return -1;
  rope_kv_write_kernel<<<T, 256, 0, s>>>((const bf16_t*)qkv, qkv_stride, (bf16_t*)q_out, q_stride,
                                         (const int32_t*)positions, (const float*)cos_t,
                                         (const float*)sin_t, (bf16_t*)k_cache, (bf16_t*)v_cache,
                                         (const int32_t*)slots, nh, nkv, D, bs);
  return static_cast<int>(hipGetLastError());
}
