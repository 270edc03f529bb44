// K1 embedding gather + K2 RMSNorm.
//
// Memory-bound; 16 B per lane (8 x bf16) in and out (G13). One 256-thread block per token row,
// the row held in registers between the sum-of-squares pass and the scale pass (single HBM read).
// Numerics: y = bf16( x * rsqrt(mean(x^2) + eps) * w ) computed in f32.
#include "common.h"

namespace llmc {

template <int MAXV>
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      bf16_t* __restrict__ y, int H, int x_stride, int y_stride,
                                                      float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int nv = H / 8;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + static_cast<int64_t>(row) * x_stride);
  u32x4 v[MAXV];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nv) {
      v[i] = xr[c];
      float f[8];
      unpack8(v[i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
    }
  }
  ss = block_sum<256>(ss, red);
  const float inv = rsqrtf(ss / H + eps);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4* yr = reinterpret_cast<u32x4*>(y + static_cast<int64_t>(row) * y_stride);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nv) {
      float f[8], g[8];
      unpack8(v[i], f);
      unpack8(wr[c], g);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = f[j] * inv * g[j];
      yr[c] = pack8(f);
    }
  }
}

// out[t, :] = table[ids[t], :]
__global__ __launch_bounds__(256) void embedding_kernel(const int32_t* __restrict__ ids, const bf16_t* __restrict__ table,
                                                        bf16_t* __restrict__ out, int H, int vocab) {
  const int t = blockIdx.x;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const u32x4* src = reinterpret_cast<const u32x4*>(table + static_cast<int64_t>(id) * H);
  u32x4* dst = reinterpret_cast<u32x4*>(out + static_cast<int64_t>(t) * H);
  for (int c = threadIdx.x; c < H / 8; c += 256) dst[c] = src[c];
}

// y = silu(x[:, gate]) * x[:, up] with gate/up rows INTERLEAVED in the GEMM output
// (column 2i = gate_i, 2i+1 = up_i), matching the fused gate_up weight layout.
__global__ __launch_bounds__(256) void silu_mul_interleaved_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ y,
                                                                   int I) {
  const int t = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;  // 4 outputs per thread
  if (c * 4 >= I) return;
  const u32x4 v = reinterpret_cast<const u32x4*>(gu + static_cast<int64_t>(t) * 2 * I)[c];
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = silu(bf16_lo(v[j])) * bf16_hi(v[j]);
  u32x2 r;
  r[0] = pack_bf16x2(o[0], o[1]);
  r[1] = pack_bf16x2(o[2], o[3]);
  reinterpret_cast<u32x2*>(y + static_cast<int64_t>(t) * I)[c] = r;
}

// Self-test of the cross-lane helpers (common.h): every lane writes each helper's result next to
// the __shfl_xor form it replaces; the GPU test compares the pairs bit for bit.
__global__ void lane_exchange_check_kernel(const float* __restrict__ in, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const float v = in[blockIdx.x * 64 + lane];
  float* o = out + (static_cast<int64_t>(blockIdx.x) * 64 + lane) * 20;
  float w = v;
  o[0] = xor16_add(v);
  o[1] = v + __shfl_xor(v, 16, 64);
  o[2] = xor32_add(v);
  o[3] = v + __shfl_xor(v, 32, 64);
  o[4] = xor16_max(v);
  o[5] = fmaxf(v, __shfl_xor(v, 16, 64));
  o[6] = xor32_max(v);
  o[7] = fmaxf(v, __shfl_xor(v, 32, 64));
  o[8] = wave_sum(v);
  for (int m = 32; m >= 1; m >>= 1) w += __shfl_xor(w, m, 64);
  o[9] = w;
  o[10] = wave_max(v);
  w = v;
  for (int m = 32; m >= 1; m >>= 1) w = fmaxf(w, __shfl_xor(w, m, 64));
  o[11] = w;
  o[12] = xor_shfl<4>(v, lane);
  o[13] = __shfl_xor(v, 4, 64);
  o[14] = xor_shfl<8>(v, lane) + xor_shfl<2>(v, lane) + xor_shfl<1>(v, lane);
  o[15] = __shfl_xor(v, 8, 64) + __shfl_xor(v, 2, 64) + __shfl_xor(v, 1, 64);
  o[16] = xor_shfl<16>(v, lane) + xor_shfl<32>(v, lane);
  o[17] = __shfl_xor(v, 16, 64) + __shfl_xor(v, 32, 64);
  o[18] = xor_tree_sum<8>(v, lane);
  w = v;
  for (int m = 8; m >= 1; m >>= 1) w += __shfl_xor(w, m, 64);
  o[19] = w;
}

}  // namespace llmc

using namespace llmc;

extern "C" {

// in: float [nb * 64]; out: float [nb * 64 * 20] (pairs (helper, __shfl_xor form))
int llmc_lane_exchange_check(const void* in, void* out, int nb, hipStream_t s) {
  if (nb <= 0) return -1;
  lane_exchange_check_kernel<<<nb, 64, 0, s>>>((const float*)in, (float*)out);
  return static_cast<int>(hipGetLastError());
}

int llmc_rmsnorm(const void* x, const void* w, void* y, int T, int H, int x_stride, int y_stride, float eps,
                 hipStream_t s) {
  if (H % 8 != 0 || H > 8 * 256 * 4) return -1;
  const int nv = H / 8;
  if (nv <= 256)
    rmsnorm_kernel<1><<<T, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, H, x_stride, y_stride, eps);
  else if (nv <= 512)
    rmsnorm_kernel<2><<<T, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, H, x_stride, y_stride, eps);
  else
    rmsnorm_kernel<4><<<T, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)w, (bf16_t*)y, H, x_stride, y_stride, eps);
  return static_cast<int>(hipGetLastError());
}

int llmc_embedding(const void* ids, const void* table, void* out, int T, int H, int vocab, hipStream_t s) {
  if (H % 8 != 0) return -1;
  embedding_kernel<<<T, 256, 0, s>>>((const int32_t*)ids, (const bf16_t*)table, (bf16_t*)out, H, vocab);
  return static_cast<int>(hipGetLastError());
}

int llmc_silu_mul_interleaved(const void* gu, void* y, int T, int I, hipStream_t s) {
  if (I % 4 != 0) return -1;
  dim3 grid((I / 4 + 255) / 256, T);
  silu_mul_interleaved_kernel<<<grid, 256, 0, s>>>((const bf16_t*)gu, (bf16_t*)y, I);
  return static_cast<int>(hipGetLastError());
}

}  // extern "C"
