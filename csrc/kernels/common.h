// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Conventions (cdna_hip_programming.md §1, §6 G13):
//  * wave = 64 lanes, blocks are multiples of 64 threads;
//  * bf16 tensors are moved 16 B per lane (8 x bf16) — never scalar bf16 loads;
//  * f32 accumulation everywhere; bf16 rounding by the hardware cvt (RNE, NaN-preserving).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmc {

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // storage type for bf16 tensors
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;  // MFMA A/B fragment (8 bf16)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float bf16_to_f32(bf16_t b) { return __uint_as_float(static_cast<uint32_t>(b) << 16); }

__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return static_cast<uint32_t>(f32_to_bf16(lo)) | (static_cast<uint32_t>(f32_to_bf16(hi)) << 16);
}

// 8 bf16 packed in a u32x4 -> 8 floats
__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = bf16_lo(v[i]);
    f[2 * i + 1] = bf16_hi(v[i]);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
  return v;
}

// f32 += dot(bf16x2 a, bf16x2 b) in one VALU op (v_dot2_f32_bf16).
__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b), c, false);
}
__device__ __forceinline__ float dot8_bf16(const u32x4& a, const u32x4& b, float c) {
  c = dot2_bf16(a[0], b[0], c);
  c = dot2_bf16(a[1], b[1], c);
  c = dot2_bf16(a[2], b[2], c);
  c = dot2_bf16(a[3], b[3], c);
  return c;
}

template <bool NT>
__device__ __forceinline__ u32x4 load16(const void* p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  } else {
    return *reinterpret_cast<const u32x4*>(p);
  }
}

// Load of a wave-uniform address through the scalar cache (s_load_dword, counted by lgkmcnt, so
// it does not queue behind the vector loads in flight). Read-only data only.
template <typename T>
__device__ __forceinline__ T ld_scalar(const T* p) {
  static_assert(sizeof(T) == 4, "32-bit scalar loads");
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

// Full-wave reductions (xor butterfly over 64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Reduction inside aligned groups of W lanes (W power of two <= 64).
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for NT threads (NT multiple of 64, <= 1024). `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / kWave; ++i) t += red[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

// Split-KV decode attention, balanced form: a fixed grid of `gc` blocks per (sequence, kv head)
// shares the sequence's L keys evenly in 32-key units (the MFMA sub-tile): n = min(gc,
// ceil(L / min_chunk)) blocks, block c owning units [c*U/n, (c+1)*U/n) of U = ceil(L/32), so
// the grid shape (and a captured graph) is independent of L and every live block gets the same
// work to within one sub-tile. chunk_arg < 0 encodes this form (min_chunk = -chunk_arg);
// chunk_arg >= 0 is the fixed-chunk form (blocks of chunk_arg keys; VALU kernels).
__device__ __forceinline__ int decode_nsplit(int L, int gc, int chunk_arg) {
  if (chunk_arg >= 0) return (L + chunk_arg - 1) / chunk_arg;
  const int n = (L + (-chunk_arg) - 1) / (-chunk_arg);
  return n < 1 ? 1 : (n < gc ? n : gc);
}
__device__ __forceinline__ void decode_range(int L, int n, int c, int chunk_arg, int& start, int& end) {
  if (chunk_arg >= 0) {
    start = c * chunk_arg;
    end = min(start + chunk_arg, L);
    return;
  }
  const int64_t units = (L + 31) / 32;
  start = static_cast<int>(32 * (c * units / n));
  end = min(L, static_cast<int>(32 * ((c + 1) * units / n)));
}

}  // namespace llmc

#define LLMC_CHECK_LAUNCH() (void)0
